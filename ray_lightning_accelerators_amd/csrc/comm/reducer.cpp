#include "comm/reducer.h"

#include <stdexcept>
#include <string>

namespace rla {
namespace comm {
namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

Reducer::Reducer(Communicator* comm, float* grad_arena, int64_t arena_numel,
                 const std::vector<int64_t>& bucket_bounds, const std::vector<int>& param_bucket, int device)
    : comm_(comm), grad_(grad_arena), device_(device), param_bucket_(param_bucket) {
  if (bucket_bounds.size() % 2 != 0 || bucket_bounds.empty()) throw std::runtime_error("bad bucket bounds");
  const int nb = (int)bucket_bounds.size() / 2;
  for (int b = 0; b < nb; ++b) {
    const int64_t s = bucket_bounds[2 * b], e = bucket_bounds[2 * b + 1];
    if (s < 0 || e <= s || e > arena_numel) throw std::runtime_error("bucket outside the gradient arena");
    starts_.push_back(s);
    ends_.push_back(e);
  }
  size_.assign(nb, 0);
  for (int b : param_bucket_) {
    if (b < 0 || b >= nb) throw std::runtime_error("parameter mapped to a missing bucket");
    ++size_[b];
  }
  pending_ = size_;
  launched_.assign(nb, 0);
  hip_check(hipSetDevice(device_), "hipSetDevice");
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreate(reducer)");
  ready_.resize(nb);
  done_.resize(nb);
  for (int b = 0; b < nb; ++b) {
    hip_check(hipEventCreateWithFlags(&ready_[b], hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&done_[b], hipEventDisableTiming), "hipEventCreate");
  }
}

Reducer::~Reducer() {
  hipSetDevice(device_);
  if (stream_) hipStreamSynchronize(stream_);
  for (auto e : ready_) hipEventDestroy(e);
  for (auto e : done_) hipEventDestroy(e);
  if (stream_) hipStreamDestroy(stream_);
}

void Reducer::prepare() {
  pending_ = size_;
  launched_.assign(launched_.size(), 0);
  next_ = 0;
}

void Reducer::launch(int b, hipStream_t producer) {
  hip_check(hipEventRecord(ready_[b], producer), "hipEventRecord(ready)");
  hip_check(hipStreamWaitEvent(stream_, ready_[b], 0), "hipStreamWaitEvent(ready)");
  float* p = grad_ + starts_[b];
  const int64_t n = ends_[b] - starts_[b];
  comm_->allreduce_f32(p, n, stream_);  // xGMI one-shot / two-shot / RCCL by size
  hip_check(hipEventRecord(done_[b], stream_), "hipEventRecord(done)");
  launched_[b] = 1;
  ++launched_total_;
}

void Reducer::launch_ready(hipStream_t producer) {
  while (next_ < (int)starts_.size() && pending_[next_] <= 0) launch(next_++, producer);
}

void Reducer::mark_ready(int param, hipStream_t producer) {
  if (param < 0 || param >= (int)param_bucket_.size()) throw std::runtime_error("bad parameter index");
  const int b = param_bucket_[param];
  if (--pending_[b] == 0) launch_ready(producer);
}

void Reducer::finish(hipStream_t consumer) {
  for (auto& p : pending_) p = 0;  // buckets of unused parameters go out now, in order
  launch_ready(consumer);
  for (size_t b = 0; b < done_.size(); ++b)
    hip_check(hipStreamWaitEvent(consumer, done_[b], 0), "hipStreamWaitEvent(done)");
  next_ = 0;
}

}  // namespace comm
}  // namespace rla
