#include "comm/fusion_engine.h"

#include <stdexcept>

namespace rla {
namespace comm {
namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

FusionEngine::FusionEngine(Communicator* comm, int64_t fusion_bytes, int device)
    : comm_(comm), device_(device), fusion_elems_(fusion_bytes / 4 > 0 ? fusion_bytes / 4 : 1) {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  // high priority: the allreduce is on the step's critical path
  hip_check(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "hipStreamCreate");
  thread_ = std::thread([this] { loop(); });
}

FusionEngine::~FusionEngine() {
  {
    std::lock_guard<std::mutex> g(mu_);
    close_open_locked();
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  hipSetDevice(device_);
  if (stream_) hipStreamSynchronize(stream_);
  for (auto e : event_pool_) hipEventDestroy(e);
  if (buffer_) hipFree(buffer_);
  if (stream_) hipStreamDestroy(stream_);
}

hipEvent_t FusionEngine::get_event() {
  if (!event_pool_.empty()) {
    hipEvent_t e = event_pool_.back();
    event_pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  return e;
}

void FusionEngine::close_open_locked() {
  if (open_ && !open_->reqs.empty()) {
    queue_.push_back(open_);
    ++inflight_;
    cv_.notify_all();
  }
  open_.reset();
}

int64_t FusionEngine::submit(float* ptr, int64_t n, float postscale, hipStream_t ready) {
  std::unique_lock<std::mutex> g(mu_);
  if (!error_.empty()) throw std::runtime_error("fusion engine failed: " + error_);
  Req r{ptr, n, postscale, get_event(), next_handle_++};
  hip_check(hipEventRecord(r.ready, ready), "hipEventRecord(ready)");
  if (open_ && !open_->reqs.empty() &&
      (open_->elems + n > fusion_elems_ || open_->reqs.size() >= (size_t)kPackMax * 64))
    close_open_locked();
  if (!open_) open_ = std::make_shared<Batch>();
  open_->reqs.push_back(r);
  open_->elems += n;
  by_handle_[r.handle] = open_;
  fingerprint_ = (fingerprint_ ^ (uint64_t)n) * 1099511628211ull;
  if (open_->elems >= fusion_elems_) close_open_locked();
  return r.handle;
}

void FusionEngine::flush() {
  std::lock_guard<std::mutex> g(mu_);
  close_open_locked();
}

bool FusionEngine::wait(int64_t handle, hipStream_t consumer) {
  std::unique_lock<std::mutex> g(mu_);
  auto it = by_handle_.find(handle);
  if (it == by_handle_.end()) return false;
  std::shared_ptr<Batch> b = it->second;
  by_handle_.erase(it);
  if (b == open_) close_open_locked();
  // the done event must be RECORDED before a stream can wait on it
  cv_done_.wait(g, [&] { return b->done != nullptr || !error_.empty(); });
  if (!error_.empty()) throw std::runtime_error("fusion engine failed: " + error_);
  hip_check(hipStreamWaitEvent(consumer, b->done, 0), "hipStreamWaitEvent");
  return true;
}

void FusionEngine::drain() {
  std::unique_lock<std::mutex> g(mu_);
  close_open_locked();
  cv_done_.wait(g, [&] { return inflight_ == 0 || !error_.empty(); });
  g.unlock();
  hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize(comm)");
  if (!error_.empty()) throw std::runtime_error("fusion engine failed: " + error_);
}

std::string FusionEngine::last_error() {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

void FusionEngine::execute(Batch& b) {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (auto& r : b.reqs) hip_check(hipStreamWaitEvent(stream_, r.ready, 0), "hipStreamWaitEvent(ready)");
  auto reduce = [&](float* p, int64_t n) { comm_->allreduce_f32(p, n, stream_); };
  auto copy = [&](bool in, float scale_override, bool use_req_scale) {
    PackTable t{};
    int64_t off = 0;
    size_t i = 0;
    while (i < b.reqs.size()) {
      t.count = 0;
      const float s = use_req_scale ? b.reqs[i].scale : scale_override;
      while (i < b.reqs.size() && t.count < kPackMax && (!use_req_scale || b.reqs[i].scale == s)) {
        const Req& r = b.reqs[i];
        t.src[t.count] = in ? r.ptr : buffer_ + off;
        t.dst[t.count] = in ? buffer_ + off : r.ptr;
        t.n[t.count] = r.n;
        ++t.count;
        off += r.n;
        ++i;
      }
      t.scale = s;
      launch_pack(t, stream_);
    }
  };
  if (b.reqs.size() == 1) {  // no packing: reduce in place, then apply the average
    const Req& r = b.reqs[0];
    reduce(r.ptr, r.n);
    if (r.scale != 1.0f) {
      PackTable t{};
      t.src[0] = r.ptr;
      t.dst[0] = r.ptr;
      t.n[0] = r.n;
      t.count = 1;
      t.scale = r.scale;
      launch_pack(t, stream_);
    }
  } else {
    const int64_t padded = (b.elems + 3) / 4 * 4;
    if (padded > buffer_elems_) {
      if (buffer_) {
        hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        hip_check(hipFree(buffer_), "hipFree");
      }
      buffer_elems_ = padded > fusion_elems_ ? padded : (fusion_elems_ + 3) / 4 * 4;
      hip_check(hipMalloc(reinterpret_cast<void**>(&buffer_), buffer_elems_ * 4), "hipMalloc(fusion buffer)");
    }
    if (padded > b.elems)
      hip_check(hipMemsetAsync(buffer_ + b.elems, 0, (padded - b.elems) * 4, stream_), "hipMemsetAsync");
    copy(true, 1.0f, false);
    reduce(buffer_, padded);
    copy(false, 1.0f, true);
  }
}

void FusionEngine::loop() {
  hipSetDevice(device_);
  for (;;) {
    std::shared_ptr<Batch> b;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !queue_.empty(); });
      if (queue_.empty()) return;
      b = queue_.front();
      queue_.pop_front();
    }
    hipEvent_t done = nullptr;
    std::string err;
    try {
      execute(*b);
      hip_check(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate(done)");
      hip_check(hipEventRecord(done, stream_), "hipEventRecord(done)");
    } catch (const std::exception& e) {
      err = e.what();
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& r : b->reqs) event_pool_.push_back(r.ready);  // consumed by the waits above
      b->done = done;
      --inflight_;
      ++executed_;
      if (!err.empty() && error_.empty()) error_ = err;
    }
    cv_done_.notify_all();
  }
}

}  // namespace comm
}  // namespace rla
