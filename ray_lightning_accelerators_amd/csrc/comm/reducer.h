// Native DDP reducer (replaces torch DDP's C++ Reducer).
//
// Buckets are contiguous slices of the flat fp32 gradient arena (no flatten /
// unflatten copies).  Autograd's post-accumulate-grad hooks call mark_ready(i);
// when a bucket's last parameter arrives, every complete bucket at the head of
// the order is launched -- strictly in bucket order, because every rank must
// issue its collectives in the same sequence -- on the reducer's high-priority
// comm stream, after an event recorded on the producer (compute) stream.  The
// collective is the xGMI one-shot allreduce when the bucket fits the peer
// receive areas and is 16-byte aligned, RCCL otherwise.  finish() launches any
// bucket that unused parameters left incomplete and makes the consumer stream
// wait for every bucket's done event: backward and communication overlap, and
// the optimizer (which folds in the 1/world average) runs after the last bucket.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "comm/communicator.h"

namespace rla {
namespace comm {

class Reducer {
 public:
  Reducer(Communicator* comm, float* grad_arena, int64_t arena_numel,
          const std::vector<int64_t>& bucket_bounds,   // [b0_start, b0_end, b1_start, ...]
          const std::vector<int>& param_bucket, int device);
  ~Reducer();
  void prepare();                                   // before a synchronising backward
  void mark_ready(int param, hipStream_t producer);  // from the grad hook
  void finish(hipStream_t consumer);                // before the optimizer step
  int64_t launched() const { return launched_total_; }
  int num_buckets() const { return (int)starts_.size(); }

 private:
  void launch_ready(hipStream_t producer);
  void launch(int b, hipStream_t producer);

  Communicator* comm_;
  float* grad_;
  int device_;
  std::vector<int64_t> starts_, ends_;
  std::vector<int> param_bucket_, size_, pending_;
  std::vector<hipEvent_t> ready_, done_;
  std::vector<char> launched_;
  int next_ = 0;
  int64_t launched_total_ = 0;
  hipStream_t stream_ = nullptr;
};

}  // namespace comm
}  // namespace rla
