// Horovod-style tensor-fusion engine (replaces horovod.torch's C++ core for the
// single-node MI355X case).
//
// Ranks submit gradient allreduce requests as autograd produces them.  Requests
// are grouped into fusion batches of up to `fusion_bytes` ON THE SUBMITTING
// THREAD, purely by submission sequence -- no timers -- so every rank forms the
// same batches without a negotiation round (Horovod's coordinator exists to
// agree on an order; here the order is the deterministic autograd hook order,
// and `fingerprint()` lets the Python layer verify it across ranks).
// A background thread executes the batches on a dedicated comm stream:
//   wait on each request's ready event -> pack (multi-tensor copy kernel) ->
//   allreduce (xGMI one-shot when it fits, else RCCL) -> unpack with the
//   1/size average folded in -> record the batch's done event.
// `wait(handle, stream)` makes a consumer stream wait on that event.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "comm/communicator.h"
#include "comm/pack.h"

namespace rla {
namespace comm {

class FusionEngine {
 public:
  FusionEngine(Communicator* comm, int64_t fusion_bytes, int device);
  ~FusionEngine();

  // Returns a handle; `ready` stream is where the tensor is produced.
  int64_t submit(float* ptr, int64_t n, float postscale, hipStream_t ready);
  // Close the open batch (called at optimizer.step / synchronize()).
  void flush();
  // Consumer stream waits for the request's batch; returns false if unknown.
  bool wait(int64_t handle, hipStream_t consumer);
  // Host-blocking wait for everything submitted so far.
  void drain();
  uint64_t fingerprint() const { return fingerprint_; }
  int64_t batches_executed() const { return executed_; }
  std::string last_error();

 private:
  struct Req {
    float* ptr;
    int64_t n;
    float scale;
    hipEvent_t ready;
    int64_t handle;
  };
  struct Batch {
    std::vector<Req> reqs;
    int64_t elems = 0;
    hipEvent_t done = nullptr;
    ~Batch() {
      if (done) hipEventDestroy(done);
    }
  };
  void loop();
  void execute(Batch& b);
  hipEvent_t get_event();
  void close_open_locked();

  Communicator* comm_;
  int device_;
  int64_t fusion_elems_;
  hipStream_t stream_ = nullptr;
  float* buffer_ = nullptr;
  int64_t buffer_elems_ = 0;
  std::mutex mu_;
  std::condition_variable cv_, cv_done_;
  std::deque<std::shared_ptr<Batch>> queue_;
  std::shared_ptr<Batch> open_;
  std::unordered_map<int64_t, std::shared_ptr<Batch>> by_handle_;
  std::vector<hipEvent_t> event_pool_;
  int64_t next_handle_ = 1;
  int64_t inflight_ = 0;
  int64_t executed_ = 0;
  uint64_t fingerprint_ = 1469598103934665603ull;
  std::string error_;
  bool stop_ = false;
  std::thread thread_;
};

}  // namespace comm
}  // namespace rla
