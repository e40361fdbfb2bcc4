// Native communicator of one rank: an RCCL communicator (bootstrapped from a
// unique id the Python side exchanges over the rendezvous store) plus the xGMI
// peer map used by the one-shot allreduce, and a watchdog thread.
//
// MI355X-first split of the data plane:
//   * small buckets (<= xgmi capacity, e.g. the 110-530 KiB MNIST gradient):
//     one-shot push allreduce through IPC-mapped peer memory -- latency is two
//     xGMI crossings instead of RCCL's protocol rounds;
//   * everything else: RCCL (ring/tree over the same links).
// Every collective is enqueued on the caller's stream, so it can be captured
// into a hipGraph together with the step's compute kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "comm/xgmi.h"

namespace rla {
namespace comm {

enum class RedOp : int { kSum = 0, kMax = 1, kMin = 2, kProd = 3 };
enum class DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kI32 = 3, kI64 = 4, kU8 = 5, kF64 = 6 };

class Communicator {
 public:
  Communicator(int rank, int world, int device);
  ~Communicator();
  Communicator(const Communicator&) = delete;
  Communicator& operator=(const Communicator&) = delete;

  static std::string unique_id();  // rank 0 creates, everyone passes it to init_rccl

  int rank() const { return rank_; }
  int world() const { return world_; }

  // ---- RCCL ----
  void init_rccl(const std::string& uid);
  bool has_rccl() const { return comm_ != nullptr; }
  // ranks the RCCL communicator itself reports (ncclCommCount; -1 without one)
  int rccl_count() const;
  void allreduce(void* buf, int64_t count, DType dt, RedOp op, hipStream_t s);
  void broadcast(void* buf, int64_t count, DType dt, int root, hipStream_t s);
  void allgather(const void* in, void* out, int64_t count, DType dt, hipStream_t s);
  void reduce_scatter(const void* in, void* out, int64_t count, DType dt, RedOp op, hipStream_t s);

  // ---- xGMI one-shot ----
  // Allocates this rank's uncached region (capacity floats per peer slot) and
  // returns its IPC handle bytes; open_peers maps every other rank's region.
  std::string xgmi_handle(int64_t capacity_floats);
  void xgmi_open(const std::vector<std::string>& handles);
  bool has_xgmi() const { return xgmi_ready_; }
  int64_t xgmi_capacity() const { return slot_stride_; }
  void allreduce_xgmi(float* buf, int64_t count, hipStream_t s);
  void set_spin_limit(int64_t n) { spin_limit_ = n; }

  // ---- xGMI two-shot (reduce-scatter + all-gather, medium/large buckets) ----
  // Own region sized for buckets of up to capacity_floats; same handle exchange.
  std::string twoshot_handle(int64_t capacity_floats);
  void twoshot_open(const std::vector<std::string>& handles);
  bool has_twoshot() const { return ts_ready_; }
  // largest bucket (floats) the two-shot region holds
  int64_t twoshot_capacity() const { return ts_ready_ ? ts_stride_ * world_ : 0; }
  void allreduce_twoshot(float* buf, int64_t count, bool bf16_wire, hipStream_t s);
  // any length: consecutive launches of at most twoshot_launch_floats() each
  void allreduce_twoshot_chunked(float* buf, int64_t count, bool bf16_wire, hipStream_t s);
  int64_t twoshot_launch_floats() const;

  // ---- routing of fp32 SUM allreduces (DDP reducer, fusion engine, Python) ----
  // one-shot up to min(one-shot capacity, oneshot_max), then two-shot up to
  // min(two-shot capacity, twoshot_max), then RCCL.  Every rank must set the same
  // limits (the Python layer agrees on them over the bootstrap group).
  void set_route_limits(int64_t oneshot_max_floats, int64_t twoshot_max_floats) {
    oneshot_max_ = oneshot_max_floats;
    twoshot_max_ = twoshot_max_floats;
  }
  // 0 = one-shot, 1 = two-shot, 2 = RCCL, 3 = two-shot in region-sized launches
  // (no RCCL, or two-shot forced), -1 = no path
  int route(const float* buf, int64_t count) const;
  void allreduce_f32(float* buf, int64_t count, hipStream_t s);
  // bf16 wire: two-shot (region-sized launches); false without a two-shot region
  bool allreduce_f32_bf16wire(float* buf, int64_t count, hipStream_t s);

  // ---- auxiliary peer region for kernels that exchange data themselves ----
  // (the fused data-parallel MLP tail pushes its gradient tiles straight into the
  // peers' receive areas; a separate region so it never aliases the one-shot
  // allreduce's areas or generations)
  std::string aux_handle(int64_t capacity_floats);
  void aux_open(const std::vector<std::string>& handles);
  // reset the region for a new exchange protocol / job (see communicator.cpp)
  void aux_rearm();
  bool has_aux() const { return aux_ready_; }
  // [world, rank, slot_stride, spin_limit, gen_ptr, err_ptr, region_ptr x world]
  std::vector<int64_t> aux_context() const;

  // ---- health ----
  // 0 healthy; 1 xGMI poll timed out; 2 RCCL async error; 3 aborted
  int error_state();
  std::string error_message();
  void start_watchdog(int period_ms);
  void abort();
  // After a failed xGMI validation: clear a latched poll timeout (state 1 only --
  // RCCL errors and aborts stay latched) so the fallback path can be used.
  // Collective: every rank calls it after a device sync + barrier.
  void reset_error();
  // Take a path that failed validation out of the C++ router (0 one-shot,
  // 1 two-shot, 2 aux exchange); its generations are desynchronised for good.
  void disable_path(int which);

 private:
  void check_rccl(ncclResult_t r, const char* what);
  void watchdog_loop(int period_ms);

  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;
  // xGMI
  char* region_ = nullptr;                 // own region (uncached device memory, pooled: uc_alloc)
  size_t region_bytes_ = 0;
  char* peers_[kXgmiMaxRanks] = {};        // mapped regions (own included)
  bool xgmi_ready_ = false;
  int64_t slot_stride_ = 0;
  uint32_t* gen_ = nullptr;                // device: per-block generations
  int* err_host_ = nullptr;                // host-mapped error word
  int* err_dev_ = nullptr;
  int64_t spin_limit_ = int64_t(1) << 24;  // ~2-4 s of s_sleep polling
  // two-shot region
  char* ts_region_ = nullptr;
  size_t ts_region_bytes_ = 0;
  char* ts_peers_[kXgmiMaxRanks] = {};
  uint32_t* ts_gen_ = nullptr;             // device: per-block generations
  int64_t ts_stride_ = 0;                  // chunk stride (fp32 elements)
  bool ts_ready_ = false;
  int64_t oneshot_max_ = INT64_MAX;
  int64_t twoshot_max_ = INT64_MAX;
  // auxiliary region
  char* aux_region_ = nullptr;
  size_t aux_region_bytes_ = 0;
  char* aux_peers_[kXgmiMaxRanks] = {};
  uint32_t* aux_gen_ = nullptr;
  int64_t aux_stride_ = 0;
  bool aux_ready_ = false;
  // health
  std::atomic<int> state_{0};
  std::string message_;
  std::mutex mu_;
  std::thread watchdog_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> aborted_{false};
};

}  // namespace comm
}  // namespace rla
