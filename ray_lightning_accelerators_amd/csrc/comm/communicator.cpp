#include "comm/communicator.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <utility>
#include <vector>

namespace rla {
namespace comm {
namespace {

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Uncached regions are never returned to the driver.  On this stack, once a
// hipDeviceMallocUncached allocation has been freed, later ordinary allocations can
// hold kernel writes that the copy engine never sees: scripts/probes/
// uncached_reuse_probe.hip found stale device-to-host copies in 11,256 of 32,043
// checks after such frees and in 0 of 32,820 with plain allocations instead
// (profiles/r6_investigation/).  That was the round-5/6 "intermittent corrupted fresh
// tensor" of the GPU suite: the MNIST data-parallel tests create and free these
// regions, and the fidelity tests that follow them compare device and host copies.
// A process-wide free list per (device, size) hands a destroyed communicator's
// regions to the next one; the driver reclaims them at process exit.
std::mutex g_uc_mu;
std::map<std::pair<int, size_t>, std::vector<void*>> g_uc_free;

void* uc_alloc(int device, size_t bytes, const char* what) {
  {
    std::lock_guard<std::mutex> g(g_uc_mu);
    auto it = g_uc_free.find({device, bytes});
    if (it != g_uc_free.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      return p;
    }
  }
  void* p = nullptr;
  hip_check(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached), what);
  return p;
}

void uc_release(int device, size_t bytes, void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> g(g_uc_mu);
  g_uc_free[{device, bytes}].push_back(p);
}

ncclDataType_t to_nccl(DType d) {
  switch (d) {
    case DType::kF32: return ncclFloat32;
    case DType::kBF16: return ncclBfloat16;
    case DType::kF16: return ncclFloat16;
    case DType::kI32: return ncclInt32;
    case DType::kI64: return ncclInt64;
    case DType::kU8: return ncclUint8;
    case DType::kF64: return ncclFloat64;
  }
  throw std::runtime_error("unsupported dtype");
}

ncclRedOp_t to_nccl(RedOp o) {
  switch (o) {
    case RedOp::kSum: return ncclSum;
    case RedOp::kMax: return ncclMax;
    case RedOp::kMin: return ncclMin;
    case RedOp::kProd: return ncclProd;
  }
  throw std::runtime_error("unsupported reduction");
}

}  // namespace

int Communicator::rccl_count() const {
  if (!comm_ || aborted_.load()) return -1;
  int n = -1;
  if (ncclCommCount(comm_, &n) != ncclSuccess) return -1;
  return n;
}

Communicator::Communicator(int rank, int world, int device) : rank_(rank), world_(world), device_(device) {
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("bad rank / world size");
}

Communicator::~Communicator() {
  stop_ = true;
  if (watchdog_.joinable()) watchdog_.join();
  hipSetDevice(device_);
  if (comm_ && !aborted_.exchange(true)) {
    if (state_.load() != 0) ncclCommAbort(comm_);
    else ncclCommDestroy(comm_);
  }
  comm_ = nullptr;
  for (int r = 0; r < world_ && r < kXgmiMaxRanks; ++r) {
    if (peers_[r] && peers_[r] != region_) hipIpcCloseMemHandle(peers_[r]);
    if (aux_peers_[r] && aux_peers_[r] != aux_region_) hipIpcCloseMemHandle(aux_peers_[r]);
    if (ts_peers_[r] && ts_peers_[r] != ts_region_) hipIpcCloseMemHandle(ts_peers_[r]);
  }
  // every kernel that used the regions has finished before they go to the next owner
  if (ts_region_ || region_ || aux_region_) hipDeviceSynchronize();
  uc_release(device_, ts_region_bytes_, ts_region_);
  if (ts_gen_) hipFree(ts_gen_);
  uc_release(device_, region_bytes_, region_);
  uc_release(device_, aux_region_bytes_, aux_region_);
  if (aux_gen_) hipFree(aux_gen_);
  if (gen_) hipFree(gen_);
  if (err_host_) hipHostFree(err_host_);
}

std::string Communicator::unique_id() {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

void Communicator::check_rccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    state_ = 2;
    std::lock_guard<std::mutex> g(mu_);
    message_ = std::string(what) + ": " + ncclGetErrorString(r);
    throw std::runtime_error(message_);
  }
}

void Communicator::init_rccl(const std::string& uid) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad RCCL unique id");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  // a failed bring-up is not a collective failure: the caller falls back (e.g. two
  // ranks sharing one device, which RCCL refuses) and the health state stays clean
  const ncclResult_t r = ncclCommInitRank(&comm_, world_, id, rank_);
  if (r != ncclSuccess) {
    comm_ = nullptr;
    throw std::runtime_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
}

void Communicator::allreduce(void* buf, int64_t count, DType dt, RedOp op, hipStream_t s) {
  if (!comm_ || aborted_.load()) throw std::runtime_error("RCCL communicator not initialised or aborted");
  check_rccl(ncclAllReduce(buf, buf, (size_t)count, to_nccl(dt), to_nccl(op), comm_, s), "ncclAllReduce");
}

void Communicator::broadcast(void* buf, int64_t count, DType dt, int root, hipStream_t s) {
  if (!comm_ || aborted_.load()) throw std::runtime_error("RCCL communicator not initialised or aborted");
  check_rccl(ncclBroadcast(buf, buf, (size_t)count, to_nccl(dt), root, comm_, s), "ncclBroadcast");
}

void Communicator::allgather(const void* in, void* out, int64_t count, DType dt, hipStream_t s) {
  if (!comm_ || aborted_.load()) throw std::runtime_error("RCCL communicator not initialised or aborted");
  check_rccl(ncclAllGather(in, out, (size_t)count, to_nccl(dt), comm_, s), "ncclAllGather");
}

void Communicator::reduce_scatter(const void* in, void* out, int64_t count, DType dt, RedOp op, hipStream_t s) {
  if (!comm_ || aborted_.load()) throw std::runtime_error("RCCL communicator not initialised or aborted");
  check_rccl(ncclReduceScatter(in, out, (size_t)count, to_nccl(dt), to_nccl(op), comm_, s), "ncclReduceScatter");
}

std::string Communicator::xgmi_handle(int64_t capacity_floats) {
  if (world_ > kXgmiMaxRanks) throw std::runtime_error("xGMI one-shot supports at most 8 ranks");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (!region_) {
    slot_stride_ = (capacity_floats + 63) / 64 * 64;
    const int64_t bytes = xgmi_region_bytes(slot_stride_);
    region_ = static_cast<char*>(uc_alloc(device_, (size_t)bytes, "hipExtMallocWithFlags(uncached)"));
    region_bytes_ = (size_t)bytes;
    hip_check(hipMemset(region_, 0, (size_t)bytes), "hipMemset(region)");
    hip_check(hipMalloc(reinterpret_cast<void**>(&gen_), kXgmiMaxBlocks * sizeof(uint32_t)), "hipMalloc(gen)");
    hip_check(hipMemset(gen_, 0, kXgmiMaxBlocks * sizeof(uint32_t)), "hipMemset(gen)");
    if (!err_host_) {
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(int), hipHostMallocMapped),
                "hipHostMalloc(error)");
      *err_host_ = 0;
      hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0),
                "hipHostGetDevicePointer");
    }
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, region_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void Communicator::xgmi_open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("need one IPC handle per rank");
  if (!region_) throw std::runtime_error("xgmi_handle() first");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) {
      peers_[r] = region_;
      continue;
    }
    if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    peers_[r] = static_cast<char*>(p);
  }
  xgmi_ready_ = true;
}

void Communicator::allreduce_xgmi(float* buf, int64_t count, hipStream_t s) {
  if (!xgmi_ready_) throw std::runtime_error("xGMI peers not open");
  if (count > slot_stride_ || (reinterpret_cast<uintptr_t>(buf) & 15))
    throw std::runtime_error("xGMI one-shot: count exceeds capacity or buffer not 16-byte aligned");
  XgmiLaunch l{};
  l.x = buf;
  l.n = count;
  for (int r = 0; r < world_; ++r) l.regions[r] = peers_[r];
  l.rank = rank_;
  l.world = world_;
  l.gen = gen_;
  l.error = err_dev_;
  l.slot_stride = slot_stride_;
  l.spin_limit = spin_limit_;
  if (launch_xgmi_oneshot(l, s) != 0) throw std::runtime_error("xGMI one-shot launch failed");
}

std::string Communicator::twoshot_handle(int64_t capacity_floats) {
  if (world_ > kXgmiMaxRanks) throw std::runtime_error("xGMI two-shot supports at most 8 ranks");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (!err_host_) {
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(int), hipHostMallocMapped),
              "hipHostMalloc(error)");
    *err_host_ = 0;
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0), "hipHostGetDevicePointer");
  }
  if (!ts_region_) {
    // chunk stride: a bucket of capacity_floats split W ways, rounded to 64 floats
    ts_stride_ = ((capacity_floats + world_ - 1) / world_ + 4 + 63) / 64 * 64;
    const int64_t bytes = twoshot_region_bytes(ts_stride_, world_);
    ts_region_ = static_cast<char*>(uc_alloc(device_, (size_t)bytes, "hipExtMallocWithFlags(uncached two-shot)"));
    ts_region_bytes_ = (size_t)bytes;
    hip_check(hipMemset(ts_region_, 0, (size_t)bytes), "hipMemset(two-shot)");
    hip_check(hipMalloc(reinterpret_cast<void**>(&ts_gen_), kTwoShotMaxBlocks * sizeof(uint32_t)),
              "hipMalloc(two-shot gen)");
    hip_check(hipMemset(ts_gen_, 0, kTwoShotMaxBlocks * sizeof(uint32_t)), "hipMemset(two-shot gen)");
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, ts_region_), "hipIpcGetMemHandle(two-shot)");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void Communicator::twoshot_open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("need one IPC handle per rank");
  if (!ts_region_) throw std::runtime_error("twoshot_handle() first");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) {
      ts_peers_[r] = ts_region_;
      continue;
    }
    if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(two-shot)");
    ts_peers_[r] = static_cast<char*>(p);
  }
  ts_ready_ = true;
}

void Communicator::allreduce_twoshot(float* buf, int64_t count, bool bf16_wire, hipStream_t s) {
  if (!ts_ready_) throw std::runtime_error("xGMI two-shot peers not open");
  XgmiLaunch l{};
  l.x = buf;
  l.n = count;
  for (int r = 0; r < world_; ++r) l.regions[r] = ts_peers_[r];
  l.rank = rank_;
  l.world = world_;
  l.gen = ts_gen_;
  l.error = err_dev_;
  l.slot_stride = ts_stride_;
  l.spin_limit = spin_limit_;
  if (launch_xgmi_twoshot(l, bf16_wire, s) != 0)
    throw std::runtime_error("xGMI two-shot: bucket exceeds capacity, buffer not 16-byte aligned, or launch failed");
}

int Communicator::route(const float* buf, int64_t count) const {
  const bool aligned = (reinterpret_cast<uintptr_t>(buf) & 15) == 0;
  if (world_ == 1) return 2;
  if (xgmi_ready_ && aligned && count <= slot_stride_ && count <= oneshot_max_) return 0;
  if (ts_ready_ && aligned && count <= twoshot_max_ && twoshot_plan(count, world_).cs <= ts_stride_) return 1;
  // larger than the two-shot region: RCCL, unless there is none or two-shot is
  // forced (allreduce_algo="twoshot" zeroes the one-shot limit) -- then the
  // bucket goes through the region in consecutive region-sized launches
  if (ts_ready_ && aligned && count <= twoshot_max_ && (!comm_ || oneshot_max_ == 0)) return 3;
  return comm_ ? 2 : -1;
}

int64_t Communicator::twoshot_launch_floats() const {
  // n <= W * stride  <=>  ceil(ceil(n / W) / 4) * 4 <= stride (stride is a multiple of 64)
  return ts_stride_ * world_;
}

void Communicator::allreduce_twoshot_chunked(float* buf, int64_t count, bool bf16_wire, hipStream_t s) {
  const int64_t m = twoshot_launch_floats();  // multiple of 4: every piece stays 16-byte aligned
  for (int64_t off = 0; off < count; off += m) allreduce_twoshot(buf + off, std::min(m, count - off), bf16_wire, s);
}

void Communicator::allreduce_f32(float* buf, int64_t count, hipStream_t s) {
  switch (route(buf, count)) {
    case 0: allreduce_xgmi(buf, count, s); return;
    case 1: allreduce_twoshot(buf, count, false, s); return;
    case 2: allreduce(buf, count, DType::kF32, RedOp::kSum, s); return;
    case 3: allreduce_twoshot_chunked(buf, count, false, s); return;
    default: throw std::runtime_error("no allreduce path for this bucket (xGMI capacity exceeded and no RCCL)");
  }
}

bool Communicator::allreduce_f32_bf16wire(float* buf, int64_t count, hipStream_t s) {
  if (!ts_ready_ || (reinterpret_cast<uintptr_t>(buf) & 15)) return false;
  allreduce_twoshot_chunked(buf, count, true, s);  // one launch when it fits the region
  return true;
}

std::string Communicator::aux_handle(int64_t capacity_floats) {
  if (world_ > kXgmiMaxRanks) throw std::runtime_error("xGMI exchange supports at most 8 ranks");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (!err_host_) {
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(int), hipHostMallocMapped),
              "hipHostMalloc(error)");
    *err_host_ = 0;
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev_), err_host_, 0), "hipHostGetDevicePointer");
  }
  if (!aux_region_) {
    aux_stride_ = (capacity_floats + 63) / 64 * 64;
    const int64_t bytes = xgmi_region_bytes(aux_stride_);
    aux_region_ = static_cast<char*>(uc_alloc(device_, (size_t)bytes, "hipExtMallocWithFlags(uncached aux)"));
    aux_region_bytes_ = (size_t)bytes;
    hip_check(hipMalloc(reinterpret_cast<void**>(&aux_gen_), kDpMaxBlocks * sizeof(uint32_t)), "hipMalloc(aux gen)");
    aux_rearm();
  }
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, aux_region_), "hipIpcGetMemHandle(aux)");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void Communicator::aux_rearm() {
  // Flags 0, every receive-area byte 0xFF (a packed granule's tag 3, a {gen, fp32}
  // granule's generation 0xFFFFFFFF: neither matches the first steps' tags), block
  // generations 0.  Collective in effect: the caller guarantees no peer kernel is
  // writing into this region (parallel/comm.py dp_rearm: device sync + barriers).
  if (!aux_region_) throw std::runtime_error("aux_handle() first");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  const int64_t bytes = xgmi_region_bytes(aux_stride_);
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hip_check(hipMemset(aux_region_, 0, (size_t)kXgmiFlagBytes), "hipMemset(aux flags)");
  hip_check(hipMemset(aux_region_ + kXgmiFlagBytes, 0xFF, (size_t)(bytes - kXgmiFlagBytes)), "hipMemset(aux data)");
  hip_check(hipMemset(aux_gen_, 0, kDpMaxBlocks * sizeof(uint32_t)), "hipMemset(aux gen)");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

void Communicator::aux_open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::runtime_error("need one IPC handle per rank");
  if (!aux_region_) throw std::runtime_error("aux_handle() first");
  hip_check(hipSetDevice(device_), "hipSetDevice");
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) {
      aux_peers_[r] = aux_region_;
      continue;
    }
    if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("bad IPC handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[r].data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(aux)");
    aux_peers_[r] = static_cast<char*>(p);
  }
  aux_ready_ = true;
}

std::vector<int64_t> Communicator::aux_context() const {
  if (!aux_ready_) throw std::runtime_error("aux region not open");
  std::vector<int64_t> v = {world_, rank_, aux_stride_, spin_limit_, reinterpret_cast<int64_t>(aux_gen_),
                            reinterpret_cast<int64_t>(err_dev_)};
  for (int r = 0; r < world_; ++r) v.push_back(reinterpret_cast<int64_t>(aux_peers_[r]));
  return v;
}

int Communicator::error_state() {
  if (state_.load() == 0 && err_host_ && __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) != 0) {
    state_ = 1;
    std::lock_guard<std::mutex> g(mu_);
    message_ = "xGMI allreduce: peer flag poll timed out (a rank is dead or desynchronised)";
  }
  if (state_.load() == 0 && comm_) {
    ncclResult_t async = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &async) == ncclSuccess && async != ncclSuccess && async != ncclInProgress) {
      state_ = 2;
      std::lock_guard<std::mutex> g(mu_);
      message_ = std::string("RCCL async error: ") + ncclGetErrorString(async);
    }
  }
  return state_.load();
}

std::string Communicator::error_message() {
  std::lock_guard<std::mutex> g(mu_);
  return message_;
}

void Communicator::watchdog_loop(int period_ms) {
  while (!stop_.load()) {
    if (error_state() != 0) {
      // a dead peer must not hang the job: abort RCCL so pending collectives return
      if (comm_ && state_.load() == 2 && !aborted_.exchange(true)) ncclCommAbort(comm_);
      return;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(period_ms));
  }
}

void Communicator::start_watchdog(int period_ms) {
  if (watchdog_.joinable()) return;
  stop_ = false;
  watchdog_ = std::thread([this, period_ms] { watchdog_loop(period_ms); });
}

void Communicator::reset_error() {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (state_.load() > 1) throw std::runtime_error("reset_error: RCCL failure or abort is not recoverable");
  if (err_host_) __atomic_store_n(err_host_, 0, __ATOMIC_RELEASE);
  state_ = 0;
  std::lock_guard<std::mutex> g(mu_);
  message_.clear();
}

void Communicator::disable_path(int which) {
  switch (which) {
    case 0: xgmi_ready_ = false; return;
    case 1: ts_ready_ = false; return;
    case 2: aux_ready_ = false; return;
    default: throw std::invalid_argument("disable_path: 0 one-shot, 1 two-shot, 2 aux");
  }
}

void Communicator::abort() {
  stop_ = true;
  if (watchdog_.joinable() && watchdog_.get_id() != std::this_thread::get_id()) watchdog_.join();
  if (comm_ && !aborted_.exchange(true)) ncclCommAbort(comm_);
  state_ = 3;
}

}  // namespace comm
}  // namespace rla
