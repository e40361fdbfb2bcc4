// One-shot allreduce over xGMI peer memory (single node, <= 8 GPUs).
//
// The MNIST gradient is one ~110-530 KiB bucket per step: far too small for a
// ring (RCCL spends its time in protocol latency, not on the links).  MI355X
// GPUs of a node are a full xGMI mesh (7 links per GPU), so the one-shot form
// is link-parallel by construction: every rank PUSHES its slice of the bucket
// straight into every peer's receive area (7 concurrent link writes), raises a
// per-(block, rank) generation flag, waits for the 7 matching flags in its own
// memory, and sums the W contributions in fixed rank order -- every rank gets
// the bitwise-identical result, with two link crossings of latency in total.
//
// Memory protocol (cross-device, so system scope throughout):
//   * receive areas and flags live in uncached device memory
//     (hipDeviceMallocUncached) mapped into every peer with hipIpcOpenMemHandle,
//     so remote writes are never hidden behind a stale L2 line;
//   * writer: data stores -> __threadfence_system() by every thread ->
//     barrier -> one system-scope flag store per destination rank;
//   * reader: system-scope flag poll (bounded, s_sleep between polls) ->
//     __threadfence_system() -> barrier -> data loads;
//   * generation numbers live in device memory (per block), so the kernel is
//     hipGraph-replayable; receive areas are double-buffered by generation
//     parity (a rank cannot start generation g+2 before every peer finished g);
//   * a poll that exceeds its bound sets a host-visible error word and the
//     block exits (no GPU hang); the host side surfaces it as an error.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comm/xgmi.h"

namespace rla {
namespace comm {
namespace {

constexpr int kThreads = 512;
typedef float v4f __attribute__((ext_vector_type(4)));

struct Args {
  float* x;                       // local bucket, reduced in place
  int64_t n;                      // floats
  char* regions[kXgmiMaxRanks];   // every rank's region, mapped here (own included)
  int rank, world;
  uint32_t* gen;                  // [kXgmiMaxBlocks] per-block generation (local device memory)
  int* error;                     // host-mapped error word
  int64_t slot_stride;            // floats per (slot, rank) receive area
  int64_t spin_limit;
};

__device__ __forceinline__ uint32_t* flag_ptr(char* region, int slot, int blk, int src) {
  return reinterpret_cast<uint32_t*>(region) + ((size_t)slot * kXgmiMaxBlocks + blk) * kXgmiMaxRanks + src;
}

__device__ __forceinline__ float* data_ptr(char* region, int slot, int src, int64_t slot_stride) {
  return reinterpret_cast<float*>(region + kXgmiFlagBytes) + ((int64_t)slot * kXgmiMaxRanks + src) * slot_stride;
}

__global__ __launch_bounds__(kThreads) void oneshot_allreduce_kernel(Args a) {
  __shared__ uint32_t sh_gen;
  __shared__ int sh_fail;
  const int blk = blockIdx.x, nblk = gridDim.x, tid = threadIdx.x;
  if (tid == 0) {
    sh_gen = a.gen[blk] + 1u;
    sh_fail = 0;
  }
  __syncthreads();
  const uint32_t gen = sh_gen;
  const int slot = gen & 1u;

  // this block's slice in float4 units; the last block also owns the n % 4 tail
  const int64_t n4 = a.n / 4;
  const int64_t per = (n4 + nblk - 1) / nblk;
  const int64_t lo = blk * per, hi = lo + per < n4 ? lo + per : n4;
  const bool tail_owner = blk == nblk - 1;
  const int64_t t0 = n4 * 4;
  const v4f* src = reinterpret_cast<const v4f*>(a.x);

  // 1. push my slice into every rank's receive area [slot][my rank]
  for (int64_t i = lo + tid; i < hi; i += kThreads) {
    const v4f v = src[i];
    for (int r = 0; r < a.world; ++r) {
      v4f* dst = reinterpret_cast<v4f*>(data_ptr(a.regions[r], slot, a.rank, a.slot_stride));
      __builtin_nontemporal_store(v, dst + i);
    }
  }
  if (tail_owner && t0 + tid < a.n) {
    const float v = a.x[t0 + tid];
    for (int r = 0; r < a.world; ++r)
      __builtin_nontemporal_store(v, data_ptr(a.regions[r], slot, a.rank, a.slot_stride) + t0 + tid);
  }
  __threadfence_system();
  __syncthreads();
  // 2. raise my flag in every rank's region
  if (tid < a.world)
    __hip_atomic_store(flag_ptr(a.regions[tid], slot, blk, a.rank), gen, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every rank's flag in my region (bounded)
  if (tid < a.world) {
    uint32_t* f = flag_ptr(a.regions[a.rank], slot, blk, tid);
    int64_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != gen) {
      if (++spins > a.spin_limit) {
        sh_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __threadfence_system();
  __syncthreads();
  // every generation entry advances on every launch (also the block indices a
  // smaller grid does not have), so all blocks of a launch agree on the slot
  // parity when consecutive buckets differ in size (see xgmi_twoshot.hip)
  if (blk == 0)
    for (int k = nblk + tid; k < kXgmiMaxBlocks; k += kThreads) a.gen[k] = gen;
  if (sh_fail) {
    if (tid == 0) {
      __hip_atomic_store(a.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      a.gen[blk] = gen;  // stay in step with the peers' numbering
    }
    return;
  }
  // 4. reduce in fixed rank order (identical bits on every rank)
  for (int64_t i = lo + tid; i < hi; i += kThreads) {
    v4f s = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.world; ++r) {
      s += __builtin_nontemporal_load(
          reinterpret_cast<const v4f*>(data_ptr(a.regions[a.rank], slot, r, a.slot_stride)) + i);
    }
    reinterpret_cast<v4f*>(a.x)[i] = s;
  }
  if (tail_owner && t0 + tid < a.n) {
    float s = 0.f;
    for (int r = 0; r < a.world; ++r)
      s += __builtin_nontemporal_load(data_ptr(a.regions[a.rank], slot, r, a.slot_stride) + t0 + tid);
    a.x[t0 + tid] = s;
  }
  if (tid == 0) a.gen[blk] = gen;
}

}  // namespace

int xgmi_blocks_for(int64_t n) {
  const int64_t n4 = (n + 3) / 4;
  int64_t b = (n4 + kThreads - 1) / kThreads;
  if (b < 1) b = 1;
  if (b > kXgmiMaxBlocks) b = kXgmiMaxBlocks;
  return (int)b;
}

int launch_xgmi_oneshot(const XgmiLaunch& l, hipStream_t stream) {
  if (l.world < 1 || l.world > kXgmiMaxRanks || l.n > l.slot_stride || (reinterpret_cast<uintptr_t>(l.x) & 15))
    return -1;
  Args a{};
  a.x = l.x;
  a.n = l.n;
  for (int r = 0; r < l.world; ++r) a.regions[r] = l.regions[r];
  a.rank = l.rank;
  a.world = l.world;
  a.gen = l.gen;
  a.error = l.error;
  a.slot_stride = l.slot_stride;
  a.spin_limit = l.spin_limit;
  hipLaunchKernelGGL(oneshot_allreduce_kernel, dim3(xgmi_blocks_for(l.n)), dim3(kThreads), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace comm
}  // namespace rla
