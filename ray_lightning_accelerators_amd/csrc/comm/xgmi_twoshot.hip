// Two-shot allreduce over xGMI peer memory (single node, <= 8 GPUs): the
// medium/large-bucket algorithm of SURVEY.md §5.8 (ResNet-50's 8-25 MiB DDP
// buckets, Horovod fusion batches), with an optional bf16 wire format.
//
// Why two-shot on MI355X: the 8 GPUs of a node are a full xGMI mesh (7
// point-to-point links per GPU).  A ring moves 2(W-1)/W * S bytes over ONE link
// per hop, so it is per-link bound; the one-shot moves S over every link.  The
// two-shot moves S/W over every link in each of its two phases, i.e. 2S/W per
// link with all 7 links busy at once:
//
//   phase 1 (reduce-scatter): chunk c of the bucket belongs to rank c.  Every
//            rank PUSHES its copy of chunk c into rank c's scatter area
//            [slot][src] (7 concurrent link writes of S/W each), then raises a
//            per-(block, src) flag in the owner's region;
//   reduce:  the owner sums the W contributions of its chunk in fixed rank
//            order (bitwise-identical on every rank, independent of arrival
//            order), writes the result into its own bucket and PUSHES it into
//            every peer's gather area [slot][owner];
//   phase 2 (all-gather): after the W phase-2 flags, every rank copies the
//            W-1 reduced chunks it received into its bucket.
//
// bf16 wire (grad_dtype="bf16"): the fp32 bucket is converted to bf16 as it is
// pushed (no separate pack kernel, half the link bytes), summed in fp32 by the
// owner, rounded to bf16 once and broadcast; the owner stores the SAME rounded
// value into its own bucket, so every replica holds identical bits.
//
// Block b of every rank owns the same sub-range of every chunk, so flags are per
// (slot, phase, block, src) and no block ever waits on another block of its own
// GPU: blocks only wait on the SAME block index of the peers, which never waits
// on us in a cycle, so a partially-resident grid or a concurrent compute kernel
// cannot deadlock the protocol.
//
// Memory protocol = the one-shot's (xgmi_allreduce.hip): uncached device memory
// mapped with hipIpcOpenMemHandle, data stores -> every wave's vmcnt(0) +
// __threadfence_system() -> barrier -> system-scope flag store; bounded
// system-scope polls -> fence -> barrier -> loads.  Generations are per block in
// device memory (hipGraph replayable) and the areas are double-buffered by
// generation parity: a rank writes slot s of generation g+2 only after every
// peer raised its phase-2 flag of g+1, i.e. after every peer's kernel of
// generation g retired.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comm/xgmi.h"

namespace rla {
namespace comm {
namespace {

constexpr int kThreads = 512;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v4b __attribute__((ext_vector_type(4)));

// wire element: fp32 (exact) or bf16 (half the bytes on the links)
template <bool BF16>
struct Wire;
template <>
struct Wire<false> {
  typedef float T;
  typedef v4f V;
  static __device__ __forceinline__ V pack(v4f v) { return v; }
  static __device__ __forceinline__ v4f unpack(V v) { return v; }
  static __device__ __forceinline__ T pack1(float v) { return v; }
  static __device__ __forceinline__ float unpack1(T v) { return v; }
};
template <>
struct Wire<true> {
  typedef __bf16 T;
  typedef v4b V;
  static __device__ __forceinline__ V pack(v4f v) { return __builtin_convertvector(v, v4b); }
  static __device__ __forceinline__ v4f unpack(V v) { return __builtin_convertvector(v, v4f); }
  static __device__ __forceinline__ T pack1(float v) { return (__bf16)v; }
  static __device__ __forceinline__ float unpack1(T v) { return (float)v; }
};

struct Args {
  float* x;
  int64_t n;
  char* regions[kXgmiMaxRanks];
  int rank, world;
  uint32_t* gen;         // [kTwoShotMaxBlocks]
  int* error;
  int64_t chunk_stride;  // wire elements per (slot, area, rank) sub-area
  int64_t cs;            // chunk length in elements (multiple of 4)
  int64_t per4;          // 4-element groups per block within a chunk
  int64_t spin_limit;
};

__device__ __forceinline__ uint32_t* ts_flag(char* region, int slot, int phase, int blk, int src) {
  return reinterpret_cast<uint32_t*>(region) +
         (((size_t)slot * 2 + phase) * kTwoShotMaxBlocks + blk) * kXgmiMaxRanks + src;
}

// area 0 = scatter (indexed by source rank), area 1 = gather (indexed by owner)
template <typename T>
__device__ __forceinline__ T* ts_area(const Args& a, char* region, int slot, int area, int r) {
  return reinterpret_cast<T*>(region + kXgmiFlagBytes) + (((int64_t)slot * 2 + area) * a.world + r) * a.chunk_stride;
}

__device__ __forceinline__ int64_t chunk_len(const Args& a, int c) {
  const int64_t l = a.n - (int64_t)c * a.cs;
  return l <= 0 ? 0 : (l < a.cs ? l : a.cs);
}

// the scalar tail of a chunk (len % 4 elements) belongs to the block whose
// group range holds index len/4 (the same block on every rank)
__device__ __forceinline__ int tail_block(const Args& a, int64_t len4) {
  const int64_t b = len4 / a.per4;
  return (int)(b < (int64_t)gridDim.x ? b : gridDim.x - 1);
}

// Raise my flag for (slot, phase, blk) in every peer's region and wait for the
// W-1 peer flags of that phase in mine.  Returns false on timeout.
__device__ __forceinline__ bool ts_barrier(const Args& a, int slot, int phase, int blk, uint32_t gen,
                                           int* sh_fail) {
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // never let the flag overtake a wave's stores
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < a.world && tid != a.rank) {
    __hip_atomic_store(ts_flag(a.regions[tid], slot, phase, blk, a.rank), gen, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = ts_flag(a.regions[a.rank], slot, phase, blk, tid);
    int64_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != gen) {
      if (++spins > a.spin_limit) {
        *sh_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __threadfence_system();
  __syncthreads();
  return *sh_fail == 0;
}

template <bool BF16>
__global__ __launch_bounds__(kThreads) void twoshot_allreduce_kernel(Args a) {
  typedef Wire<BF16> Wr;
  typedef typename Wr::T T;
  typedef typename Wr::V V;
  __shared__ uint32_t sh_gen;
  __shared__ int sh_fail;
  const int blk = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    sh_gen = a.gen[blk] + 1u;
    sh_fail = 0;
  }
  __syncthreads();
  const uint32_t gen = sh_gen;
  const int slot = gen & 1u;
  const int me = a.rank;
  const int64_t lo4 = blk * a.per4, hi4 = lo4 + a.per4;
  bool ok;

  // ---- phase 1: push chunk c of my bucket into rank c's scatter area [slot][me]
  for (int64_t i = lo4 + tid; i < hi4; i += kThreads) {
    for (int c = 0; c < a.world; ++c) {
      if (c == me || i >= chunk_len(a, c) / 4) continue;
      const v4f v = reinterpret_cast<const v4f*>(a.x + (int64_t)c * a.cs)[i];
      __builtin_nontemporal_store(Wr::pack(v), reinterpret_cast<V*>(ts_area<T>(a, a.regions[c], slot, 0, me)) + i);
    }
  }
  for (int c = 0; c < a.world; ++c) {
    const int64_t len = chunk_len(a, c), len4 = len / 4, e = len4 * 4 + tid;
    if (c != me && tail_block(a, len4) == blk && e < len)
      __builtin_nontemporal_store(Wr::pack1(a.x[(int64_t)c * a.cs + e]), ts_area<T>(a, a.regions[c], slot, 0, me) + e);
  }
  ok = ts_barrier(a, slot, 0, blk, gen, &sh_fail);

  // ---- reduce my chunk in fixed rank order, keep it, push it to every gather area
  if (ok) {
    const int64_t len = chunk_len(a, me), len4 = len / 4;
    float* own = a.x + (int64_t)me * a.cs;
    const int64_t end4 = hi4 < len4 ? hi4 : len4;
    for (int64_t i = lo4 + tid; i < end4; i += kThreads) {
      v4f s = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < a.world; ++r)
        s += r == me ? Wr::unpack(Wr::pack(reinterpret_cast<const v4f*>(own)[i]))
                     : Wr::unpack(__builtin_nontemporal_load(
                           reinterpret_cast<const V*>(ts_area<T>(a, a.regions[me], slot, 0, r)) + i));
      const V w = Wr::pack(s);
      reinterpret_cast<v4f*>(own)[i] = Wr::unpack(w);
      for (int r = 0; r < a.world; ++r)
        if (r != me) __builtin_nontemporal_store(w, reinterpret_cast<V*>(ts_area<T>(a, a.regions[r], slot, 1, me)) + i);
    }
    const int64_t e = len4 * 4 + tid;
    if (tail_block(a, len4) == blk && e < len) {
      float s = 0.f;
      for (int r = 0; r < a.world; ++r)
        s += r == me ? Wr::unpack1(Wr::pack1(own[e]))
                     : Wr::unpack1(__builtin_nontemporal_load(ts_area<T>(a, a.regions[me], slot, 0, r) + e));
      const T w = Wr::pack1(s);
      own[e] = Wr::unpack1(w);
      for (int r = 0; r < a.world; ++r)
        if (r != me) __builtin_nontemporal_store(w, ts_area<T>(a, a.regions[r], slot, 1, me) + e);
    }
    ok = ts_barrier(a, slot, 1, blk, gen, &sh_fail);
  }

  // ---- phase 2: copy the W-1 reduced chunks I received into my bucket
  if (ok) {
    for (int64_t i = lo4 + tid; i < hi4; i += kThreads) {
      for (int c = 0; c < a.world; ++c) {
        if (c == me || i >= chunk_len(a, c) / 4) continue;
        reinterpret_cast<v4f*>(a.x + (int64_t)c * a.cs)[i] = Wr::unpack(
            __builtin_nontemporal_load(reinterpret_cast<const V*>(ts_area<T>(a, a.regions[me], slot, 1, c)) + i));
      }
    }
    for (int c = 0; c < a.world; ++c) {
      const int64_t len = chunk_len(a, c), len4 = len / 4, e = len4 * 4 + tid;
      if (c != me && tail_block(a, len4) == blk && e < len)
        a.x[(int64_t)c * a.cs + e] =
            Wr::unpack1(__builtin_nontemporal_load(ts_area<T>(a, a.regions[me], slot, 1, c) + e));
    }
  }
  if (tid == 0) {
    if (!ok) __hip_atomic_store(a.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    a.gen[blk] = gen;  // also on failure: stay in step with the peers' numbering
  }
  // Every generation entry advances on every launch, also those of block indices
  // this (smaller) grid does not have: the slot parity must be the same for ALL
  // blocks of a launch, or a block of launch m could write the slot a different
  // block of a peer's launch m-1 still reads when consecutive buckets differ in size.
  if (blk == 0)
    for (int k = gridDim.x + tid; k < kTwoShotMaxBlocks; k += kThreads) a.gen[k] = gen;
}

}  // namespace

TwoShotPlan twoshot_plan(int64_t n, int world) {
  TwoShotPlan p{};
  // chunk length: ceil(n / W) rounded up to whole groups of 4, so every chunk
  // starts 16-byte aligned when the bucket does
  int64_t cs = (n + world - 1) / world;
  cs = (cs + 3) / 4 * 4;
  if (cs < 4) cs = 4;
  const int64_t cs4 = cs / 4;
  // ~2 passes of 512 threads per block, at most kTwoShotMaxBlocks blocks
  // (<< 256 CUs, so the grid is resident while it polls)
  int64_t b = (cs4 + 2 * kThreads - 1) / (2 * kThreads);
  if (b < 1) b = 1;
  if (b > kTwoShotMaxBlocks) b = kTwoShotMaxBlocks;
  p.cs = cs;
  p.blocks = (int)b;
  p.per4 = (cs4 + b - 1) / b;
  return p;
}

int launch_xgmi_twoshot(const XgmiLaunch& l, bool bf16_wire, hipStream_t stream) {
  if (l.world < 2 || l.world > kXgmiMaxRanks || (reinterpret_cast<uintptr_t>(l.x) & 15)) return -1;
  const TwoShotPlan p = twoshot_plan(l.n, l.world);
  // the region is sized in fp32 elements; a bf16 wire uses half of each area
  if (p.cs > l.slot_stride) return -1;
  Args a{};
  a.x = l.x;
  a.n = l.n;
  for (int r = 0; r < l.world; ++r) a.regions[r] = l.regions[r];
  a.rank = l.rank;
  a.world = l.world;
  a.gen = l.gen;
  a.error = l.error;
  a.chunk_stride = bf16_wire ? 2 * l.slot_stride : l.slot_stride;
  a.cs = p.cs;
  a.per4 = p.per4;
  a.spin_limit = l.spin_limit;
  if (bf16_wire)
    hipLaunchKernelGGL(twoshot_allreduce_kernel<true>, dim3(p.blocks), dim3(kThreads), 0, stream, a);
  else
    hipLaunchKernelGGL(twoshot_allreduce_kernel<false>, dim3(p.blocks), dim3(kThreads), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace comm
}  // namespace rla
