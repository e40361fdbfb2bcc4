// Cross-XCD coherence probe (diagnostic, not part of the package build).
//
// Question: the one-launch MNIST step (csrc/mlp_step3.hip, mlp3_one_kernel) lets every
// block's head prefetch BOTH ring slots of H1pre / the label ring while other blocks of
// the same launch write the "next" slot (atomics / plain stores).  The value read from
// the next slot is discarded -- but can such a racing read leave a line in the reading
// XCD's L2 (or scalar cache) that is still STALE in the next launch, where that slot is
// the one consumed?
//
// Each trial: reset (kernel) -> race (readers + writers in one launch, uneven start
// delays) -> check (every block re-reads every line in a NEW launch and counts words
// that differ from the value the writers left).  Modes:
//   0  writers: agent atomics (like the H1pre partial sums), readers: plain loads, racing
//   1  writers: plain stores of a per-trial value (like the label ring), readers racing
//   2  as 0, but the readers finish before any writer starts (read-before-write, no race:
//      the steady-state pattern of the one-launch step)
//   3  as 0, check kernel reads through the scalar path (s_load)
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probes/coherence_probe.hip -o build/coherence_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

constexpr int kLineWords = 16;  // 128-byte lines of int64
constexpr int kThreads = 256;

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

__device__ __forceinline__ unsigned mix(unsigned a, unsigned b) {
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

__global__ void reset_kernel(long long* buf, int nlines) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nlines * kLineWords; i += gridDim.x * blockDim.x)
    buf[i] = 0;
}

__device__ __forceinline__ void spin_cycles(long long cycles) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  // memrealtime runs at 100 MHz: cycles are 10-ns ticks; bounded by construction
  for (int i = 0; i < 100000; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 >= cycles) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

// readers: even blocks; writers: odd blocks
__global__ void race_kernel(long long* buf, int nlines, int mode, unsigned trial, long long* sink) {
  const int blk = blockIdx.x, tid = threadIdx.x;
  const bool reader = (blk & 1) == 0;
  const unsigned h = mix(blk, trial);
  if (mode == 2) {
    if (!reader) spin_cycles(3000);  // 30 us: every reader is done first
  } else {
    spin_cycles(h % 800);  // 0..8 us of uneven start
  }
  if (reader) {
    long long acc = 0;
    for (int rep = 0; rep < 4; ++rep)
      for (int l = tid; l < nlines; l += kThreads) acc += buf[(long long)l * kLineWords];
    if (acc == 0x7fffffffffffffffLL) sink[blk] = acc;  // keep the loads
  } else {
    const int wid = blk >> 1;
    for (int l = tid; l < nlines; l += kThreads) {
      long long* p = buf + (long long)l * kLineWords;
      if (mode == 1) {
        // one writer owns each line: plain store of the trial's value
        if ((l % (gridDim.x / 2)) == wid) *p = (long long)trial + 1;
      } else {
        atomicAdd(reinterpret_cast<unsigned long long*>(p), 1ull);
      }
    }
  }
}

__global__ void check_kernel(const long long* buf, int nlines, long long expect, int scalar,
                             unsigned long long* bad_by_xcc, unsigned long long* checked) {
  const unsigned x = xcc_id() & 7;
  unsigned long long bad = 0, n = 0;
  if (scalar) {
    // scalar path: one wave, uniform addresses (s_load through the constant address space)
    if (threadIdx.x < 64) {
      const __attribute__((address_space(4))) long long* c =
          (const __attribute__((address_space(4))) long long*)buf;
      for (int l = (blockIdx.x * 7) % nlines, k = 0; k < 64; ++k, l = (l + 61) % nlines) {
        const long long v = c[(long long)l * kLineWords];
        if (threadIdx.x == 0) { bad += v != expect; ++n; }
      }
    }
  } else {
    for (int l = threadIdx.x; l < nlines; l += kThreads) {
      bad += buf[(long long)l * kLineWords] != expect;
      ++n;
    }
  }
  if (n) atomicAdd(checked, n);
  if (bad) atomicAdd(bad_by_xcc + x, bad);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const int trials = argc > 2 ? std::atoi(argv[2]) : 500;
  const int nlines = argc > 3 ? std::atoi(argv[3]) : 2048;
  const int grid = 512;
  long long *buf, *sink;
  unsigned long long *bad, *checked;
  CK(hipMalloc(&buf, (size_t)nlines * kLineWords * 8));
  CK(hipMalloc(&sink, grid * 8));
  CK(hipMalloc(&bad, 8 * 8));
  CK(hipMalloc(&checked, 8));
  CK(hipMemset(bad, 0, 64));
  CK(hipMemset(checked, 0, 8));
  const long long expect_atomic = grid / 2;
  unsigned long long trials_bad = 0;
  std::vector<unsigned long long> hb(8), prev(8, 0);
  for (int t = 0; t < trials; ++t) {
    hipLaunchKernelGGL(reset_kernel, dim3(256), dim3(kThreads), 0, 0, buf, nlines);
    hipLaunchKernelGGL(race_kernel, dim3(grid), dim3(kThreads), 0, 0, buf, nlines, mode, (unsigned)t, sink);
    const long long expect = mode == 1 ? (long long)t + 1 : expect_atomic;
    hipLaunchKernelGGL(check_kernel, dim3(grid), dim3(kThreads), 0, 0, buf, nlines, expect, mode == 3 ? 1 : 0,
                       bad, checked);
    if ((t & 63) == 63 || t == trials - 1) {
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(hb.data(), bad, 64, hipMemcpyDeviceToHost));
      unsigned long long tot = 0, ptot = 0;
      for (int i = 0; i < 8; ++i) { tot += hb[i]; ptot += prev[i]; }
      if (tot != ptot) ++trials_bad;
      prev = hb;
    }
  }
  CK(hipDeviceSynchronize());
  unsigned long long hc = 0;
  CK(hipMemcpy(hb.data(), bad, 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hc, checked, 8, hipMemcpyDeviceToHost));
  unsigned long long tot = 0;
  for (int i = 0; i < 8; ++i) tot += hb[i];
  std::printf("{\"mode\": %d, \"trials\": %d, \"lines\": %d, \"checked_words\": %llu, \"stale_words\": %llu, "
              "\"windows_with_stale\": %llu, \"stale_by_xcc\": [%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu]}\n",
              mode, trials, nlines, hc, tot, trials_bad, hb[0], hb[1], hb[2], hb[3], hb[4], hb[5], hb[6], hb[7]);
  return 0;
}
