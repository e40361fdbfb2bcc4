// Do writes that are NOT made by a kernel (copy engines, host writes, memsets) become
// visible to the next kernel on every XCD, when that kernel's XCDs already hold the
// lines in their L2 from an earlier kernel?  (Diagnostic for the one-launch MNIST step,
// whose first step reads buffers the host just filled: order, labels, pixels, params.)
//
// Per trial: fill kernel writes A -> read kernel (512 blocks, every XCD caches every
// line) -> the buffer is overwritten with B by METHOD -> check kernel counts words != B
// per XCD.  METHOD: 0 hipMemcpy H2D from pageable memory, 1 hipMemcpyAsync H2D from
// pinned memory, 2 hipMemsetD32Async, 3 hipMemcpyAsync D2D, 4 hipMemcpy H2D pageable
// issued on a second stream, then hipStreamSynchronize, then the check on stream 0.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probes/dma_coherence_probe.hip -o build/dma_coherence_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v;
}

__global__ void fill_kernel(unsigned* buf, long n, unsigned v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) buf[i] = v;
}

__global__ void read_kernel(const unsigned* buf, long n, unsigned* sink) {
  unsigned acc = 0;
  // every block reads every line (one word per 128-B line), so every XCD caches them
  for (long i = threadIdx.x * 32; i < n; i += (long)blockDim.x * 32) acc += buf[i];
  if (acc == 0xDEADBEEF) sink[blockIdx.x] = acc;
}

__global__ void check_kernel(const unsigned* buf, long n, unsigned expect, unsigned long long* bad_by_xcc) {
  const unsigned x = xcc_id() & 7;
  unsigned long long bad = 0;
  for (long i = threadIdx.x * 32; i < n; i += (long)blockDim.x * 32) bad += buf[i] != expect;
  if (bad) atomicAdd(bad_by_xcc + x, bad);
}

int main(int argc, char** argv) {
  const int method = argc > 1 ? std::atoi(argv[1]) : 0;
  const int trials = argc > 2 ? std::atoi(argv[2]) : 300;
  const long bytes = argc > 3 ? std::atol(argv[3]) : 65536;
  const long n = bytes / 4;
  unsigned *buf, *src_dev, *sink;
  unsigned long long* bad;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&src_dev, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMalloc(&bad, 64));
  CK(hipMemset(bad, 0, 64));
  std::vector<unsigned> pageable(n);
  unsigned* pinned = nullptr;
  CK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
  hipStream_t side;
  CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
  unsigned long long windows_bad = 0, prev = 0;
  for (int t = 0; t < trials; ++t) {
    const unsigned A = 2u * t + 1u, B = 2u * t + 2u;
    hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, buf, n, A);
    hipLaunchKernelGGL(read_kernel, dim3(512), dim3(256), 0, 0, buf, n, sink);
    if (method == 0 || method == 4) {
      for (long i = 0; i < n; ++i) pageable[i] = B;
      if (method == 0) {
        CK(hipMemcpy(buf, pageable.data(), bytes, hipMemcpyHostToDevice));
      } else {
        CK(hipDeviceSynchronize());
        CK(hipMemcpyAsync(buf, pageable.data(), bytes, hipMemcpyHostToDevice, side));
        CK(hipStreamSynchronize(side));
      }
    } else if (method == 1) {
      CK(hipDeviceSynchronize());  // the previous trial's async copy has read `pinned`
      for (long i = 0; i < n; ++i) pinned[i] = B;
      CK(hipMemcpyAsync(buf, pinned, bytes, hipMemcpyHostToDevice, 0));
    } else if (method == 2) {
      CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(buf), B, n, 0));
    } else {
      hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, 0, src_dev, n, B);
      CK(hipMemcpyAsync(buf, src_dev, bytes, hipMemcpyDeviceToDevice, 0));
    }
    hipLaunchKernelGGL(check_kernel, dim3(512), dim3(256), 0, 0, buf, n, B, bad);
    if ((t & 31) == 31 || t == trials - 1) {
      CK(hipDeviceSynchronize());
      unsigned long long hb[8], tot = 0;
      CK(hipMemcpy(hb, bad, 64, hipMemcpyDeviceToHost));
      for (int i = 0; i < 8; ++i) tot += hb[i];
      if (tot != prev) ++windows_bad;
      prev = tot;
    }
  }
  CK(hipDeviceSynchronize());
  unsigned long long hb[8], tot = 0;
  CK(hipMemcpy(hb, bad, 64, hipMemcpyDeviceToHost));
  for (int i = 0; i < 8; ++i) tot += hb[i];
  std::printf("{\"method\": %d, \"trials\": %d, \"bytes\": %ld, \"checked_words\": %lld, \"stale_words\": %llu, "
              "\"windows_with_stale\": %llu, \"stale_by_xcc\": [%llu,%llu,%llu,%llu,%llu,%llu,%llu,%llu]}\n",
              method, trials, bytes, (long long)trials * 512 * ((n + 31) / 32), tot, windows_bad, hb[0], hb[1], hb[2],
              hb[3], hb[4], hb[5], hb[6], hb[7]);
  CK(hipHostFree(pinned));
  return 0;
}
