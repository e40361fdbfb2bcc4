// ARCHIVED DEBUG KERNEL (not built; removed from the _C extension in round 6).
// LDS poison fill used for the round-5 one-launch investigation
// (profiles/r5_mnist/poison_full_128.log); build it standalone if needed again.
// Debug tooling: fill every CU's LDS with a bit pattern (e.g. bf16 +Inf pairs), so a
// kernel that reads LDS it never wrote shows it deterministically instead of only
// after some earlier kernel happened to leave such bytes there (tests / probes only).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace rla {
namespace {

constexpr int kPoisonBytes = 160 * 1024;

__global__ __launch_bounds__(256) void lds_poison_kernel(uint32_t pattern, int* sink) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_words[];
  for (int i = threadIdx.x; i < kPoisonBytes / 4; i += blockDim.x) lds_words[i] = pattern;
  __syncthreads();
  // keep the stores observable: one lane of one block writes a word it read back
  if (blockIdx.x == 0 && threadIdx.x == 0) sink[0] = (int)lds_words[kPoisonBytes / 4 - 1];
}

}  // namespace

int launch_lds_poison(uint32_t pattern, int* sink, int blocks, hipStream_t s) {
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&lds_poison_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kPoisonBytes) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(256), kPoisonBytes, s, pattern, sink);
  return 0;
}

}  // namespace rla
