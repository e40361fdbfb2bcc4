// Fusion-buffer pack / unpack for the Horovod-style engine: one launch copies up
// to kPackMax tensors (fp32) into / out of the flat fusion buffer, optionally
// scaling (the 1/size average is folded into the unpack).  The descriptor table
// travels as a by-value kernel argument, so no host->device copy per cycle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "comm/pack.h"

namespace rla {
namespace comm {
namespace {

__global__ __launch_bounds__(256) void pack_kernel(PackTable t) {
  const int e = blockIdx.y;
  if (e >= t.count) return;
  const float* __restrict__ src = t.src[e];
  float* __restrict__ dst = t.dst[e];
  const int64_t n = t.n[e];
  const float s = t.scale;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // 16-byte path when both ends are aligned (the common case: arena views)
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = i0; i < n4; i += stride) {
      float4 v = reinterpret_cast<const float4*>(src)[i];
      v.x *= s; v.y *= s; v.z *= s; v.w *= s;
      reinterpret_cast<float4*>(dst)[i] = v;
    }
    for (int64_t i = n4 * 4 + i0; i < n; i += stride) dst[i] = src[i] * s;
  } else {
    for (int64_t i = i0; i < n; i += stride) dst[i] = src[i] * s;
  }
}

}  // namespace

void launch_pack(const PackTable& t, hipStream_t stream) {
  if (t.count <= 0) return;
  int64_t maxn = 0;
  for (int i = 0; i < t.count; ++i) maxn = t.n[i] > maxn ? t.n[i] : maxn;
  int bx = (int)((maxn / 4 + 255) / 256);
  if (bx < 1) bx = 1;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(pack_kernel, dim3(bx, t.count), dim3(256), 0, stream, t);
}

}  // namespace comm
}  // namespace rla
