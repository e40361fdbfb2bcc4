// NHWC bf16 max pooling with a compact window argmax, gfx950 (ResNet-50's stem:
// 3x3 / stride 2 / pad 1 over [N, 112, 112, 64]).
//
// Why (profiles/r1_resnet50_v2/kernel_stats_native_fusedbn.csv): PyTorch-ROCm's
// max_pool_backward_nhwc took 316 us per step -- it scatters through int64 indices
// (8 bytes per output element, as large as the bf16 input itself) -- and the forward
// writes those indices.  Here the forward stores the position inside the k x k
// window as ONE byte, and the backward GATHERS: each thread owns 8 channels (one
// 16-byte vector) of one input pixel and sums the gradient of every output window
// (<= ceil(k/s)^2 of them) whose argmax is that pixel -- no atomics, each input
// gradient written once, fully coalesced.  Tie / NaN rule as PyTorch (first maximum
// in row-major window order wins; NaN propagates), so gradients match it exactly.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kernels.h"

namespace rla {
namespace {

typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f8 ld8(const uint16_t* p) {
  return __builtin_convertvector(__builtin_bit_cast(b8, *reinterpret_cast<const u16x8*>(p)), f8);
}

// one thread: 8 channels of one output pixel.
// BN (the stem's BatchNorm + ReLU folded in, round 5): the input is the BatchNorm's
// INPUT and each window element is first mapped exactly as bn_apply_kernel<relu>
// would store it -- bf16(max(x * scale + shift, 0)) with one fused multiply-add --
// so the pooled values and argmax equal the unfused pair's, and the 205 MB
// activation between them is never written or re-read.  ss = the finalize's
// [4, C] stats (rows 2, 3: scale, shift); nbt_inc as bn_apply's.
template <bool BN>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int OH, int OW, int k, int s, int pad,
                                                          const float* __restrict__ ss, int64_t* nbt_inc) {
  const int G = C >> 3;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (BN && nbt_inc && t == 0) nbt_inc[0] += 1;
  const int64_t total = (int64_t)N * OH * OW * G;
  if (t >= total) return;
  const int g = (int)(t % G);
  f8 sc, sf;
  if (BN) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      sc[c] = ss[2 * C + g * 8 + c];
      sf[c] = ss[3 * C + g * 8 + c];
    }
  }
  int64_t p = t / G;
  const int ow = (int)(p % OW);
  p /= OW;
  const int oh = (int)(p % OH);
  const int n = (int)(p / OH);
  f8 m;
  uint8_t a[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    m[c] = -INFINITY;
    a[c] = 0;
  }
  const int h0 = oh * s - pad, w0 = ow * s - pad;
  for (int kh = 0; kh < k; ++kh) {
    const int h = h0 + kh;
    if (h < 0 || h >= H) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int w = w0 + kw;
      if (w < 0 || w >= W) continue;
      f8 v = ld8(x + (((int64_t)n * H + h) * W + w) * C + g * 8);
      if (BN) {
        v = __builtin_elementwise_fma(v, sc, sf);
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = v[c] > 0.f ? v[c] : 0.f;
        v = __builtin_convertvector(__builtin_convertvector(v, b8), f8);  // the bf16 bn_apply stores
      }
      const uint8_t pos = (uint8_t)(kh * k + kw);
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (v[c] > m[c] || isnan(v[c])) {  // PyTorch's rule, NaN included
          m[c] = v[c];
          a[c] = pos;
        }
    }
  }
  *reinterpret_cast<u16x8*>(y + t * 8) = __builtin_bit_cast(u16x8, __builtin_convertvector(m, b8));
  uint64_t packed = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) packed |= (uint64_t)a[c] << (8 * c);
  *reinterpret_cast<uint64_t*>(arg + t * 8) = packed;
}

// one thread: 8 channels of one input pixel; gathers the windows that contain it
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ arg, uint16_t* __restrict__ dx,
                                                          int N, int H, int W, int C, int OH, int OW, int k, int s,
                                                          int pad) {
  const int G = C >> 3;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)N * H * W * G;
  if (t >= total) return;
  const int g = (int)(t % G);
  int64_t p = t / G;
  const int w = (int)(p % W);
  p /= W;
  const int h = (int)(p % H);
  const int n = (int)(p / H);
  // windows oh with oh*s - pad <= h <= oh*s - pad + k - 1
  const int hp = h + pad, wp = w + pad;
  const int oh_lo = hp >= k ? (hp - k) / s + 1 : 0, oh_hi = min(hp / s, OH - 1);
  const int ow_lo = wp >= k ? (wp - k) / s + 1 : 0, ow_hi = min(wp / s, OW - 1);
  f8 acc;
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.f;
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int kh = hp - oh * s;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int kw = wp - ow * s;
      const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * C + g * 8;
      const uint64_t packed = *reinterpret_cast<const uint64_t*>(arg + o);
      const f8 d = ld8(dy + o);
      const uint8_t pos = (uint8_t)(kh * k + kw);
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if ((uint8_t)(packed >> (8 * c)) == pos) acc[c] += d[c];
    }
  }
  *reinterpret_cast<u16x8*>(dx + t * 8) = __builtin_bit_cast(u16x8, __builtin_convertvector(acc, b8));
}

// Global average pool backward: dx[n][p][c] = dy[n][c] / HW over NHWC rows, one
// 16-byte store of 8 channels per thread (autograd's expand + channels_last copy
// ran as an unvectorised broadcast copy, ~44 us per ResNet-50 step).
__global__ __launch_bounds__(256) void gap_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx,
                                                      int N, int HW, int C, float scale) {
  const int G = C >> 3;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * HW * G) return;
  const int g = (int)(t % G);
  const int n = (int)(t / ((int64_t)HW * G));
  const f8 d = ld8(dy + (int64_t)n * C + g * 8) * scale;
  *reinterpret_cast<u16x8*>(dx + t * 8) = __builtin_bit_cast(u16x8, __builtin_convertvector(d, b8));
}

// d[n][oh s][ow s][:] += g[(n OH + oh) OW + ow][:] over NHWC bf16 rows: the strided
// downsample branch's input gradient added into every s-th pixel of the parked one
// (ops/conv.py GradFork).  One thread = 8 channels: fp32 add, one bf16 rounding --
// exactly ATen's bf16 add_, which ran this strided view through its non-vectorised
// elementwise path (~22 us a call, profiles/r5_final3/kernel_stats_rn50.csv).
__global__ __launch_bounds__(256) void strided_add_kernel(uint16_t* __restrict__ d, const uint16_t* __restrict__ g,
                                                          int N, int H, int W, int C, int OH, int OW, int s) {
  const int G = C >> 3;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * OH * OW * G) return;
  const int gi = (int)(t % G);
  const int64_t p = t / G;
  const int ow = (int)(p % OW);
  const int64_t q = p / OW;
  const int oh = (int)(q % OH), n = (int)(q / OH);
  uint16_t* dp = d + (((int64_t)n * H + (int64_t)oh * s) * W + (int64_t)ow * s) * C + gi * 8;
  const f8 a = ld8(dp) + ld8(g + t * 8);
  *reinterpret_cast<u16x8*>(dp) = __builtin_bit_cast(u16x8, __builtin_convertvector(a, b8));
}

}  // namespace

int launch_strided_add(uint16_t* d, const uint16_t* g, int N, int H, int W, int C, int OH, int OW, int s,
                       hipStream_t stream) {
  if (C % 8 || s < 1 || (OH - 1) * s >= H || (OW - 1) * s >= W) return -1;
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffff) return -2;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(strided_add_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d, g, N, H, W, C, OH, OW, s);
  return 0;
}

int launch_gap_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t stream) {
  if (C % 8 || HW < 1) return -1;
  const int64_t total = (int64_t)N * HW * (C / 8);
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffff) return -2;
  hipLaunchKernelGGL(gap_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, dy, dx, N, HW, C, 1.0f / (float)HW);
  return 0;
}

int launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int OH, int OW,
                       int k, int s, int pad, hipStream_t stream, const float* bn_ss, int64_t* nbt_inc) {
  if (C % 8 || k < 1 || k > 15 || s < 1) return -1;
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffff) return -2;
  if (bn_ss)
    hipLaunchKernelGGL(maxpool_fwd_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, arg, N, H, W, C,
                       OH, OW, k, s, pad, bn_ss, nbt_inc);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, arg, N, H, W,
                       C, OH, OW, k, s, pad, nullptr, nullptr);
  return 0;
}

int launch_maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int OH,
                       int OW, int k, int s, int pad, hipStream_t stream) {
  if (C % 8 || k < 1 || k > 15 || s < 1) return -1;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffff) return -2;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, dy, arg, dx, N, H, W, C, OH,
                     OW, k, s, pad);
  return 0;
}

}  // namespace rla
