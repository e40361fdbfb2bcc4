// Max-pool backward as a per-element gather, for kernels that CONSUME the pooled
// layer's input gradient (csrc/bn_act.hip POOL: the ResNet stem's BatchNorm backward
// reads its dy through this instead of a materialised maxpool_bwd output).
// Same windows, order and bf16 rounding as pool.hip's maxpool_bwd_kernel, so the
// value is bitwise what that kernel would have stored.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"  // PoolGrad

namespace rla {

// dy of input pixel (n, h, w) (row = (n H + h) W + w), channels col .. col + 8, as fp32
// of the bf16 the unfused kernel stores
template <typename F8, typename B8, typename U8>
__device__ __forceinline__ F8 pool_grad8(const PoolGrad& pg, int C, int64_t row, int col) {
  const int w = (int)(row % pg.W);
  const int64_t nh = row / pg.W;
  const int h = (int)(nh % pg.H);
  const int n = (int)(nh / pg.H);
  const int hp = h + pg.pad, wp = w + pg.pad;
  const int oh_lo = hp >= pg.k ? (hp - pg.k) / pg.s + 1 : 0, oh_hi = min(hp / pg.s, pg.OH - 1);
  const int ow_lo = wp >= pg.k ? (wp - pg.k) / pg.s + 1 : 0, ow_hi = min(wp / pg.s, pg.OW - 1);
  F8 acc;
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.f;
  for (int oh = oh_lo; oh <= oh_hi; ++oh) {
    const int kh = hp - oh * pg.s;
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const int kw = wp - ow * pg.s;
      const int64_t o = (((int64_t)n * pg.OH + oh) * pg.OW + ow) * C + col;
      const uint64_t packed = *reinterpret_cast<const uint64_t*>(pg.arg + o);
      const F8 d = __builtin_convertvector(__builtin_bit_cast(B8, *reinterpret_cast<const U8*>(pg.g + o)), F8);
      const uint8_t pos = (uint8_t)(kh * pg.k + kw);
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if ((uint8_t)(packed >> (8 * c)) == pos) acc[c] += d[c];
    }
  }
  return __builtin_convertvector(__builtin_convertvector(acc, B8), F8);
}

}  // namespace rla
