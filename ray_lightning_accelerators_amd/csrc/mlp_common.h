// Shared pieces of the fused MNIST-MLP kernels (mlp_step3.hip step, mlp_adam.hip
// arena Adam): arena offsets, Adam scalar math, LDS fragment loaders.
#pragma once
#include <math.h>

#include "common.h"

namespace rla {
namespace mlp {

constexpr int kD = 784;   // input features
constexpr int kNC = 10;   // classes
constexpr int kTiles = kD / 16;  // 16-pixel W1 column tiles (49)

// fp32 arena == bf16 shadow row-major copy; W2^T / W3^T follow in the shadow.
template <int L1, int L2>
struct Off {
  static constexpr int64_t W1 = 0, B1 = (int64_t)L1 * kD, W2 = B1 + L1, B2 = W2 + (int64_t)L2 * L1,
                           W3 = B2 + L2, B3 = W3 + kNC * L2, NP = B3 + kNC;
  static constexpr int64_t W2T = (NP + 7) / 8 * 8, W3T = W2T + (int64_t)L1 * L2;
};

struct AdamScal {
  float lr, step_size, bc2_sqrt, beta1, beta2, eps, wd;
  int adamw;
};

// torch.optim.Adam's bias corrections, in double like the eager optimizer.
__device__ __forceinline__ void adam_scalars(AdamScal& o, int64_t t, float lr, float b1, float b2, float eps,
                                             float wd, int adamw) {
  const double bc1 = 1.0 - pow((double)b1, (double)t);
  const double bc2 = 1.0 - pow((double)b2, (double)t);
  o.lr = lr;
  o.step_size = (float)((double)lr / bc1);
  o.bc2_sqrt = (float)sqrt(bc2);
  o.beta1 = b1; o.beta2 = b2; o.eps = eps; o.wd = wd; o.adamw = adamw;
}

// Explicit FMAs and no compiler contraction: every kernel that inlines this (tail
// epilogues, the one-launch step's tiles, the arena Adam) computes the same bits.
__device__ __forceinline__ float adam1(float p, float g, float& m, float& v, const AdamScal& o) {
#pragma clang fp contract(off)
  if (o.wd != 0.f) {
    if (o.adamw) p = p * (1.f - o.lr * o.wd);
    else g = fmaf(o.wd, p, g);
  }
  m = fmaf(1.f - o.beta1, g - m, m);
  v = fmaf(1.f - o.beta2, g * g, v * o.beta2);
  const float denom = sqrtf(v) / o.bc2_sqrt + o.eps;
  return fmaf(-o.step_size, m / denom, p);
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
// ds_read_b64_tr_b16: lane i of each 16-lane group receives column i of the
// 4x16 bf16 block whose rows lanes 4q+p point at.
__device__ __forceinline__ bf16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
__device__ __forceinline__ bf16x8 ld8(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// u8 pixels (16 per uint4) -> two bf16x8, scaled by 1/255 (torchvision ToTensor).
__device__ __forceinline__ void u8x16_to_bf16(const uint4 v, bf16x8& lo, bf16x8& hi) {
  const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
  constexpr float inv255 = 1.0f / 255.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    lo[j] = (__bf16)((float)((wd[0] >> (8 * j)) & 0xffu) * inv255);
    lo[4 + j] = (__bf16)((float)((wd[1] >> (8 * j)) & 0xffu) * inv255);
    hi[j] = (__bf16)((float)((wd[2] >> (8 * j)) & 0xffu) * inv255);
    hi[4 + j] = (__bf16)((float)((wd[3] >> (8 * j)) & 0xffu) * inv255);
  }
}

}  // namespace mlp
}  // namespace rla
