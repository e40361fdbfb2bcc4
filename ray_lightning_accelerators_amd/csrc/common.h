// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this package.
//
// Everything here is written for 64-lane wavefronts and the CDNA4 MFMA register
// layouts documented in the package README (`docs/KERNELS.md`): no CUDA shims,
// no warp-32 idioms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rla {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// Plain 16-byte vector of floats (addressable lanes, unlike HIP's float4 accessors).
struct alignas(16) F4 {
  float v[4];
};

// v_mfma_f32_16x16x32_bf16: lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15],
// D[(l>>4)*4+i][l&15].
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// A deferred BatchNorm + ReLU on two packed bf16 channels (ops/bn.py DeferredApply):
// bf16(relu(x * s + f)) per half, as bn_apply_kernel stores it for every finite
// input -- fp32 fma (one rounding), round-to-nearest-even to bf16, then the sign test
// on the bf16 bits (a negative or -0 result becomes +0; bn_apply tests before the
// rounding, which gives the same bits).  NaN with a clear sign bit passes through
// (bn_apply maps it to 0).  Packed form: one v_pk_fma_f32, one v_cvt_pk_bf16_f32 and
// one v_pk_max_i16 per word -- the operand-staging loops that call it run between
// MFMA stages with little VALU slack.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t bn_relu_bf16x2(uint32_t w, f32x2 s, f32x2 f) {
  const f32x2 x = {__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)};
  const f32x2 a = __builtin_elementwise_fma(x, s, f);
  const bf16x2v b = __builtin_convertvector(a, bf16x2v);
  const i16x2 m = __builtin_elementwise_max(__builtin_bit_cast(i16x2, b), (i16x2){0, 0});
  return __builtin_bit_cast(uint32_t, m);
}

__device__ __forceinline__ bf16x8 cvt8(float4 lo, float4 hi) {
  bf16x8 r;
  r[0] = (__bf16)lo.x; r[1] = (__bf16)lo.y; r[2] = (__bf16)lo.z; r[3] = (__bf16)lo.w;
  r[4] = (__bf16)hi.x; r[5] = (__bf16)hi.y; r[6] = (__bf16)hi.z; r[7] = (__bf16)hi.w;
  return r;
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (__bf16)0.0f;
  return r;
}

__device__ __forceinline__ float bf2f(__bf16 x) { return (float)x; }

// Raw bf16 bit helpers for host-visible uint16 buffers.
__device__ __forceinline__ uint16_t f2bf_bits(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bfbits2f(uint16_t u) {
  return __builtin_bit_cast(float, ((uint32_t)u) << 16);
}

}  // namespace rla
