// Fused training step of the MNIST classifier MLP (784 -> L1 -> L2 -> 10) for
// gfx950: forward (3 GEMMs + bias + ReLU), log_softmax + NLL + accuracy,
// backward (5 GEMMs, ReLU masks, bias column sums) and, at world size 1, the
// Adam update fused into the weight-gradient epilogues -- ONE launch per step.
//
// Why one workgroup: at the reference's default config (batch 32, layers
// 32/64; reference examples/ray_ddp_example.py:167) a step is
// ~3.5 MFLOP over a ~110 KB weight set; it is launch- and latency-bound, not
// FLOP-bound.  A single 512-thread workgroup keeps every
// activation in LDS, uses bf16 MFMA (v_mfma_f32_16x16x32_bf16, fp32 accumulate)
// for all eight products and never round-trips an activation through HBM.
//
// Layout conventions (16x16x32 bf16 MFMA, wave64):
//   A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15], D[row 4(l>>4)+i][col l&15]
//   * forward operands are read k-contiguous: X rows and W rows (nn.Linear
//     stores W as [out, in], so W rows ARE the B-operand columns);
//   * activations are written twice, row-major (next forward A operand) and
//     transposed [feature][batch] (the batch-contracted weight-gradient
//     operands), each as a 4-element packed store straight from the MFMA
//     accumulator;
//   * dW1 contracts over the batch of the pixel tile: its A operand (X^T) is
//     read from the row-major X image with ds_read_b64_tr_b16 (hardware
//     transpose read), so X is staged in LDS once and never re-read.
// The parameter arena layout equals nn.Linear state_dict order:
//   W1[L1,784] b1[L1] W2[L2,L1] b2[L2] W3[10,L2] b3[10].
#include "common.h"
#include "kernels.h"
#include <math.h>

namespace rla {
namespace {

constexpr int kD = 784;        // input features
constexpr int kKS1 = 25;       // ceil(784 / 32) K-steps of layer 1
constexpr int kXS = 808;       // LDS row stride of X (bf16): 1616 B -> rows 20 dwords apart, conflict-free b128
constexpr int kNC = 10;        // classes
constexpr int kThreads = 512;  // 8 waves
constexpr int kWaves = kThreads / 64;
constexpr int kDZS = 40;       // dZ row stride (K padded to 32 + 8)

constexpr size_t cmax(size_t a, size_t b) { return a > b ? a : b; }

template <int BC, int L1, int L2>
struct Cfg {
  static constexpr int H1S = L1 + 8, H2S = L2 + 8, TS = BC + 8;
  static constexpr int MT = BC / 16, TN1 = L1 / 16, TN2 = L2 / 16;
  static constexpr size_t oX = 0;
  static constexpr size_t oH1 = oX + (size_t)BC * kXS * 2;
  static constexpr size_t oH1T = oH1 + (size_t)BC * H1S * 2;
  static constexpr size_t oH2 = oH1T + (size_t)L1 * TS * 2;
  static constexpr size_t oH2T = oH2 + (size_t)BC * H2S * 2;
  static constexpr size_t oR = oH2T + (size_t)L2 * TS * 2;
  // region R is time-shared: layer-1 split-K accumulator -> logits -> dH2^T, dH1^T
  static constexpr size_t szR =
      cmax(cmax((size_t)(L2 + L1) * TS * 2, (size_t)BC * L1 * 4), (size_t)BC * 16 * 4);
  static constexpr size_t odH2T = oR;
  static constexpr size_t odH1T = oR + (size_t)L2 * TS * 2;
  static constexpr size_t odZ = oR + ((szR + 15) / 16) * 16;
  static constexpr size_t odZT = odZ + (size_t)BC * kDZS * 2;
  static constexpr size_t oY = odZT + (size_t)16 * TS * 2;
  static constexpr size_t oMisc = oY + (size_t)BC * 4;
  static constexpr size_t total = oMisc + 64;
  static_assert(L1 % 32 == 0 && L2 % 32 == 0 && L1 <= 128 && L2 <= 256, "layer widths");
  static_assert(BC == 32 || BC == 64, "row chunk");
};

struct Smem {
  __bf16 *X, *H1, *H1T, *H2, *H2T, *dH2T, *dH1T, *dZ, *dZT;
  float *acc1, *Z, *misc;
  int* ys;
  int64_t* stamps;  // diagnostic phase timestamps (s_memrealtime, 100 MHz) or null
};

// Phase stamps for the diagnostic build path: thread 0, right after a barrier.
#define RLA_STAMP(s, k)                                                        \
  do {                                                                         \
    if ((s).stamps && threadIdx.x == 0) (s).stamps[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

template <class C>
__device__ __forceinline__ Smem carve(char* smem) {
  Smem s;
  s.X = (__bf16*)(smem + C::oX);
  s.H1 = (__bf16*)(smem + C::oH1);
  s.H1T = (__bf16*)(smem + C::oH1T);
  s.H2 = (__bf16*)(smem + C::oH2);
  s.H2T = (__bf16*)(smem + C::oH2T);
  s.dH2T = (__bf16*)(smem + C::odH2T);
  s.dH1T = (__bf16*)(smem + C::odH1T);
  s.acc1 = (float*)(smem + C::oR);
  s.Z = (float*)(smem + C::oR);
  s.dZ = (__bf16*)(smem + C::odZ);
  s.dZT = (__bf16*)(smem + C::odZT);
  s.ys = (int*)(smem + C::oY);
  s.misc = (float*)(smem + C::oMisc);
  s.stamps = nullptr;
  return s;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ bf16x8 lds8(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// Transposed 4x16 read (ds_read_b64_tr_b16): lane i of each 16-lane group gets
// column i of the 4 rows whose addresses lanes 4q+p supply (row q, cols 4p..4p+3).
// (The v4bf16 form is used directly: element-wise bit casts out of the v4i16 form
// were mis-lowered by hipcc 7.2 into duplicated dwords.)
__device__ __forceinline__ bf16x4 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}

// -------------------------------------------------------------------------
// Phase: stage the batch chunk's rows into LDS as bf16 (u8 pixels / 255, or
// fp32 features), zero the K padding, fetch labels.
// -------------------------------------------------------------------------
template <int BC, int L1, bool U8>
__device__ __forceinline__ void stage_inputs(const Smem& s, const uint8_t* x_u8, const float* x_f32,
                                             const int64_t* labels, const int64_t* idx, int row0,
                                             int nvalid) {
  const int tid = threadIdx.x;
  for (int i = tid; i < BC * L1; i += kThreads) s.acc1[i] = 0.f;
  if constexpr (U8) {
    constexpr int CPR = kD / 16;  // 49 x 16-byte chunks per row
    for (int t = tid; t < BC * CPR; t += kThreads) {
      const int r = t / CPR, cc = t - r * CPR;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (r < nvalid) {
        const int64_t src = idx[row0 + r];
        v = *reinterpret_cast<const uint4*>(x_u8 + src * kD + cc * 16);
      }
      const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
      bf16x8 lo, hi;
      constexpr float inv255 = 1.0f / 255.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        lo[j] = (__bf16)((float)((wds[0] >> (8 * j)) & 0xffu) * inv255);
        lo[4 + j] = (__bf16)((float)((wds[1] >> (8 * j)) & 0xffu) * inv255);
        hi[j] = (__bf16)((float)((wds[2] >> (8 * j)) & 0xffu) * inv255);
        hi[4 + j] = (__bf16)((float)((wds[3] >> (8 * j)) & 0xffu) * inv255);
      }
      __bf16* dst = s.X + r * kXS + cc * 16;
      *reinterpret_cast<bf16x8*>(dst) = lo;
      *reinterpret_cast<bf16x8*>(dst + 8) = hi;
    }
  } else {
    constexpr int CPR = kD / 8;  // 98 x 32-byte chunks per row
    for (int t = tid; t < BC * CPR; t += kThreads) {
      const int r = t / CPR, cc = t - r * CPR;
      bf16x8 v = zero8();
      if (r < nvalid) {
        const float* src = x_f32 + (int64_t)(row0 + r) * kD + cc * 8;
        v = cvt8(ld4(src), ld4(src + 4));
      }
      *reinterpret_cast<bf16x8*>(s.X + r * kXS + cc * 8) = v;
    }
  }
  for (int t = tid; t < BC * 3; t += kThreads) {
    const int r = t / 3, j = t - r * 3;
    *reinterpret_cast<bf16x8*>(s.X + r * kXS + kD + j * 8) = zero8();
  }
  if (tid < BC) {
    int y = -1;
    if (tid < nvalid) y = (int)(U8 ? labels[idx[row0 + tid]] : labels[row0 + tid]);
    s.ys[tid] = y;
  }
}

// -------------------------------------------------------------------------
// Forward: H1 = relu(X W1^T + b1), H2 = relu(H1 W2^T + b2), Z = H2 W3^T + b3
// -------------------------------------------------------------------------
template <int BC, int L1, int L2>
__device__ __forceinline__ void forward(const Smem& s, const float* P) {
  using C = Cfg<BC, L1, L2>;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const float* W1 = P;
  const float* b1 = W1 + L1 * kD;
  const float* W2 = b1 + L1;
  const float* b2 = W2 + L2 * L1;
  const float* W3 = b2 + L2;
  const float* b3 = W3 + kNC * L2;

  // ---- layer 1: each wave owns one 16-column tile and a K range (split-K) ----
  {
    constexpr int NSPLIT = kWaves / C::TN1;
    const int ct = w % C::TN1, sp = w / C::TN1;
    const int ks0 = sp * kKS1 / NSPLIT, ks1 = (sp + 1) * kKS1 / NSPLIT;
    f32x4 acc[C::MT];
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* wrow = W1 + (ct * 16 + r16) * kD;
    float4 nlo = make_float4(0.f, 0.f, 0.f, 0.f), nhi = nlo;
    {
      const int k = ks0 * 32 + 8 * g;
      if (k < kD) { nlo = ld4(wrow + k); nhi = ld4(wrow + k + 4); }
    }
    for (int ks = ks0; ks < ks1; ++ks) {
      const float4 clo = nlo, chi = nhi;
      const int kn = (ks + 1) * 32 + 8 * g;
      if (ks + 1 < ks1) {
        if (kn < kD) { nlo = ld4(wrow + kn); nhi = ld4(wrow + kn + 4); }
        else { nlo = make_float4(0.f, 0.f, 0.f, 0.f); nhi = nlo; }
      }
      const bf16x8 bfrag = cvt8(clo, chi);
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) {
        const bf16x8 afrag = lds8(s.X + (mt * 16 + r16) * kXS + ks * 32 + 8 * g);
        acc[mt] = mfma16(afrag, bfrag, acc[mt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* dst = s.acc1 + (mt * 16 + 4 * g + i) * L1 + ct * 16 + r16;
        if constexpr (NSPLIT == 1) *dst = acc[mt][i];
        else atomicAdd(dst, acc[mt][i]);
      }
  }
  __syncthreads();
  RLA_STAMP(s, 2);
  for (int e = tid; e < BC * L1; e += kThreads) {
    const int b = e / L1, j = e - b * L1;
    const __bf16 h = (__bf16)fmaxf(s.acc1[e] + b1[j], 0.f);
    s.H1[b * C::H1S + j] = h;
    s.H1T[j * C::TS + b] = h;
  }
  __syncthreads();
  RLA_STAMP(s, 3);

  // ---- layer 2 ----
  for (int tile = w; tile < C::MT * C::TN2; tile += kWaves) {
    const int mt = tile % C::MT, nt = tile / C::MT;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wrow = W2 + (nt * 16 + r16) * L1;
#pragma unroll
    for (int ks = 0; ks < L1 / 32; ++ks) {
      const int k = ks * 32 + 8 * g;
      const bf16x8 bfrag = cvt8(ld4(wrow + k), ld4(wrow + k + 4));
      const bf16x8 afrag = lds8(s.H1 + (mt * 16 + r16) * C::H1S + k);
      acc = mfma16(afrag, bfrag, acc);
    }
    const int n = nt * 16 + r16;
    const float bias = b2[n];
    bf16x4 t4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const __bf16 h = (__bf16)fmaxf(acc[i] + bias, 0.f);
      s.H2[(mt * 16 + 4 * g + i) * C::H2S + n] = h;
      t4[i] = h;
    }
    *reinterpret_cast<bf16x4*>(s.H2T + n * C::TS + mt * 16 + 4 * g) = t4;
  }
  __syncthreads();
  RLA_STAMP(s, 4);

  // ---- layer 3 (logits, classes padded to 16) ----
  if (w < C::MT) {
    const int mt = w;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < L2 / 32; ++ks) {
      const int k = ks * 32 + 8 * g;
      bf16x8 bfrag = zero8();
      if (r16 < kNC) bfrag = cvt8(ld4(W3 + r16 * L2 + k), ld4(W3 + r16 * L2 + k + 4));
      const bf16x8 afrag = lds8(s.H2 + (mt * 16 + r16) * C::H2S + k);
      acc = mfma16(afrag, bfrag, acc);
    }
    if (r16 < kNC) {
      const float bias = b3[r16];
#pragma unroll
      for (int i = 0; i < 4; ++i) s.Z[(mt * 16 + 4 * g + i) * 16 + r16] = acc[i] + bias;
    }
  }
  __syncthreads();
  RLA_STAMP(s, 5);
}

// log_softmax + NLL + argmax for one row; returns false for padded rows.
__device__ __forceinline__ bool row_softmax(const float* zrow, int y, float* prob, float& loss,
                                            int& correct, float& lse_out) {
  if (y < 0) return false;
  float z[kNC];
  float m = -INFINITY;
  int arg = 0;
#pragma unroll
  for (int j = 0; j < kNC; ++j) {
    z[j] = zrow[j];
    if (z[j] > m) { m = z[j]; arg = j; }
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < kNC; ++j) {
    prob[j] = expf(z[j] - m);
    sum += prob[j];
  }
  const float inv = 1.f / sum;
#pragma unroll
  for (int j = 0; j < kNC; ++j) prob[j] *= inv;
  const float lse = m + logf(sum);
  lse_out = lse;
  loss = lse - z[y];
  correct = (arg == y) ? 1 : 0;
  return true;
}

struct AdamScal {
  float lr, step_size, bc2_sqrt, beta1, beta2, eps, wd;
  int adamw;
};

__device__ __forceinline__ float adam1(float p, float g, float& m, float& v, const AdamScal& o) {
  if (o.wd != 0.f) {
    if (o.adamw) p = p * (1.f - o.lr * o.wd);
    else g = g + o.wd * p;
  }
  m = m + (1.f - o.beta1) * (g - m);
  v = v * o.beta2 + (1.f - o.beta2) * (g * g);
  const float denom = sqrtf(v) / o.bc2_sqrt + o.eps;
  return p + (-o.step_size) * (m / denom);
}

struct GradSink {
  float *P, *G, *M, *V;
  bool accum, adam;
  AdamScal o;
  __device__ __forceinline__ void put1(int64_t i, float g) const {
    if (accum) g += G[i];
    if (adam) {
      float m = M[i], v = V[i];
      P[i] = adam1(P[i], g, m, v, o);
      M[i] = m; V[i] = v;
    } else {
      G[i] = g;
    }
  }
  __device__ __forceinline__ void put4(int64_t i, f32x4 acc) const {
    F4 g{{acc[0], acc[1], acc[2], acc[3]}};
    if (accum) {
      const F4 o4 = *reinterpret_cast<const F4*>(G + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) g.v[k] += o4.v[k];
    }
    if (adam) {
      F4 p = *reinterpret_cast<const F4*>(P + i), m = *reinterpret_cast<const F4*>(M + i),
         v = *reinterpret_cast<const F4*>(V + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) p.v[k] = adam1(p.v[k], g.v[k], m.v[k], v.v[k], o);
      *reinterpret_cast<F4*>(P + i) = p;
      *reinterpret_cast<F4*>(M + i) = m;
      *reinterpret_cast<F4*>(V + i) = v;
    } else {
      *reinterpret_cast<F4*>(G + i) = g;
    }
  }
};

// -------------------------------------------------------------------------
// Backward for one chunk.  invB = 1 / full batch size (mean NLL).
// -------------------------------------------------------------------------
template <int BC, int L1, int L2>
__device__ __forceinline__ void backward(const Smem& s, const GradSink& sink, float invB) {
  using C = Cfg<BC, L1, L2>;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const float* P = sink.P;
  const float* W2 = P + L1 * kD + L1;
  const float* W3 = W2 + L2 * L1 + L2;
  const int64_t offB1 = (int64_t)L1 * kD, offW2 = offB1 + L1, offB2 = offW2 + L2 * L1,
                offW3 = offB2 + L2, offB3 = offW3 + kNC * L2;

  // ---- softmax / NLL / dZ: one thread per row ----
  if (tid < BC) {
    const int r = tid;
    float prob[kNC], loss = 0.f, lse = 0.f;
    int correct = 0;
    const int y = s.ys[r];
    bf16x8 d8[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) d8[q] = zero8();
    if (row_softmax(s.Z + r * 16, y, prob, loss, correct, lse)) {
      atomicAdd(&s.misc[0], loss);
      atomicAdd(&s.misc[1], (float)correct);
      atomicAdd(&s.misc[2], 1.f);
#pragma unroll
      for (int j = 0; j < kNC; ++j) {
        const float d = (prob[j] - (j == y ? 1.f : 0.f)) * invB;
        d8[j >> 3][j & 7] = (__bf16)d;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(s.dZ + r * kDZS + 8 * q) = d8[q];
#pragma unroll
    for (int j = 0; j < 16; ++j) s.dZT[j * C::TS + r] = (j < kNC) ? d8[j >> 3][j & 7] : (__bf16)0.f;
  }
  __syncthreads();
  RLA_STAMP(s, 6);

  // ---- dH2 = (dZ W3) * (H2 > 0); written in place of H2 and transposed ----
  for (int tile = w; tile < C::MT * C::TN2; tile += kWaves) {
    const int mt = tile % C::MT, nt = tile / C::MT, n = nt * 16 + r16;
    const bf16x8 afrag = lds8(s.dZ + (mt * 16 + r16) * kDZS + 8 * g);
    bf16x8 bfrag = zero8();
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = 8 * g + jj;
      if (j < kNC) bfrag[jj] = (__bf16)W3[j * L2 + n];
    }
    const f32x4 acc = mfma16(afrag, bfrag, f32x4{0.f, 0.f, 0.f, 0.f});
    bf16x4 t4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __bf16* hp = s.H2 + (mt * 16 + 4 * g + i) * C::H2S + n;
      const __bf16 d = ((float)(*hp) > 0.f) ? (__bf16)acc[i] : (__bf16)0.f;
      *hp = d;
      t4[i] = d;
    }
    *reinterpret_cast<bf16x4*>(s.dH2T + n * C::TS + mt * 16 + 4 * g) = t4;
  }
  __syncthreads();
  RLA_STAMP(s, 7);

  // ---- dH1 = (dH2 W2) * (H1 > 0), stored transposed ----
  for (int tile = w; tile < C::MT * C::TN1; tile += kWaves) {
    const int mt = tile % C::MT, ct = tile / C::MT, m = ct * 16 + r16;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < L2 / 32; ++ks) {
      const int k = ks * 32 + 8 * g;
      const bf16x8 afrag = lds8(s.H2 + (mt * 16 + r16) * C::H2S + k);
      bf16x8 bfrag;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) bfrag[jj] = (__bf16)W2[(k + jj) * L1 + m];
      acc = mfma16(afrag, bfrag, acc);
    }
    bf16x4 t4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const __bf16 hv = s.H1[(mt * 16 + 4 * g + i) * C::H1S + m];
      t4[i] = ((float)hv > 0.f) ? (__bf16)acc[i] : (__bf16)0.f;
    }
    *reinterpret_cast<bf16x4*>(s.dH1T + m * C::TS + mt * 16 + 4 * g) = t4;
  }
  __syncthreads();
  RLA_STAMP(s, 8);

  // ---- weight gradients (+ fused Adam): dW1 tiles, dW2 tiles, dW3 tiles ----
  constexpr int NT_W1 = (kD / 16) * C::TN1;
  constexpr int NT_W2 = C::TN2 * C::TN1;
  constexpr int NT_W3 = C::TN2;
  for (int task = w; task < NT_W1 + NT_W2 + NT_W3; task += kWaves) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (task < NT_W1) {
      // dW1^T[pix][m] = sum_b X[b][pix] dH1[b][m]
      const int kt = task % (kD / 16), ct = task / (kD / 16);
      const int q = r16 >> 2, p = r16 & 3;
#pragma unroll
      for (int ks = 0; ks < BC / 32; ++ks) {
        const int b0 = ks * 32 + 8 * g;
        const bf16x4 lo = tr_read(s.X + (b0 + q) * kXS + kt * 16 + 4 * p);
        const bf16x4 hi = tr_read(s.X + (b0 + 4 + q) * kXS + kt * 16 + 4 * p);
        const bf16x8 afrag = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        const bf16x8 bfrag = lds8(s.dH1T + (ct * 16 + r16) * C::TS + b0);
        acc = mfma16(afrag, bfrag, acc);
      }
      const int m = ct * 16 + r16, pix = kt * 16 + 4 * g;
      sink.put4((int64_t)m * kD + pix, acc);
    } else if (task < NT_W1 + NT_W2) {
      // dW2[n][m] = sum_b dH2[b][n] H1[b][m]
      const int t2 = task - NT_W1;
      const int nt = t2 % C::TN2, ct = t2 / C::TN2;
#pragma unroll
      for (int ks = 0; ks < BC / 32; ++ks) {
        const int b0 = ks * 32 + 8 * g;
        const bf16x8 afrag = lds8(s.dH2T + (nt * 16 + r16) * C::TS + b0);
        const bf16x8 bfrag = lds8(s.H1T + (ct * 16 + r16) * C::TS + b0);
        acc = mfma16(afrag, bfrag, acc);
      }
      const int m = ct * 16 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) sink.put1(offW2 + (int64_t)(nt * 16 + 4 * g + i) * L1 + m, acc[i]);
    } else {
      // dW3[j][n] = sum_b dZ[b][j] H2[b][n]
      const int nt = task - NT_W1 - NT_W2;
#pragma unroll
      for (int ks = 0; ks < BC / 32; ++ks) {
        const int b0 = ks * 32 + 8 * g;
        const bf16x8 afrag = lds8(s.dZT + r16 * C::TS + b0);
        const bf16x8 bfrag = lds8(s.H2T + (nt * 16 + r16) * C::TS + b0);
        acc = mfma16(afrag, bfrag, acc);
      }
      const int n = nt * 16 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = 4 * g + i;
        if (j < kNC) sink.put1(offW3 + (int64_t)j * L2 + n, acc[i]);
      }
    }
  }
  // ---- bias gradients: column sums of dH1, dH2, dZ over the chunk ----
  for (int e = tid; e < L1 + L2 + kNC; e += kThreads) {
    const __bf16* row;
    int64_t gi;
    if (e < L1) { row = s.dH1T + e * C::TS; gi = offB1 + e; }
    else if (e < L1 + L2) { row = s.dH2T + (e - L1) * C::TS; gi = offB2 + (e - L1); }
    else { row = s.dZT + (e - L1 - L2) * C::TS; gi = offB3 + (e - L1 - L2); }
    float sum = 0.f;
#pragma unroll 8
    for (int b = 0; b < BC; ++b) sum += (float)row[b];
    sink.put1(gi, sum);
  }
  __syncthreads();
  RLA_STAMP(s, 9);
}

template <int BC, int L1, int L2, bool U8>
__global__ __launch_bounds__(kThreads) void mlp_train_kernel(MLPStepArgs a) {
  using C = Cfg<BC, L1, L2>;
  __shared__ __attribute__((aligned(16))) char smem[C::total];
  Smem s = carve<C>(smem);
  s.stamps = a.stamps;
  __shared__ int64_t sh_t, sh_cursor;
  __shared__ AdamScal sh_o;
  if (threadIdx.x == 0) {
    const int64_t t = (a.counters ? a.counters[0] : 0) + 1;
    sh_t = t;
    sh_cursor = (U8 && a.counters) ? a.counters[1] : 0;
    const float lr = a.lr_ptr ? a.lr_ptr[0] : a.lr;
    const double bc1 = 1.0 - pow((double)a.beta1, (double)t);
    const double bc2 = 1.0 - pow((double)a.beta2, (double)t);
    sh_o.lr = lr;
    sh_o.step_size = (float)((double)lr / bc1);
    sh_o.bc2_sqrt = (float)sqrt(bc2);
    sh_o.beta1 = a.beta1; sh_o.beta2 = a.beta2; sh_o.eps = a.eps; sh_o.wd = a.weight_decay;
    sh_o.adamw = a.adamw;
    s.misc[0] = 0.f; s.misc[1] = 0.f; s.misc[2] = 0.f;
  }
  __syncthreads();
  RLA_STAMP(s, 0);
  const int64_t* idx = U8 ? a.order + sh_cursor * a.B : nullptr;
  const float invB = 1.f / (float)a.B;
  const int nchunks = (a.B + BC - 1) / BC;
  for (int c = 0; c < nchunks; ++c) {
    const int row0 = c * BC;
    const int nvalid = min(BC, a.B - row0);
    stage_inputs<BC, L1, U8>(s, a.x_u8, a.x_f32, a.labels, idx, row0, nvalid);
    __syncthreads();
    RLA_STAMP(s, 1);
    forward<BC, L1, L2>(s, a.params);
    GradSink sink;
    sink.P = a.params; sink.G = a.grads; sink.M = a.exp_avg; sink.V = a.exp_avg_sq;
    sink.accum = a.accumulate_grad || c > 0;
    sink.adam = a.apply_adam && (c == nchunks - 1);
    sink.o = sh_o;
    backward<BC, L1, L2>(s, sink, invB);
  }
  RLA_STAMP(s, 10);
  if (threadIdx.x == 0) {
    const int64_t t = sh_t;
    if (a.counters) {
      if (a.advance_step) a.counters[0] = t;
      if (U8) a.counters[1] = (a.n_batches > 0) ? (sh_cursor + 1) % a.n_batches : sh_cursor + 1;
    }
    if (a.stats) {
      const int slot = (int)((t - 1) % (a.stats_ring > 0 ? a.stats_ring : 1));
      float* st = a.stats + slot * 4;
      st[0] = s.misc[0] * invB;
      st[1] = s.misc[1];
      st[2] = s.misc[2];
      st[3] = (float)t;
    }
  }
}

// Forward-only evaluation (validation / test): one 32-row chunk per workgroup,
// the chunks spread over the grid (a 5,000-sample validation split is ~160
// workgroups, one wave of the chip).  ``partials`` mode writes each chunk's
// (sum NLL, #correct) to out[2c..2c+1] -- no atomics, so the epoch's sums are
// reduced deterministically by the caller; otherwise one atomic pair per block.
template <int BC, int L1, int L2, bool U8>
__global__ __launch_bounds__(kThreads) void mlp_eval_kernel(MLPEvalArgs a) {
  using C = Cfg<BC, L1, L2>;
  __shared__ __attribute__((aligned(16))) char smem[C::total];
  const Smem s = carve<C>(smem);
  const int nchunks = (a.B + BC - 1) / BC;
  float loss_sum = 0.f, correct_sum = 0.f;
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int row0 = c * BC;
    const int nvalid = min(BC, a.B - row0);
    stage_inputs<BC, L1, U8>(s, a.x_u8, a.x_f32, a.labels, a.index, row0, nvalid);
    __syncthreads();
    forward<BC, L1, L2>(s, a.params);
    float l = 0.f, k = 0.f;
    if (threadIdx.x < BC) {
      const int r = threadIdx.x;
      float prob[kNC], loss, lse;
      int correct;
      if (row_softmax(s.Z + r * 16, s.ys[r], prob, loss, correct, lse)) {
        l = loss;
        k = (float)correct;
        if (a.logits)
          for (int j = 0; j < kNC; ++j) a.logits[(int64_t)(row0 + r) * kNC + j] = s.Z[r * 16 + j] - lse;
      }
    }
    if (threadIdx.x < 64) {  // wave 0 (BC <= 64 rows): full-wave reduction, every lane active
      for (int off = 32; off > 0; off >>= 1) {
        l += __shfl_down(l, off, 64);
        k += __shfl_down(k, off, 64);
      }
      if (threadIdx.x == 0) {
        if (a.partials) {
          a.out[2 * c] = l;
          a.out[2 * c + 1] = k;
        } else {
          loss_sum += l;
          correct_sum += k;
        }
      }
    }
    __syncthreads();
  }
  if (!a.partials && threadIdx.x == 0 && blockIdx.x < nchunks) {
    atomicAdd(&a.out[0], loss_sum);
    atomicAdd(&a.out[1], correct_sum);
  }
}

template <int BC, int L1, int L2>
constexpr bool fits() {
  return Cfg<BC, L1, L2>::total + 256 <= 160 * 1024;
}

template <int L1, int L2>
int dispatch_train(const MLPStepArgs& a, hipStream_t stream) {
  const bool u8 = a.x_u8 != nullptr;
  const bool big = a.B > 32;
  if constexpr (fits<64, L1, L2>()) {
    if (big) {
      if (u8) hipLaunchKernelGGL((mlp_train_kernel<64, L1, L2, true>), dim3(1), dim3(kThreads), 0, stream, a);
      else hipLaunchKernelGGL((mlp_train_kernel<64, L1, L2, false>), dim3(1), dim3(kThreads), 0, stream, a);
      return 0;
    }
  }
  if (u8) hipLaunchKernelGGL((mlp_train_kernel<32, L1, L2, true>), dim3(1), dim3(kThreads), 0, stream, a);
  else hipLaunchKernelGGL((mlp_train_kernel<32, L1, L2, false>), dim3(1), dim3(kThreads), 0, stream, a);
  return 0;
}

template <int L1, int L2>
int dispatch_eval(const MLPEvalArgs& a, hipStream_t stream) {
  const bool u8 = a.x_u8 != nullptr;
  const int nchunks = (a.B + 31) / 32;
  // partials: one block per chunk (every chunk owns its output pair); atomics: a
  // grid-stride over at most one block per CU
  const int grid = a.partials ? nchunks : (nchunks < 256 ? nchunks : 256);
  if (u8) hipLaunchKernelGGL((mlp_eval_kernel<32, L1, L2, true>), dim3(grid), dim3(kThreads), 0, stream, a);
  else hipLaunchKernelGGL((mlp_eval_kernel<32, L1, L2, false>), dim3(grid), dim3(kThreads), 0, stream, a);
  return 0;
}

#define RLA_MLP_SHAPES(X) \
  X(32, 32) X(32, 64) X(32, 128) X(32, 256) \
  X(64, 64) X(64, 128) X(64, 256) \
  X(128, 128) X(128, 256) X(128, 64)

}  // namespace

bool mlp_supported(int L1, int L2) {
#define RLA_CASE(a1, a2) if (L1 == a1 && L2 == a2) return true;
  RLA_MLP_SHAPES(RLA_CASE)
#undef RLA_CASE
  return false;
}

int launch_mlp_train_step(const MLPStepArgs& a, hipStream_t stream) {
#define RLA_CASE(a1, a2) if (a.L1 == a1 && a.L2 == a2) return dispatch_train<a1, a2>(a, stream);
  RLA_MLP_SHAPES(RLA_CASE)
#undef RLA_CASE
  return -1;
}

int launch_mlp_eval(const MLPEvalArgs& a, hipStream_t stream) {
  if (a.B <= 0) return 0;
#define RLA_CASE(a1, a2) if (a.L1 == a1 && a.L2 == a2) return dispatch_eval<a1, a2>(a, stream);
  RLA_MLP_SHAPES(RLA_CASE)
#undef RLA_CASE
  return -1;
}

}  // namespace rla
