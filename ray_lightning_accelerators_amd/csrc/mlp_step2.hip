// Fused MNIST-MLP training step, v2: two launches per step, bf16 weight shadows.
//
// Measured on MI355X (profiles/r1_first/mlp_phases_v1.json), the one-workgroup
// v1 step spent its 30 us almost entirely in serialized global round trips:
// 7 us streaming W1 (fp32) with a 1-deep prefetch, 15 us in the dW1 + Adam
// epilogue (one CU reading/writing 500 KB of Adam state tile by tile) and
// 2.7 us in an LDS-atomic softmax.  v2 re-partitions the step by where its
// bytes live:
//
//   head kernel   (1 workgroup, 8 waves)  forward, log_softmax/NLL/accuracy,
//                 dH2, dH1, dW2/dW3/bias grads + Adam for those (2.7 K params),
//                 hands dH1^T (bf16, <= 8 KB) to the W1 kernel through HBM;
//   W1 kernel     (49 workgroups, one per 16-pixel tile)  dW1 tile by MFMA
//                 (X^T by ds_read_b64_tr_b16 from an LDS slice it gathers
//                 itself) + Adam on its 16 x L1 weights -- the 25 K-parameter
//                 optimizer traffic spread over 49 CUs instead of one.
//
// Weights are read as bf16 from a shadow buffer the optimizer epilogues keep
// current (row-major copy, plus W2^T and W3^T so the backward's B operands are
// 16-byte loads too); every weight fragment a wave needs is issued at kernel
// start so its latency hides under the X gather.  fp32 master weights and Adam
// state stay authoritative.
#include "common.h"
#include "kernels.h"
#include "mlp_common.h"

namespace rla {

MLPShadowLayout mlp_shadow_layout(int L1, int L2) {
  MLPShadowLayout s;
  s.np = (int64_t)L1 * 784 + L1 + (int64_t)L2 * L1 + L2 + 10 * (int64_t)L2 + 10;
  s.w2t = (s.np + 7) / 8 * 8;
  s.w3t = s.w2t + (int64_t)L1 * L2;
  s.total = s.w3t + 16 * (int64_t)L2;
  return s;
}

namespace {

using namespace mlp;

constexpr int kKS1 = 25;
constexpr int kXS = 808;
constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kDZS = 40;

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
  static constexpr size_t szR =
      cmax(cmax((size_t)(L2 + L1) * TS * 2, (size_t)BC * L1 * 4), (size_t)BC * 16 * 4);
  static constexpr size_t odH2T = oR;
  static constexpr size_t odH1T = oR + (size_t)L2 * TS * 2;
  static constexpr size_t odZ = oR + ((szR + 15) / 16) * 16;
  static constexpr size_t odZT = odZ + (size_t)BC * kDZS * 2;
  static constexpr size_t oY = odZT + (size_t)16 * TS * 2;
  static constexpr size_t oMisc = oY + (size_t)BC * 4;
  static constexpr size_t total = oMisc + 64;
};

// ---------------------------------------------------------------------------
// Head kernel
// ---------------------------------------------------------------------------
template <int BC, int L1, int L2, bool U8>
__global__ __launch_bounds__(kThreads) void mlp_head_kernel(MLPStepArgs a) {
  using C = Cfg<BC, L1, L2>;
  using O = Off<L1, L2>;
  __shared__ __attribute__((aligned(16))) char smem[C::total];
  __bf16* sX = (__bf16*)(smem + C::oX);
  __bf16* sH1 = (__bf16*)(smem + C::oH1);
  __bf16* sH1T = (__bf16*)(smem + C::oH1T);
  __bf16* sH2 = (__bf16*)(smem + C::oH2);
  __bf16* sH2T = (__bf16*)(smem + C::oH2T);
  __bf16* sdH2T = (__bf16*)(smem + C::odH2T);
  __bf16* sdH1T = (__bf16*)(smem + C::odH1T);
  float* sAcc = (float*)(smem + C::oR);
  float* sZ = (float*)(smem + C::oR);
  __bf16* sdZ = (__bf16*)(smem + C::odZ);
  __bf16* sdZT = (__bf16*)(smem + C::odZT);
  int* sY = (int*)(smem + C::oY);
  float* misc = (float*)(smem + C::oMisc);
  __shared__ int64_t sh_t, sh_cursor;
  __shared__ AdamScal sh_o;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const __bf16* SH = reinterpret_cast<const __bf16*>(a.shadow);
  __bf16* SHW = reinterpret_cast<__bf16*>(a.shadow);
  const float* P = a.params;

  if (tid == 0) {
    const int64_t t = a.counters[0] + 1;
    sh_t = t;
    sh_cursor = U8 ? a.counters[1] : 0;
    adam_scalars(sh_o, t, a.lr_ptr ? a.lr_ptr[0] : a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.adamw);
    misc[0] = 0.f; misc[1] = 0.f; misc[2] = 0.f;
    if (a.stamps) a.stamps[0] = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  const int64_t* idx = U8 ? a.order + sh_cursor * a.B : nullptr;
  const float invB = 1.f / (float)a.B;
  const int Bp = (a.B + 31) / 32 * 32;
  const int nchunks = (a.B + BC - 1) / BC;

  constexpr int NSPLIT = kWaves / C::TN1;
  constexpr int KMAX = (kKS1 + NSPLIT - 1) / NSPLIT;
  constexpr int D = KMAX < 13 ? KMAX : 13;
  constexpr int KS2 = L1 / 32, KS3 = L2 / 32, KSH = L2 / 32;
  constexpr int P3 = KS3 < 4 ? KS3 : 4;
  constexpr int PH = KSH < 4 ? KSH : 4;

  for (int c = 0; c < nchunks; ++c) {
    const int row0 = c * BC;
    const int nvalid = min(BC, a.B - row0);
    const bool accum = a.accumulate_grad || c > 0;
    const bool adam = a.apply_adam && (c == nchunks - 1);

    // ---------------- prefetch weight fragments (batch independent) ----------------
    const int ct1 = w % C::TN1, sp = w / C::TN1;
    const int ks0 = sp * kKS1 / NSPLIT, ks1 = (sp + 1) * kKS1 / NSPLIT;
    const __bf16* w1row = SH + O::W1 + (int64_t)(ct1 * 16 + r16) * kD;
    bf16x8 wf[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int k = (ks0 + j) * 32 + 8 * g;
      wf[j] = (ks0 + j < ks1 && k < kD) ? ld8(w1row + k) : zero8();
    }
    bf16x8 w2f[KS2];
    {
      const int tile = w;  // first layer-2 tile of this wave
      const int nt = tile / C::MT;
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks)
        w2f[ks] = (tile < C::MT * C::TN2) ? ld8(SH + O::W2 + (int64_t)(nt * 16 + r16) * L1 + ks * 32 + 8 * g)
                                          : zero8();
    }
    bf16x8 w3f[P3];
#pragma unroll
    for (int ks = 0; ks < P3; ++ks)
      w3f[ks] = (w < C::MT && r16 < kNC) ? ld8(SH + O::W3 + (int64_t)r16 * L2 + ks * 32 + 8 * g) : zero8();
    bf16x8 w3tf;
    {
      const int nt = w / C::MT;
      w3tf = (w < C::MT * C::TN2 && g < 2) ? ld8(SH + O::W3T + (int64_t)(nt * 16 + r16) * 16 + 8 * g) : zero8();
    }
    bf16x8 w2tf[PH];
    {
      const int ct = w / C::MT;
#pragma unroll
      for (int ks = 0; ks < PH; ++ks)
        w2tf[ks] = (w < C::MT * C::TN1) ? ld8(SH + O::W2T + (int64_t)(ct * 16 + r16) * L2 + ks * 32 + 8 * g)
                                         : zero8();
    }

    // ---------------- stage the batch chunk into LDS ----------------
    for (int i = tid; i < BC * L1; i += kThreads) sAcc[i] = 0.f;
    if constexpr (U8) {
      constexpr int CPR = kD / 16;
      for (int t = tid; t < BC * CPR; t += kThreads) {
        const int r = t / CPR, cc = t - r * CPR;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (r < nvalid) v = *reinterpret_cast<const uint4*>(a.x_u8 + idx[row0 + r] * kD + cc * 16);
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        bf16x8 lo, hi;
        constexpr float inv255 = 1.0f / 255.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          lo[j] = (__bf16)((float)((wd[0] >> (8 * j)) & 0xffu) * inv255);
          lo[4 + j] = (__bf16)((float)((wd[1] >> (8 * j)) & 0xffu) * inv255);
          hi[j] = (__bf16)((float)((wd[2] >> (8 * j)) & 0xffu) * inv255);
          hi[4 + j] = (__bf16)((float)((wd[3] >> (8 * j)) & 0xffu) * inv255);
        }
        __bf16* dst = sX + r * kXS + cc * 16;
        *reinterpret_cast<bf16x8*>(dst) = lo;
        *reinterpret_cast<bf16x8*>(dst + 8) = hi;
      }
    } else {
      constexpr int CPR = kD / 8;
      for (int t = tid; t < BC * CPR; t += kThreads) {
        const int r = t / CPR, cc = t - r * CPR;
        bf16x8 v = zero8();
        if (r < nvalid) {
          const float* src = a.x_f32 + (int64_t)(row0 + r) * kD + cc * 8;
          v = cvt8(ld4(src), ld4(src + 4));
        }
        *reinterpret_cast<bf16x8*>(sX + r * kXS + cc * 8) = v;
      }
    }
    for (int t = tid; t < BC * 3; t += kThreads) {
      const int r = t / 3, j = t - r * 3;
      *reinterpret_cast<bf16x8*>(sX + r * kXS + kD + j * 8) = zero8();
    }
    if (tid < BC) {
      int y = -1;
      if (tid < nvalid) y = (int)(U8 ? a.labels[idx[row0 + tid]] : a.labels[row0 + tid]);
      sY[tid] = y;
    }
    __syncthreads();
    if (a.stamps && tid == 0) a.stamps[1] = __builtin_amdgcn_s_memrealtime();

    // ---------------- layer 1 (split-K over waves, prefetched ring) ----------------
    {
      f32x4 acc[C::MT];
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int base = 0; base < KMAX; base += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
          const int ks = ks0 + base + j;
          if (base + j < KMAX && ks < ks1) {
            const bf16x8 bfrag = wf[j];
            if (base + j + D < KMAX) {
              const int kn = (ks + D) * 32 + 8 * g;
              wf[j] = (ks + D < ks1 && kn < kD) ? ld8(w1row + kn) : zero8();
            }
#pragma unroll
            for (int mt = 0; mt < C::MT; ++mt)
              acc[mt] = mfma16(ld8(sX + (mt * 16 + r16) * kXS + ks * 32 + 8 * g), bfrag, acc[mt]);
          }
        }
      }
#pragma unroll
      for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float* dst = sAcc + (mt * 16 + 4 * g + i) * L1 + ct1 * 16 + r16;
          if constexpr (NSPLIT == 1) *dst = acc[mt][i];
          else atomicAdd(dst, acc[mt][i]);
        }
    }
    __syncthreads();
    for (int e = tid; e < BC * L1; e += kThreads) {
      const int b = e / L1, j = e - b * L1;
      const __bf16 h = (__bf16)fmaxf(sAcc[e] + P[O::B1 + j], 0.f);
      sH1[b * C::H1S + j] = h;
      sH1T[j * C::TS + b] = h;
    }
    __syncthreads();
    if (a.stamps && tid == 0) a.stamps[2] = __builtin_amdgcn_s_memrealtime();

    // ---------------- layer 2 ----------------
    for (int tile = w; tile < C::MT * C::TN2; tile += kWaves) {
      const int mt = tile % C::MT, nt = tile / C::MT;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks) {
        const bf16x8 bfrag = (tile == w) ? w2f[ks] : ld8(SH + O::W2 + (int64_t)(nt * 16 + r16) * L1 + ks * 32 + 8 * g);
        acc = mfma16(ld8(sH1 + (mt * 16 + r16) * C::H1S + ks * 32 + 8 * g), bfrag, acc);
      }
      const int n = nt * 16 + r16;
      const float bias = P[O::B2 + n];
      bf16x4 t4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const __bf16 h = (__bf16)fmaxf(acc[i] + bias, 0.f);
        sH2[(mt * 16 + 4 * g + i) * C::H2S + n] = h;
        t4[i] = h;
      }
      *reinterpret_cast<bf16x4*>(sH2T + n * C::TS + mt * 16 + 4 * g) = t4;
    }
    __syncthreads();

    // ---------------- layer 3 (logits) ----------------
    if (w < C::MT) {
      const int mt = w;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS3; ++ks) {
        bf16x8 bfrag;
        if (ks < P3) bfrag = w3f[ks < P3 ? ks : 0];
        else bfrag = (r16 < kNC) ? ld8(SH + O::W3 + (int64_t)r16 * L2 + ks * 32 + 8 * g) : zero8();
        acc = mfma16(ld8(sH2 + (mt * 16 + r16) * C::H2S + ks * 32 + 8 * g), bfrag, acc);
      }
      if (r16 < kNC) {
        const float bias = P[O::B3 + r16];
#pragma unroll
        for (int i = 0; i < 4; ++i) sZ[(mt * 16 + 4 * g + i) * 16 + r16] = acc[i] + bias;
      }
    }
    __syncthreads();
    if (a.stamps && tid == 0) a.stamps[3] = __builtin_amdgcn_s_memrealtime();

    // ---------------- log_softmax / NLL / accuracy / dZ (wave 0, one row per lane) -------------
    if (w == 0) {
      const int r = lane;
      float loss = 0.f, correct = 0.f, cnt = 0.f;
      bf16x8 d8[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) d8[q] = zero8();
      const int y = (r < BC) ? sY[r] : -1;
      if (y >= 0) {
        float z[kNC];
        float m = -INFINITY;
        int arg = 0;
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
          z[j] = sZ[r * 16 + j];
          if (z[j] > m) { m = z[j]; arg = j; }
        }
        float sum = 0.f, pr[kNC], zy = 0.f;
#pragma unroll
        for (int j = 0; j < kNC; ++j) {
          pr[j] = __expf(z[j] - m);
          sum += pr[j];
          zy = (j == y) ? z[j] : zy;
        }
        const float inv = 1.f / sum;
        loss = m + __logf(sum) - zy;
        correct = (arg == y) ? 1.f : 0.f;
        cnt = 1.f;
#pragma unroll
        for (int j = 0; j < kNC; ++j) d8[j >> 3][j & 7] = (__bf16)((pr[j] * inv - (j == y ? 1.f : 0.f)) * invB);
      }
      if (r < BC) {
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<bf16x8*>(sdZ + r * kDZS + 8 * q) = d8[q];
#pragma unroll
        for (int j = 0; j < 16; ++j) sdZT[j * C::TS + r] = (j < kNC) ? d8[j >> 3][j & 7] : (__bf16)0.f;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        loss += __shfl_xor(loss, off, 64);
        correct += __shfl_xor(correct, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
      }
      if (lane == 0) { misc[0] += loss; misc[1] += correct; misc[2] += cnt; }
    }
    __syncthreads();

    // ---------------- dH2 = (dZ W3) * (H2 > 0) ----------------
    for (int tile = w; tile < C::MT * C::TN2; tile += kWaves) {
      const int mt = tile % C::MT, nt = tile / C::MT, n = nt * 16 + r16;
      const bf16x8 bfrag = (tile == w) ? w3tf
                                       : ((g < 2) ? ld8(SH + O::W3T + (int64_t)n * 16 + 8 * g) : zero8());
      const f32x4 acc = mfma16(ld8(sdZ + (mt * 16 + r16) * kDZS + 8 * g), bfrag, f32x4{0.f, 0.f, 0.f, 0.f});
      bf16x4 t4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __bf16* hp = sH2 + (mt * 16 + 4 * g + i) * C::H2S + n;
        const __bf16 d = ((float)(*hp) > 0.f) ? (__bf16)acc[i] : (__bf16)0.f;
        *hp = d;
        t4[i] = d;
      }
      *reinterpret_cast<bf16x4*>(sdH2T + n * C::TS + mt * 16 + 4 * g) = t4;
    }
    __syncthreads();

    // ---------------- dH1 = (dH2 W2) * (H1 > 0)  -> LDS (for dW2/db1) and HBM (for the W1 kernel) ----
    for (int tile = w; tile < C::MT * C::TN1; tile += kWaves) {
      const int mt = tile % C::MT, ct = tile / C::MT, m = ct * 16 + r16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KSH; ++ks) {
        bf16x8 bfrag;
        if (tile == w && ks < PH) bfrag = w2tf[ks < PH ? ks : 0];
        else bfrag = ld8(SH + O::W2T + (int64_t)m * L2 + ks * 32 + 8 * g);
        acc = mfma16(ld8(sH2 + (mt * 16 + r16) * C::H2S + ks * 32 + 8 * g), bfrag, acc);
      }
      bf16x4 t4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const __bf16 hv = sH1[(mt * 16 + 4 * g + i) * C::H1S + m];
        t4[i] = ((float)hv > 0.f) ? (__bf16)acc[i] : (__bf16)0.f;
      }
      *reinterpret_cast<bf16x4*>(sdH1T + m * C::TS + mt * 16 + 4 * g) = t4;
      if (row0 + mt * 16 + 4 * g < Bp)  // padded rows of the last chunk stay inside the [L1][Bp] image
        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.dh1t) + (int64_t)m * Bp + row0 + mt * 16 + 4 * g) = t4;
    }
    __syncthreads();
    if (a.stamps && tid == 0) a.stamps[4] = __builtin_amdgcn_s_memrealtime();

    // ---------------- small-parameter grads (+ Adam + shadow refresh) ----------------
    const AdamScal o = sh_o;
    constexpr int NT_W2 = C::TN2 * C::TN1;
    constexpr int NT_W3 = C::TN2;
    for (int task = w; task < NT_W2 + NT_W3; task += kWaves) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      int64_t gi[4];
      bool valid[4];
      int rowv, colv;
      if (task < NT_W2) {
        const int nt = task % C::TN2, ct = task / C::TN2;
#pragma unroll
        for (int ks = 0; ks < BC / 32; ++ks) {
          const int b0 = ks * 32 + 8 * g;
          acc = mfma16(ld8(sdH2T + (nt * 16 + r16) * C::TS + b0), ld8(sH1T + (ct * 16 + r16) * C::TS + b0), acc);
        }
        rowv = nt * 16 + 4 * g;  // n
        colv = ct * 16 + r16;    // m
#pragma unroll
        for (int i = 0; i < 4; ++i) { gi[i] = O::W2 + (int64_t)(rowv + i) * L1 + colv; valid[i] = true; }
      } else {
        const int nt = task - NT_W2;
#pragma unroll
        for (int ks = 0; ks < BC / 32; ++ks) {
          const int b0 = ks * 32 + 8 * g;
          acc = mfma16(ld8(sdZT + r16 * C::TS + b0), ld8(sH2T + (nt * 16 + r16) * C::TS + b0), acc);
        }
        rowv = 4 * g;            // j
        colv = nt * 16 + r16;    // n
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          valid[i] = (rowv + i) < kNC;
          gi[i] = O::W3 + (int64_t)(valid[i] ? rowv + i : 0) * L2 + colv;
        }
      }
      // issue every load of the epilogue before any math (one round trip)
      float gv[4], pv[4], mv[4], vv[4], go[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gv[i] = acc[i];
        go[i] = (accum && valid[i]) ? a.grads[gi[i]] : 0.f;
        if (adam && valid[i]) { pv[i] = P[gi[i]]; mv[i] = a.exp_avg[gi[i]]; vv[i] = a.exp_avg_sq[gi[i]]; }
      }
      bf16x4 sh4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sh4[i] = (__bf16)0.f;
        if (!valid[i]) continue;
        const float gg = gv[i] + go[i];
        if (adam) {
          float m_ = mv[i], v_ = vv[i];
          const float p_ = adam1(pv[i], gg, m_, v_, o);
          a.params[gi[i]] = p_;
          a.exp_avg[gi[i]] = m_;
          a.exp_avg_sq[gi[i]] = v_;
          SHW[gi[i]] = (__bf16)p_;
          sh4[i] = (__bf16)p_;
        } else {
          a.grads[gi[i]] = gg;
        }
      }
      if (adam) {
        if (task < NT_W2) *reinterpret_cast<bf16x4*>(SHW + O::W2T + (int64_t)colv * L2 + rowv) = sh4;
        else *reinterpret_cast<bf16x4*>(SHW + O::W3T + (int64_t)colv * 16 + rowv) = sh4;
      }
    }
    // bias grads: column sums over the chunk
    for (int e = tid; e < L1 + L2 + kNC; e += kThreads) {
      const __bf16* row;
      int64_t gidx;
      if (e < L1) { row = sdH1T + e * C::TS; gidx = O::B1 + e; }
      else if (e < L1 + L2) { row = sdH2T + (e - L1) * C::TS; gidx = O::B2 + (e - L1); }
      else { row = sdZT + (e - L1 - L2) * C::TS; gidx = O::B3 + (e - L1 - L2); }
      float pv = 0.f, mv = 0.f, vv = 0.f, go = 0.f;
      if (accum) go = a.grads[gidx];
      if (adam) { pv = P[gidx]; mv = a.exp_avg[gidx]; vv = a.exp_avg_sq[gidx]; }
      float sum = 0.f;
#pragma unroll 8
      for (int b = 0; b < BC; ++b) sum += (float)row[b];
      sum += go;
      if (adam) {
        const float p_ = adam1(pv, sum, mv, vv, o);
        a.params[gidx] = p_;
        a.exp_avg[gidx] = mv;
        a.exp_avg_sq[gidx] = vv;
        SHW[gidx] = (__bf16)p_;
      } else {
        a.grads[gidx] = sum;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    const int64_t t = sh_t;
    if (a.advance_step) a.counters[0] = t;
    a.counters[2] = sh_cursor;  // batch the W1 kernel must gather
    if (U8) a.counters[1] = (a.n_batches > 0) ? (sh_cursor + 1) % a.n_batches : sh_cursor + 1;
    if (a.stats) {
      const int slot = (int)((t - 1) % (a.stats_ring > 0 ? a.stats_ring : 1));
      float* st = a.stats + slot * 4;
      st[0] = misc[0] * invB;
      st[1] = misc[1];
      st[2] = misc[2];
      st[3] = (float)t;
    }
    if (a.stamps) a.stamps[5] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------------
// W1 kernel: one workgroup per 16-pixel tile, one wave per 16-neuron tile.
// ---------------------------------------------------------------------------
template <int L1, bool U8>
__global__ __launch_bounds__(64 * (L1 / 16)) void mlp_w1_kernel(MLPStepArgs a) {
  constexpr int TN1 = L1 / 16;
  constexpr int XSS = 24;  // LDS row stride (16 pixels + 8 pad) in bf16
  constexpr int BMAX = 256;
  __shared__ __attribute__((aligned(16))) __bf16 sX[BMAX * XSS];
  __shared__ AdamScal sh_o;
  __shared__ int64_t sh_cursor;
  const int tid = threadIdx.x, lane = tid & 63, ct = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int kt = blockIdx.x;
  const int B = a.B;
  const int Bp = (B + 31) / 32 * 32;
  const bool adam = a.apply_adam;
  const bool accum = a.accumulate_grad;
  const int m = ct * 16 + r16, pix = kt * 16 + 4 * g;
  const int64_t gidx = (int64_t)m * kD + pix;
  // Adam state / old grads of this lane's 4 weights: issued first
  F4 p4{}, m4{}, v4{}, g4{};
  if (adam) {
    p4 = *reinterpret_cast<const F4*>(a.params + gidx);
    m4 = *reinterpret_cast<const F4*>(a.exp_avg + gidx);
    v4 = *reinterpret_cast<const F4*>(a.exp_avg_sq + gidx);
  }
  if (accum) g4 = *reinterpret_cast<const F4*>(a.grads + gidx);
  if (tid == 0) {
    const int64_t t = a.counters[0];  // already advanced by the head kernel
    sh_cursor = a.counters[2];
    adam_scalars(sh_o, t, a.lr_ptr ? a.lr_ptr[0] : a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.adamw);
  }
  __syncthreads();
  // gather this tile's 16-pixel slice of the batch rows
  const int64_t* idx = U8 ? a.order + sh_cursor * B : nullptr;
  for (int b = tid; b < Bp; b += 64 * TN1) {
    bf16x8 lo = zero8(), hi = zero8();
    if (b < B) {
      if constexpr (U8) {
        const uint4 v = *reinterpret_cast<const uint4*>(a.x_u8 + idx[b] * kD + kt * 16);
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        constexpr float inv255 = 1.0f / 255.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          lo[j] = (__bf16)((float)((wd[0] >> (8 * j)) & 0xffu) * inv255);
          lo[4 + j] = (__bf16)((float)((wd[1] >> (8 * j)) & 0xffu) * inv255);
          hi[j] = (__bf16)((float)((wd[2] >> (8 * j)) & 0xffu) * inv255);
          hi[4 + j] = (__bf16)((float)((wd[3] >> (8 * j)) & 0xffu) * inv255);
        }
      } else {
        const float* src = a.x_f32 + (int64_t)b * kD + kt * 16;
        lo = cvt8(ld4(src), ld4(src + 4));
        hi = cvt8(ld4(src + 8), ld4(src + 12));
      }
    }
    *reinterpret_cast<bf16x8*>(sX + b * XSS) = lo;
    *reinterpret_cast<bf16x8*>(sX + b * XSS + 8) = hi;
  }
  // dH1^T fragments (B operand) from the head kernel
  const __bf16* dh = reinterpret_cast<const __bf16*>(a.dh1t) + (int64_t)m * Bp;
  __syncthreads();
  const int q = r16 >> 2, pp = r16 & 3;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < Bp / 32; ++ks) {
    const int b0 = ks * 32 + 8 * g;
    const bf16x4 lo = tr_read(sX + (b0 + q) * XSS + 4 * pp);
    const bf16x4 hi = tr_read(sX + (b0 + 4 + q) * XSS + 4 * pp);
    const bf16x8 afrag = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    acc = mfma16(afrag, ld8(dh + b0), acc);
  }
  // D[row = pixel pix+i][col = m]
  const AdamScal o = sh_o;
  F4 gg{{acc[0] + g4.v[0], acc[1] + g4.v[1], acc[2] + g4.v[2], acc[3] + g4.v[3]}};
  if (adam) {
    bf16x4 sh4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p4.v[i] = adam1(p4.v[i], gg.v[i], m4.v[i], v4.v[i], o);
      sh4[i] = (__bf16)p4.v[i];
    }
    *reinterpret_cast<F4*>(a.params + gidx) = p4;
    *reinterpret_cast<F4*>(a.exp_avg + gidx) = m4;
    *reinterpret_cast<F4*>(a.exp_avg_sq + gidx) = v4;
    *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.shadow) + gidx) = sh4;
  } else {
    *reinterpret_cast<F4*>(a.grads + gidx) = gg;
  }
}

// ---------------------------------------------------------------------------
// Multi-workgroup Adam over the whole MLP arena + shadow refresh (world size > 1,
// after the gradient allreduce), or shadow refresh only (update = 0).
// ---------------------------------------------------------------------------
template <int L1, int L2>
__global__ __launch_bounds__(256) void mlp_adam_kernel(MLPAdamArgs a) {
  using O = Off<L1, L2>;
  __shared__ AdamScal sh_o;
  if (threadIdx.x == 0 && a.update) {
    const int64_t t = a.step_ptr[0];
    adam_scalars(sh_o, t, a.lr_ptr ? a.lr_ptr[0] : a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.adamw);
  }
  __syncthreads();
  const AdamScal o = sh_o;
  __bf16* SHW = reinterpret_cast<__bf16*>(a.shadow);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < O::NP; i += (int64_t)gridDim.x * blockDim.x) {
    float p = a.params[i];
    if (a.update) {
      float m = a.exp_avg[i], v = a.exp_avg_sq[i];
      p = adam1(p, a.grads[i] * a.grad_scale, m, v, o);
      a.params[i] = p;
      a.exp_avg[i] = m;
      a.exp_avg_sq[i] = v;
    }
    const __bf16 pb = (__bf16)p;
    SHW[i] = pb;
    if (i >= O::W2 && i < O::B2) {
      const int64_t r = i - O::W2;
      const int n = (int)(r / L1), mm = (int)(r - (int64_t)n * L1);
      SHW[O::W2T + (int64_t)mm * L2 + n] = pb;
    } else if (i >= O::W3 && i < O::B3) {
      const int64_t r = i - O::W3;
      const int j = (int)(r / L2), n = (int)(r - (int64_t)j * L2);
      SHW[O::W3T + (int64_t)n * 16 + j] = pb;
    }
  }
  // zero the W3^T class padding (j = 10..15)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)L2 * 6; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / 6), j = 10 + (int)(i - (int64_t)n * 6);
    SHW[O::W3T + (int64_t)n * 16 + j] = (__bf16)0.f;
  }
}

template <int BC, int L1, int L2>
constexpr bool fits() {
  return Cfg<BC, L1, L2>::total + 256 <= 160 * 1024;
}

template <int L1, int L2>
int dispatch2(const MLPStepArgs& a, hipStream_t stream) {
  const bool u8 = a.x_u8 != nullptr;
  bool launched = false;
  if constexpr (fits<64, L1, L2>()) {
    if (a.B > 32) {
      if (u8) hipLaunchKernelGGL((mlp_head_kernel<64, L1, L2, true>), dim3(1), dim3(kThreads), 0, stream, a);
      else hipLaunchKernelGGL((mlp_head_kernel<64, L1, L2, false>), dim3(1), dim3(kThreads), 0, stream, a);
      launched = true;
    }
  }
  if (!launched) {
    if (u8) hipLaunchKernelGGL((mlp_head_kernel<32, L1, L2, true>), dim3(1), dim3(kThreads), 0, stream, a);
    else hipLaunchKernelGGL((mlp_head_kernel<32, L1, L2, false>), dim3(1), dim3(kThreads), 0, stream, a);
  }
  if (u8) hipLaunchKernelGGL((mlp_w1_kernel<L1, true>), dim3(kD / 16), dim3(64 * (L1 / 16)), 0, stream, a);
  else hipLaunchKernelGGL((mlp_w1_kernel<L1, false>), dim3(kD / 16), dim3(64 * (L1 / 16)), 0, stream, a);
  return 0;
}

template <int L1, int L2>
int dispatch_adam(const MLPAdamArgs& a, hipStream_t stream) {
  const int64_t np = Off<L1, L2>::NP;
  int blocks = (int)((np + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL((mlp_adam_kernel<L1, L2>), dim3(blocks), dim3(256), 0, stream, a);
  return 0;
}

#define RLA_MLP2_SHAPES(X) \
  X(32, 32) X(32, 64) X(32, 128) X(32, 256) \
  X(64, 64) X(64, 128) X(64, 256) \
  X(128, 128) X(128, 256) X(128, 64)

}  // namespace

int launch_mlp_train_step2(const MLPStepArgs& a, hipStream_t stream) {
  if (a.B > 256) return -2;
#define RLA_CASE(a1, a2) if (a.L1 == a1 && a.L2 == a2) return dispatch2<a1, a2>(a, stream);
  RLA_MLP2_SHAPES(RLA_CASE)
#undef RLA_CASE
  return -1;
}

int launch_mlp_adam(const MLPAdamArgs& a, hipStream_t stream) {
#define RLA_CASE(a1, a2) if (a.L1 == a1 && a.L2 == a2) return dispatch_adam<a1, a2>(a, stream);
  RLA_MLP2_SHAPES(RLA_CASE)
#undef RLA_CASE
  return -1;
}

}  // namespace rla
