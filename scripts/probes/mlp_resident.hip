// ARCHIVED NEGATIVE RESULT (not built; removed from the _C extension in round 6).
// The resident one-workgroup training loop measured 14.1 vs 8.4 us/step for the
// pipelined one-launch step (profiles/r4_resident/); kept for reference only.  It
// needs the ResidentArgs declaration that kernels.h carried until round 5.
// Resident MNIST training loop: K optimizer steps of the 784-32-64-10 MLP (batch
// 32, bf16 MFMA compute, fp32 master weights, Adam) in ONE workgroup of ONE launch.
//
// Why (profiles/r4_dp/step_barrier.log, dp_phases): the one-launch step spreads a
// step over 60 CUs, and any hand-off between steps -- a kernel boundary in a
// hipGraph or an in-kernel grid barrier -- costs ~2.7 us on MI355X, a third of the
// 8.4 us step.  The whole training state is small: 27,882 parameters x (weight, m,
// v) = 335 KB, which fits one CU's 512 KB register file plus its 160 KB LDS, and a
// step is ~3.6 MFLOP.  So one workgroup keeps every parameter, its Adam state and
// the operand images resident for all K steps: no global traffic for the model
// inside the loop and no cross-CU synchronisation -- only barriers between the
// phases of a step.  Per step the HBM traffic is the next batch (32 gathered u8
// rows, copied straight into LDS by global_load_lds a step ahead) and one stats row.
//
// Layout: 4 waves (256 threads: one wave per SIMD, so a wave may hold 512
// registers); lane l: r = l & 31, h = l >> 5; MFMA v_mfma_f32_32x32x16_bf16 with A
// rows i = r / k = 8h..8h+7, B cols j = r / k = 8h.., D col j = r, rows
// i = (e & 3) + 8 (e >> 2) + 4 h.
//   W1 (32 x 784): 24 column tiles of 32 pixels, tile t owned by wave t % 4 (six
//     each).  A tile's dW1 comes out of the MFMA as D[pixel][neuron]; its fp32
//     weight / m / v live in that layout in the owning lanes (48 registers a tile,
//     288 a lane), and the forward's W1 operand is rebuilt from them every step
//     (bf16, one v_permlane32_swap per 4 values) -- no W1 image in LDS.  Pixels
//     768..783 (a half tile) and the other 2,794 parameters (b1, W2, b2, W3, b3)
//     are "small": their fp32 state is in LDS, 13 per thread.
//   LDS: the batch as u8 rows, double-buffered (this step's; the next one landing);
//     the small layers' bf16 weights; every activation / gradient image of a step;
//     the small parameters' gradients and Adam state.
// A step: F1 (each wave its own six W1 tiles' 12 k-steps, partial sums reduced in
// LDS) -> F2 -> F3 -> log-softmax / NLL / accuracy -> dW3, dH2 -> dW2, dH1, db2, db3
// -> dW1 + Adam on the owned tiles, db1 -> Adam on the small parameters.  Phases
// are separated by raw s_barrier + lgkmcnt(0): __syncthreads() would also wait for
// the in-flight next-batch DMA, which is waited for once, at the end of the step.
// Adam: torch.optim.Adam's update with its bias corrections in double (one thread,
// per step), v_sqrt / v_rcp instead of IEEE divisions (<= 2 ulp per update; the
// trajectory test bounds the drift against fp32 torch).
// Counters / order / stats follow the engine's device-state convention
// (mlp_step3.hip): counters[0] step, [1] next cursor, [2] last consumed cursor,
// [4] order buffer; stats ring rows (mean NLL, #correct, #rows, step).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "common.h"
#include "kernels.h"
#include "mlp_common.h"

namespace rla {
namespace {

using namespace mlp;

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kRB = 32, kRL1 = 32, kRL2 = 64, kRT = 256, kRW = kRT / 64;
constexpr int kS40 = 40;   // 32-wide images (80 B rows: 5 x 16 B, conflict-free b128 rows)
constexpr int kS72 = 72;   // 64-wide images (144 B rows)
constexpr int kS24 = 24;   // 16-wide images (48 B rows)
constexpr int kW1Tiles = 24;                    // full 32-pixel tiles (pixels 0..767)
constexpr int kTilesPerWave = kW1Tiles / kRW;   // 6
constexpr int kXBytes = kRB * kD;               // one batch, u8
constexpr int kXPieces = kXBytes / 16;          // 1568 16-byte DMA pieces
constexpr int kNSmall = 16 * kRL1 + kRL1 + kRL2 * kRL1 + kRL2 + kNC * kRL2 + kNC;  // 3,306
constexpr int kSmallPer = (kNSmall + kRT - 1) / kRT;                                  // 13
// small-parameter index s -> segments
constexpr int kSW1 = 0, kSB1 = 16 * kRL1, kSW2 = kSB1 + kRL1, kSB2 = kSW2 + kRL2 * kRL1, kSW3 = kSB2 + kRL2,
              kSB3 = kSW3 + kNC * kRL2;
static_assert(kSB3 + kNC == kNSmall, "small parameter segments");

// LDS image (bf16 unless noted); the F1 partials alias the backward images, which
// are dead while F1 runs
struct Lds {
  uint8_t x[2][kXBytes];      // X[b][pixel] u8: this step's batch, the next one (DMA)
  __bf16 w1h[kRL1 * kS24];    // W1[n1][768 + c], the half tile
  __bf16 h1[kRB * kS40];      // H1[b][n1]
  __bf16 h1t[kRL1 * kS40];    // H1^T[n1][b]
  __bf16 h2[kRB * kS72];      // H2[b][n2]
  __bf16 h2t[kRL2 * kS40];    // H2^T[n2][b]
  __bf16 w2[kRL2 * kS40];     // W2[n2][n1]
  __bf16 w3[32 * kS72];       // W3[c][n2], rows 10..31 zero
  union {
    float part[kRW - 1][16][64];  // F1 partial sums of waves 1.., D layout [slot][e][lane]
    struct {
      __bf16 dz[kRB * kS24];      // dZ[b][c], c 10..15 zero
      __bf16 dzt[32 * kS40];      // dZ^T[c][b] (rows >= 10 unused)
      __bf16 dh2[kRB * kS72];     // dH2[b][n2]
      __bf16 dh2t[kRL2 * kS40];   // dH2^T[n2][b]
      __bf16 dh1t[kRL1 * kS40];   // dH1^T[n1][b]
    } bw;
  } u;
  float z[kRB * 16];          // logits, then dZ (fp32) for db3
  float g[kNSmall + 14];      // small-parameter gradients
  float sw[kNSmall], sm[kNSmall], sv[kNSmall];  // small-parameter fp32 weight / m / v
  float b1[kRL1], b2[kRL2], b3[16];
  int64_t idx[2][kRB];        // sample indices of the batch a slot holds
  int lab[2][kRB];
  float stepsc[4];            // this step's Adam scalars: step_size, 1 / sqrt(bc2)
  float red[8];               // loss / correct sums
};

// global -> LDS copy of 16 bytes per lane (lane-linear from the wave-uniform LDS
// address `lds`), issued as inline asm: the compiler's memory model would treat the
// builtin's LDS write as aliasing every later ds_read and wait for the copy right
// there (s_waitcnt vmcnt(0) before the next phase's first LDS read -- the whole HBM
// latency exposed every step).  The copy is waited for explicitly at the step end.
// M0 is saved and restored around it (cdna_hip_programming.md, LDS-DMA recipe).
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// phase barrier: LDS writes visible, but in-flight global loads / DMA left alone
__device__ __forceinline__ void phase_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// 8 u8 pixels -> bf16x8 scaled by 1/255 (torchvision ToTensor; as u8x16_to_bf16)
__device__ __forceinline__ bf16x8 u8x8_to_bf16(uint32_t lo, uint32_t hi) {
  constexpr float inv255 = 1.0f / 255.0f;
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (__bf16)((float)((lo >> (8 * j)) & 0xffu) * inv255);
    r[4 + j] = (__bf16)((float)((hi >> (8 * j)) & 0xffu) * inv255);
  }
  return r;
}
// X row fragment: lane (batch r, pixels k0 + 8h .. + 7)
__device__ __forceinline__ bf16x8 x_row(const uint8_t* X, int k0, int lane) {
  const uint2 v = *reinterpret_cast<const uint2*>(X + (lane & 31) * kD + k0 + (lane >> 5) * 8);
  return u8x8_to_bf16(v.x, v.y);
}
// X^T fragment: lane (pixel p0 + r, batch rows k0 + 8h .. + 7)
__device__ __forceinline__ bf16x8 x_col(const uint8_t* X, int k0, int p0, int lane) {
  const uint8_t* p = X + (k0 + (lane >> 5) * 8) * kD + p0 + (lane & 31);
  uint32_t lo = 0u, hi = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    lo |= (uint32_t)p[q * kD] << (8 * q);
    hi |= (uint32_t)p[(q + 4) * kD] << (8 * q);
  }
  return u8x8_to_bf16(lo, hi);
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const __bf16 x = (__bf16)a, y = (__bf16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}
// the forward's W1 operand (B: col n1 = r, k = pixels p0 + 16s + 8h .. + 7) from the
// D-layout fp32 weights of the tile: lane (r, h) holds pixels drow(e, h); the
// partner lane (r, 1 - h) holds the other four of each group of eight
__device__ __forceinline__ bf16x8 w1_frag(const float (&w)[16], int s, int h) {
  const int e0 = 8 * s;
  const uint32_t lo0 = pack2(w[e0 + 0], w[e0 + 1]), lo1 = pack2(w[e0 + 2], w[e0 + 3]);  // pixels 16s + 4h + 0..3
  const uint32_t hi0 = pack2(w[e0 + 4], w[e0 + 5]), hi1 = pack2(w[e0 + 6], w[e0 + 7]);  // 16s + 8 + 4h + 0..3
  // h = 0 keeps its 0..3 and needs the partner's 4..7 (its lo); h = 1 keeps its
  // 12..15 and needs the partner's 8..11 (its hi)
  const uint32_t s0 = h ? lo0 : hi0, s1 = h ? lo1 : hi1;
  const auto x0 = __builtin_amdgcn_permlane32_swap(s0, s0, false, false);
  const auto x1 = __builtin_amdgcn_permlane32_swap(s1, s1, false, false);
  const uint32_t r0 = h ? x0[0] : x0[1], r1 = h ? x1[0] : x1[1];  // the partner's value
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  const u32x4v d = h ? u32x4v{r0, r1, hi0, hi1} : u32x4v{lo0, lo1, r0, r1};
  return __builtin_bit_cast(bf16x8, d);
}

__device__ __forceinline__ bf16x4 tr4(const __bf16* p) { return tr_read(p); }

// B (or A) fragment of a k-strided image I[k][j] (row stride S): k rows k0..k0+15,
// columns j0..j0+31 -> lane (j = j0 + r, k = k0 + 8h..): two transposed reads
__device__ __forceinline__ bf16x8 frag_tr(const __bf16* I, int S, int k0, int j0, int lane) {
  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int cho = 16 * (gq & 1) + 4 * p4, rwo = 8 * (gq >> 1) + q4;
  const __bf16* p = I + (k0 + rwo) * S + j0 + cho;
  return __builtin_shufflevector(tr4(p), tr4(p + 4 * S), 0, 1, 2, 3, 4, 5, 6, 7);
}
// row fragment: lane (row = i0 + r, k = k0 + 8h .. + 7) of a row-major image
__device__ __forceinline__ bf16x8 frag_row(const __bf16* I, int S, int i0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(I + (i0 + (lane & 31)) * S + k0 + (lane >> 5) * 8);
}
__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  return z;
}
// D-layout row of accumulator element e for lane half h
__device__ __forceinline__ int drow(int e, int h) { return (e & 3) + 8 * (e >> 2) + 4 * h; }

// fast Adam (see header): returns the new weight; m, v updated in place
__device__ __forceinline__ float adam_fast(float p, float g, float& m, float& v, float b1, float b2, float step_size,
                                           float inv_bc2, float eps, float wd, int adamw, float lr) {
  if (wd != 0.f) {
    if (adamw) p = p * (1.f - lr * wd);
    else g = fmaf(wd, p, g);
  }
  m = fmaf(1.f - b1, g - m, m);
  v = fmaf(1.f - b2, g * g, v * b2);
  const float denom = fmaf(__builtin_amdgcn_sqrtf(v), inv_bc2, eps);
  return fmaf(-step_size, m * __builtin_amdgcn_rcpf(denom), p);
}

// small parameter s -> (arena index)
__device__ __forceinline__ int64_t small_arena(int s) {
  using O = Off<kRL1, kRL2>;
  if (s < kSB1) return (int64_t)(s >> 4) * kD + 768 + (s & 15);
  if (s < kSW2) return O::B1 + (s - kSB1);
  if (s < kSB2) return O::W2 + (s - kSW2);
  if (s < kSW3) return O::B2 + (s - kSB2);
  if (s < kSB3) return O::W3 + (s - kSW3);
  return O::B3 + (s - kSB3);
}

// small parameter s: its new value into the operand images
__device__ __forceinline__ void small_publish(Lds& L, int s, float w) {
  if (s < kSB1) L.w1h[(s >> 4) * kS24 + (s & 15)] = (__bf16)w;
  else if (s < kSW2) L.b1[s - kSB1] = w;
  else if (s < kSB2) { const int i = s - kSW2; L.w2[(i / kRL1) * kS40 + (i % kRL1)] = (__bf16)w; }
  else if (s < kSW3) L.b2[s - kSB2] = w;
  else if (s < kSB3) { const int i = s - kSW3; L.w3[(i / kRL2) * kS72 + (i % kRL2)] = (__bf16)w; }
  else L.b3[s - kSB3] = w;
}

__global__ __launch_bounds__(kRT) void mlp_resident_kernel(ResidentArgs a) {
  __shared__ __attribute__((aligned(16))) Lds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;

  // ---------------------------------------------------------------- load state
  // W1 tiles owned by this wave: tile t = wave + 4u, D layout (col n1 = r, rows
  // pixel = 32 t + drow(e, h))
  float w1p[kTilesPerWave][16], w1m[kTilesPerWave][16], w1v[kTilesPerWave][16];
#pragma unroll
  for (int u = 0; u < kTilesPerWave; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t gi = (int64_t)r * kD + 32 * (wave + kRW * u) + drow(e, h);
      w1p[u][e] = a.params[gi];
      w1m[u][e] = a.exp_avg[gi];
      w1v[u][e] = a.exp_avg_sq[gi];
    }
  for (int q = tid; q < kNSmall; q += kRT) {
    const int64_t gi = small_arena(q);
    L.sw[q] = a.params[gi];
    L.sm[q] = a.exp_avg[gi];
    L.sv[q] = a.exp_avg_sq[gi];
  }
  for (int q = tid; q < 32 * kS72; q += kRT) L.w3[q] = (__bf16)0.f;
  __syncthreads();
  for (int q = tid; q < kNSmall; q += kRT) small_publish(L, q, L.sw[q]);
  if (tid < 16) L.b3[tid] = tid < kNC ? L.b3[tid] : 0.f;

  // device state
  const int64_t t0 = a.counters[0];
  int64_t cursor = a.counters[1], ob = a.counters[4];
  const float lr = a.lr_ptr ? *a.lr_ptr : a.lr;
  const double b1d = (double)a.beta1, b2d = (double)a.beta2;
  double b1t = 0.0, b2t = 0.0;
  if (tid == 0) {
    b1t = pow(b1d, (double)t0);
    b2t = pow(b2d, (double)t0);
  }
  auto next_cursor = [&](int64_t& c, int64_t& o) {
    if (++c >= a.n_batches) { c = 0; o ^= 1; }
  };
  auto order_at = [&](int64_t c, int64_t o, int b) {
    // clamped: a look-ahead past the window may read an order buffer the host refills
    // later (its indices are always a valid shard order, the clamp is the guard)
    const int64_t v = a.order[o * a.order_stride + c * kRB + b];
    return v < 0 ? (int64_t)0 : (v >= a.n_data ? a.n_data - 1 : v);
  };
  // slots: batch k lives in slot k & 1 (indices, labels, pixels)
  int64_t c1 = cursor, o1 = ob;
  next_cursor(c1, o1);  // batch 1
  if (tid < kRB) {
    const int64_t i0 = order_at(cursor, ob, tid);
    L.idx[0][tid] = i0;
    L.lab[0][tid] = (int)a.labels[i0];
    L.idx[1][tid] = order_at(c1, o1, tid);
  }
  __syncthreads();
  for (int q = tid; q < kXPieces; q += kRT) {
    const int b = q / 49, kt = q - b * 49;
    *reinterpret_cast<uint4*>(L.x[0] + q * 16) = *reinterpret_cast<const uint4*>(a.x_u8 + L.idx[0][b] * kD + kt * 16);
  }
  for (int q = tid; q < kRB * kS24; q += kRT) L.u.bw.dz[q] = (__bf16)0.f;
  __syncthreads();

  int64_t last_cursor = cursor;
  int64_t c2 = c1, o2 = o1;
  next_cursor(c2, o2);  // batch 2: its indices are fetched during step 0
  for (int k = 0; k < a.K; ++k) {
    const int cur = k & 1, nxt = cur ^ 1;
    const int64_t t = t0 + k + 1;
    // batch k + 2's indices and batch k + 1's labels, into registers until the step's end
    int64_t idx2 = 0;
    int lab1 = 0;
    if (tid < kRB) {
      idx2 = order_at(c2, o2, tid);
      lab1 = (int)a.labels[L.idx[nxt][tid]];
    }
    // batch k + 1's pixels (issued after the loads above, so no wait for those
    // registers lands behind the copy): global -> LDS slot nxt (lane-linear DMA pieces), in
    // flight for the whole step
    for (int i = wave; i * 64 < kXPieces; i += kRW) {
      const int q = i * 64 + lane;
      const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_addr(L.x[nxt] + i * 64 * 16));
      if (q < kXPieces) {
        const int b = q / 49, kt = q - b * 49;
        dma16(a.x_u8 + L.idx[nxt][b] * kD + kt * 16, dst);
      }
    }
    if (tid == 0) {
      b1t *= b1d;
      b2t *= b2d;
      L.stepsc[0] = (float)((double)lr / (1.0 - b1t));
      L.stepsc[1] = (float)(1.0 / sqrt(1.0 - b2t));
    }
    const uint8_t* X = L.x[cur];

    // ---------------------------------------------------- F1: H1 = relu(X W1^T + b1)
    {
      f32x16 acc = zero16();
#pragma unroll
      for (int u = 0; u < kTilesPerWave; ++u) {
        const int p0 = 32 * (wave + kRW * u);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) acc = mfma(x_row(X, p0 + 16 * s2, lane), w1_frag(w1p[u], s2, h), acc);
      }
      if (wave == 0) acc = mfma(x_row(X, 768, lane), frag_row(L.w1h, kS24, 0, 0, lane), acc);
      if (wave > 0) {
#pragma unroll
        for (int e = 0; e < 16; ++e) L.u.part[wave - 1][e][lane] = acc[e];
      }
      phase_barrier();
      if (wave == 0) {
        // D[b][n1]: col n1 = r, rows b = drow(e, h); fixed summation order
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float sum = acc[e] + L.u.part[0][e][lane] + L.u.part[1][e][lane] + L.u.part[2][e][lane] + L.b1[r];
          const __bf16 v = (__bf16)(sum > 0.f ? sum : 0.f);
          L.h1[drow(e, h) * kS40 + r] = v;
          L.h1t[r * kS40 + drow(e, h)] = v;
        }
      }
      phase_barrier();
    }

    // ---------------------------------------------------- F2: H2 = relu(H1 W2^T + b2)
    if (wave < 2) {
      const int j0 = 32 * wave;
      f32x16 acc = zero16();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        acc = mfma(frag_row(L.h1, kS40, 0, 16 * s2, lane), frag_row(L.w2, kS40, j0, 16 * s2, lane), acc);
      const float bias = L.b2[j0 + r];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float sum = acc[e] + bias;
        const __bf16 v = (__bf16)(sum > 0.f ? sum : 0.f);
        L.h2[drow(e, h) * kS72 + j0 + r] = v;
        L.h2t[(j0 + r) * kS40 + drow(e, h)] = v;
      }
    }
    phase_barrier();

    // ---------------------------------------------------- F3: logits = H2 W3^T + b3
    if (wave == 0) {
      f32x16 acc = zero16();
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        acc = mfma(frag_row(L.h2, kS72, 0, 16 * s2, lane), frag_row(L.w3, kS72, 0, 16 * s2, lane), acc);
      if (r < kNC) {
#pragma unroll
        for (int e = 0; e < 16; ++e) L.z[drow(e, h) * 16 + r] = acc[e] + L.b3[r];
      }
    }
    phase_barrier();

    // ---------------------------------------------------- log-softmax, NLL, dZ
    if (tid < kRB) {
      const int b = tid, y = L.lab[cur][b];
      float zb[kNC];
      float mx = -INFINITY;
      int am = 0;
#pragma unroll
      for (int c = 0; c < kNC; ++c) {
        zb[c] = L.z[b * 16 + c];
        if (zb[c] > mx) { mx = zb[c]; am = c; }
      }
      const float zy = L.z[b * 16 + y];
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < kNC; ++c) {
        zb[c] = __expf(zb[c] - mx);
        se += zb[c];
      }
      const float loss = mx + __logf(se) - zy;
      const float inv = 1.f / se;
#pragma unroll
      for (int c = 0; c < kNC; ++c) {
        const float d = (zb[c] * inv - (c == y ? 1.f : 0.f)) * (1.f / kRB);
        const __bf16 db = (__bf16)d;
        L.u.bw.dz[b * kS24 + c] = db;
        L.u.bw.dzt[c * kS40 + b] = db;
        L.z[b * 16 + c] = d;
      }
#pragma unroll
      for (int c = kNC; c < 16; ++c) L.u.bw.dz[b * kS24 + c] = (__bf16)0.f;
      // batch sums of the loss and #correct over lanes 0..31
      float ls = loss, cs = am == y ? 1.f : 0.f;
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) {
        ls += __shfl_xor(ls, o, 32);
        cs += __shfl_xor(cs, o, 32);
      }
      if (tid == 0 && a.stats) {
        float* st = a.stats + (int)((t - 1) % (a.stats_ring > 0 ? a.stats_ring : 1)) * 4;
        st[0] = ls * (1.f / kRB);
        st[1] = cs;
        st[2] = (float)kRB;
        st[3] = (float)t;
      }
    }
    phase_barrier();

    // ---------------------------------------------------- dW3, dH2
    if (wave < 2) {
      // dW3 D[c][n2] = dZ^T . H2 (k = batch): col n2 = j0 + r, rows c
      const int j0 = 32 * wave;
      f32x16 acc = zero16();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        acc = mfma(frag_row(L.u.bw.dzt, kS40, 0, 16 * s2, lane), frag_row(L.h2t, kS40, j0, 16 * s2, lane), acc);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = drow(e, h);
        if (c < kNC) L.g[kSW3 + c * kRL2 + j0 + r] = acc[e];
      }
    } else {
      // dH2 D[b][n2] = dZ . W3 (k = class, one step of 16): B = W3^T by transposed reads
      const int j0 = 32 * (wave - 2);
      const f32x16 acc = mfma(frag_row(L.u.bw.dz, kS24, 0, 0, lane), frag_tr(L.w3, kS72, 0, j0, lane), zero16());
      const int n2 = j0 + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // rows b = 8g + 4h .. + 3: the ReLU mask from H2^T
        const bf16x4 hv = *reinterpret_cast<const bf16x4*>(L.h2t + n2 * kS40 + 8 * g + 4 * h);
        bf16x4 dv;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          dv[q] = (__bf16)((float)hv[q] > 0.f ? acc[4 * g + q] : 0.f);
          L.u.bw.dh2[(8 * g + 4 * h + q) * kS72 + n2] = dv[q];
        }
        *reinterpret_cast<bf16x4*>(L.u.bw.dh2t + n2 * kS40 + 8 * g + 4 * h) = dv;
      }
    }
    phase_barrier();

    // ---------------------------------------------------- dW2, dH1, db2, db3
    if (wave < 2) {
      // dW2 D[n2][n1] = dH2^T . H1 (k = batch): col n1 = r, rows n2 = i0 + drow
      const int i0 = 32 * wave;
      f32x16 acc = zero16();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        acc = mfma(frag_row(L.u.bw.dh2t, kS40, i0, 16 * s2, lane), frag_row(L.h1t, kS40, 0, 16 * s2, lane), acc);
#pragma unroll
      for (int e = 0; e < 16; ++e) L.g[kSW2 + (i0 + drow(e, h)) * kRL1 + r] = acc[e];
    } else if (wave == 2) {
      // dH1 D[b][n1] = dH2 . W2 (k = n2, 4 steps): B = W2^T by transposed reads
      f32x16 acc = zero16();
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        acc = mfma(frag_row(L.u.bw.dh2, kS72, 0, 16 * s2, lane), frag_tr(L.w2, kS40, 16 * s2, 0, lane), acc);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bf16x4 hv = *reinterpret_cast<const bf16x4*>(L.h1t + r * kS40 + 8 * g + 4 * h);
        bf16x4 dv;
#pragma unroll
        for (int q = 0; q < 4; ++q) dv[q] = (__bf16)((float)hv[q] > 0.f ? acc[4 * g + q] : 0.f);
        *reinterpret_cast<bf16x4*>(L.u.bw.dh1t + r * kS40 + 8 * g + 4 * h) = dv;
      }
    } else {
      // wave 3: db2 (lane = n2) and db3 (lanes < 10): column sums over the batch
      float sum = 0.f;
#pragma unroll
      for (int b = 0; b < kRB; ++b) sum += (float)L.u.bw.dh2t[lane * kS40 + b];
      L.g[kSB2 + lane] = sum;
      if (lane < kNC) {
        float c3 = 0.f;
        for (int b = 0; b < kRB; ++b) c3 += L.z[b * 16 + lane];
        L.g[kSB3 + lane] = c3;
      }
    }
    phase_barrier();

    // ---------------------------------------------------- dW1 + Adam (owned tiles), db1
    {
      const float step_size = L.stepsc[0], inv_bc2 = L.stepsc[1];
#pragma unroll
      for (int u = 0; u < kTilesPerWave; ++u) {
        __builtin_amdgcn_sched_barrier(0);  // one tile at a time: bounded register live ranges
        const int p0 = 32 * (wave + kRW * u);
        // D[pixel][n1] = X^T . dH1 (k = batch)
        f32x16 acc = zero16();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          acc = mfma(x_col(X, 16 * s2, p0, lane), frag_row(L.u.bw.dh1t, kS40, 0, 16 * s2, lane), acc);
#pragma unroll
        for (int e = 0; e < 16; ++e)
          w1p[u][e] = adam_fast(w1p[u][e], acc[e], w1m[u][e], w1v[u][e], a.beta1, a.beta2, step_size, inv_bc2,
                                a.eps, a.weight_decay, a.adamw, lr);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (wave == 0) {
        // the half tile (pixels 768..783): gradient only, Adam by its small owners
        f32x16 acc = zero16();
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          acc = mfma(x_col(X, 16 * s2, 768, lane), frag_row(L.u.bw.dh1t, kS40, 0, 16 * s2, lane), acc);
#pragma unroll
        for (int e = 0; e < 8; ++e) L.g[kSW1 + r * 16 + drow(e, h)] = acc[e];  // rows < 16
      } else if (wave == 1 && lane < kRL1) {
        float sum = 0.f;
#pragma unroll
        for (int b = 0; b < kRB; ++b) sum += (float)L.u.bw.dh1t[lane * kS40 + b];
        L.g[kSB1 + lane] = sum;
      }
    }
    phase_barrier();

    // ---------------------------------------------------- Adam (small parameters)
    {
      const float step_size = L.stepsc[0], inv_bc2 = L.stepsc[1];
      for (int q = tid; q < kNSmall; q += kRT) {
        float m = L.sm[q], v = L.sv[q];
        const float w = adam_fast(L.sw[q], L.g[q], m, v, a.beta1, a.beta2, step_size, inv_bc2, a.eps,
                                  a.weight_decay, a.adamw, lr);
        L.sw[q] = w;
        L.sm[q] = m;
        L.sv[q] = v;
        small_publish(L, q, w);
      }
    }
    // the next batch: its pixels (DMA), labels and the indices after it
    if (tid < kRB) {
      L.lab[nxt][tid] = lab1;
      L.idx[cur][tid] = idx2;  // batch k + 2 takes slot k & 1
    }
    last_cursor = cursor;
    cursor = c1;
    ob = o1;
    c1 = c2;
    o1 = o2;
    next_cursor(c2, o2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---------------------------------------------------------------- write back
#pragma unroll
  for (int u = 0; u < kTilesPerWave; ++u)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t gi = (int64_t)r * kD + 32 * (wave + kRW * u) + drow(e, h);
      a.params[gi] = w1p[u][e];
      a.exp_avg[gi] = w1m[u][e];
      a.exp_avg_sq[gi] = w1v[u][e];
    }
  for (int q = tid; q < kNSmall; q += kRT) {
    const int64_t gi = small_arena(q);
    a.params[gi] = L.sw[q];
    a.exp_avg[gi] = L.sm[q];
    a.exp_avg_sq[gi] = L.sv[q];
  }
  if (tid == 0 && a.K > 0) {
    a.counters[0] = t0 + a.K;
    a.counters[1] = cursor;
    a.counters[2] = last_cursor;
    a.counters[4] = ob;
    for (int i = 0; i < 5; ++i) a.counters[5 + i] = a.counters[i];
  }
}

}  // namespace

bool resident_supported(int L1, int L2, int B) { return L1 == kRL1 && L2 == kRL2 && B == kRB; }

int launch_mlp_resident(const ResidentArgs& a, hipStream_t stream) {
  if (!resident_supported(a.L1, a.L2, a.B) || a.K < 0 || a.n_batches < 1) return -1;
  if (a.K == 0) return 0;
  hipLaunchKernelGGL(mlp_resident_kernel, dim3(1), dim3(kRT), 0, stream, a);
  return 0;
}

}  // namespace rla
