// ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels) on the MFMA units,
// NHWC bf16, optionally with the following BatchNorm's batch statistics in the epilogue.
//
//   y[n][oh][ow][co] = sum over r, s, c of x[n][2 oh - 3 + r][2 ow - 3 + s][c] * w[co][r][s][c]
//
// Why a kernel of our own: MIOpen's implicit GEMM for this layer runs at ~90 TFLOP/s
// (173 us a step at batch 128, profiles/r5_prof/kernel_stats_rn50.csv: 3 input
// channels make its K tiles mostly padding), and BatchNorm then re-reads the 205 MB
// output once more for its statistics.  The layer is output-bound: 205 MB of bf16 y
// against 38 MB of input and 15 GFLOP.
//
// Implicit GEMM D[co][m] = W[co][k] . X[k][m] with k = (r, s, c) laid out as r x 32
// slots, slot j = 4 s + c (c = 3 and s = 7 are zero weights): K = 224 = 14 MFMA
// k-steps of 16.
//   * the tile is kT = 2 output rows x (up to) 128 output columns of one image; its
//     2 kT + 5 = 9 input rows sit in LDS as 4-channel pixels (8 bytes: the 4th channel
//     written as 0) with the conv's 3 pad pixels on the left, so the 16 slots of a
//     lane's k-step are 16 CONTIGUOUS bytes: pixel 2 ow + s of row r starts at byte
//     16 ow + 8 s -- one 16-byte-aligned ds_read_b128 per MFMA pair, no gather.  Slot
//     s = 7 reads the next pixel (real data, zero weight);
//   * the whole weight (64 x 224 slots) lives in VGPRs as A fragments, built once per
//     workgroup from an LDS copy of the raw [64][7][7][3] shadow;
//   * 4 waves = 4 x 32 output columns; a wave computes 2 rows x 32 columns x 64
//     channels per tile (4 accumulator blocks);
//   * persistent: one workgroup per CU walks a contiguous tile range; the next tile's
//     input rows are loaded into registers (12-byte pixel pairs) while this tile is
//     multiplied, then converted to 4-channel pixels in the other LDS buffer;
//   * ST: each lane keeps the bf16-rounded outputs' sums and sums of squares for its
//     32 channels across all its tiles; one fixed-order LDS reduction per workgroup
//     writes row g of part [G][2][64] (bn_finalize's layout; deterministic).
// Requires W even, OW <= 128, W <= 256 (host checks).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "kernels.h"

namespace rla {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kStThreads = 256;
constexpr int kT = 2;                // output rows per tile
constexpr int kRowsIn = 2 * kT + 5;  // input rows a tile touches
constexpr int kKS = 14;              // k-steps: 7 rows x 32 slots / 16
constexpr int kNP = 5;               // 12-byte pixel-pair pieces per thread and tile (9 rows x <= 128 pairs)
constexpr int kMaxW = 256;
constexpr int kRowPx = kMaxW + 8;    // 3 pad pixels left, >= 5 right (slot overrun)
constexpr int kBufBytes = kRowsIn * kRowPx * 8;
constexpr int kWBytes = 64 * 147 * 2;
constexpr int kRedBytes = 4 * 32 * 2 * 65 * 4;  // ST: [wave][pixel lane][stat][64 channels (+1 pad)]
constexpr int kLdsBytes = (2 * kBufBytes + kWBytes) > kRedBytes ? (2 * kBufBytes + kWBytes) : kRedBytes;

struct Piece {
  uint32_t v[3];  // two 3-channel bf16 pixels
};

template <bool ST>
__global__ __launch_bounds__(kStThreads) void stem_fwd_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ w,
                                                              uint16_t* __restrict__ y, float* __restrict__ part,
                                                              StemGeom g) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rowb = (g.W + 8) * 8;  // bytes per padded 4-channel input row
  const int bufb = kRowsIn * rowb;
  const int ohp = (g.OH + kT - 1) / kT;
  const int ntile = g.N * ohp;
  const int t_lo = (int)((int64_t)ntile * blockIdx.x / gridDim.x);
  const int t_hi = (int)((int64_t)ntile * (blockIdx.x + 1) / gridDim.x);

  // raw weight -> LDS; both input buffers zeroed (pad columns are never written again)
  uint16_t* wl = reinterpret_cast<uint16_t*>(lds + 2 * bufb);
  for (int i = tid; i < 64 * 147; i += kStThreads) wl[i] = w[i];
  for (int i = tid * 16; i < 2 * bufb; i += kStThreads * 16) *reinterpret_cast<u32x4*>(lds + i) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  // A fragments: lane (co = 32 i + lane & 31) holds slots 8 (lane >> 5) .. + 8 of k-step kk
  bf16x8 fa[kKS][2];
#pragma unroll
  for (int kk = 0; kk < kKS; ++kk)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = 32 * i + (lane & 31);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = kk * 16 + 8 * (lane >> 5) + e;
        const int r = k >> 5, j = k & 31, s = j >> 2, c = j & 3;
        const uint16_t b = (c < 3 && s < 7) ? wl[co * 147 + (r * 7 + s) * 3 + c] : (uint16_t)0;
        fa[kk][i][e] = __builtin_bit_cast(__bf16, b);
      }
    }

  const int pp = g.W >> 1;  // pixel pairs per input row
  const int npieces = kRowsIn * pp;
  uint8_t* scratch = lds + 2 * bufb;  // the weight staging area, dead after the prologue
  __syncthreads();                    // (every wave built its fragments from it)
  Piece pc[kNP];
  // the tile's 9 input rows, 12 bytes (a pixel pair) per piece; rows outside the image read row 0 (zeroed at store)
  auto load = [&](int t) {
    const int n = t / ohp, oh0 = (t - n * ohp) * kT;
#pragma unroll
    for (int u = 0; u < kNP; ++u) {
      int p = tid + u * kStThreads;
      p = p < npieces ? p : npieces - 1;
      const int q = p / pp, c2 = p - q * pp;
      int ih = 2 * oh0 - 3 + q;
      ih = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(x + (((int64_t)n * g.H + ih) * g.W + 2 * c2) * 3);
      pc[u].v[0] = src[0];
      pc[u].v[1] = src[1];
      pc[u].v[2] = src[2];
    }
  };
  // pixel pair (c0 c1 c2)(c0 c1 c2) -> two 4-channel pixels, 16 bytes at pixel 3 + 2 c2 of row q
  auto store = [&](int t, int buf) {
    const int n = t / ohp, oh0 = (t - n * ohp) * kT;
    uint8_t* B = lds + buf * bufb;
#pragma unroll
    for (int u = 0; u < kNP; ++u) {
      // unconditional (surplus pieces go to a dead scratch slot): a store under a branch
      // lets hipcc sink the piece's global load into it and wait for it right there
      const int p = tid + u * kStThreads;
      const int q = p / pp, c2 = p - q * pp;
      const int ih = 2 * oh0 - 3 + q;
      const bool ok = ih >= 0 && ih < g.H;
      const uint32_t a0 = ok ? pc[u].v[0] : 0u, a1 = ok ? pc[u].v[1] : 0u, a2 = ok ? pc[u].v[2] : 0u;
      // bf16 elements e0..e5 = (a0.lo a0.hi a1.lo a1.hi a2.lo a2.hi)
      const u32x2 lo = {a0, a1 & 0xFFFFu};                          // e0 e1 | e2 0
      const u32x2 hi = {(a1 >> 16) | (a2 << 16), a2 >> 16};         // e3 e4 | e5 0
      uint8_t* dst = p < npieces ? B + q * rowb + (3 + 2 * c2) * 8 : scratch;
      *reinterpret_cast<u32x2*>(dst) = lo;
      *reinterpret_cast<u32x2*>(dst + 8) = hi;
    }
  };

  f32x16 acc[kT][2];
  float bs[2][16], bq[2][16];
  if constexpr (ST) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) bs[i][k] = bq[i][k] = 0.f;
  }
  const int ow = 32 * wave + (lane & 31);
  const int owc = ow < g.OW ? ow : g.OW - 1;  // columns past the image compute a duplicate, never stored

  auto compute = [&](int buf) {
    const uint8_t* B = lds + buf * bufb + owc * 16 + 16 * (lane >> 5);
#pragma unroll
    for (int h = 0; h < kT; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[h][i] = f32x16{};
#pragma unroll
    for (int kk = 0; kk < kKS; ++kk) {
#pragma unroll
      for (int h = 0; h < kT; ++h) {
        // k-step kk: kernel row r = kk / 2, slots 16 (kk & 1) + 8 (lane >> 5) .. + 8
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(B + (2 * h + (kk >> 1)) * rowb + 32 * (kk & 1));
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[h][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[kk][i], fb, acc[h][i], 0, 0, 0);
      }
    }
  };

  // D[co][m]: lane -> output column (lane & 31); accumulator k -> channel (k & 3) + 8 (k >> 2) + 4 (lane >> 5)
  auto epilogue = [&](int t) {
    const int n = t / ohp, oh0 = (t - n * ohp) * kT;
#pragma unroll
    for (int h = 0; h < kT; ++h) {
      const int oh = oh0 + h;
      // lanes l and l ^ 32 hold the same pixel (the swap stays in-pixel); one
      // v_permlane32_swap per dword of each channel-group pair (q, q + 1) gives lane
      // half hl channels 16 p + 8 hl .. + 8: 16-byte stores instead of 8-byte ones
      const bool ok = oh < g.OH && ow < g.OW;
      uint16_t* yo = y + (((int64_t)n * g.OH + (ok ? oh : 0)) * g.OW + (ok ? ow : 0)) * 64 + 8 * (lane >> 5);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        uint32_t v[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x4 b;
#pragma unroll
          for (int e = 0; e < 4; ++e) b[e] = (__bf16)acc[h][i][4 * q + e];
          if constexpr (ST) {
            if (ok) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float f = (float)b[e];
                bs[i][4 * q + e] += f;
                bq[i][4 * q + e] = __builtin_fmaf(f, f, bq[i][4 * q + e]);
              }
            }
          }
          const u32x2 pk = __builtin_bit_cast(u32x2, b);
          v[q][0] = pk[0];
          v[q][1] = pk[1];
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const auto s0 = __builtin_amdgcn_permlane32_swap(v[2 * p][0], v[2 * p + 1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(v[2 * p][1], v[2 * p + 1][1], false, false);
          const u32x4 o = {s0[0], s1[0], s0[1], s1[1]};
          if (ok) *reinterpret_cast<u32x4*>(yo + 32 * i + 16 * p) = o;
        }
      }
    }
  };

  if (t_lo < t_hi) {
    load(t_lo);
    store(t_lo, 0);
    __syncthreads();
    for (int t = t_lo; t < t_hi; ++t) {
      const int buf = (t - t_lo) & 1;
      // in flight behind this tile's MFMAs; unconditional (the last tile re-loads itself):
      // a load under a branch makes the loaded registers a join value, and hipcc then
      // waits for each load right after issuing it to copy the registers
      load(t + 1 < t_hi ? t + 1 : t);
      compute(buf);
      store(t + 1 < t_hi ? t + 1 : t, buf ^ 1);  // (the last tile: a dead copy of itself)
      epilogue(t);
      __syncthreads();
    }
  }
  if constexpr (ST) {
    constexpr int kSR = 65;
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
    const int row = (wave * 32 + (lane & 31)) * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int co = i * 32 + 8 * (k >> 2) + 4 * (lane >> 5) + (k & 3);
        red[row * kSR + co] = bs[i][k];
        red[(row + 1) * kSR + co] = bq[i][k];
      }
    __syncthreads();
    if (tid < 128) {  // (stat, channel): 128 rows in a fixed order
      const int st = tid >> 6, c = tid & 63;
      float a = 0.f;
      for (int r = 0; r < 4 * 32; ++r) a += red[(2 * r + st) * kSR + c];
      part[((int64_t)blockIdx.x * 2 + st) * 64 + c] = a;
    }
  }
}

// ---------------------------------------------------------------- weight gradient
// dW[co][r][s][c] = sum over output pixels m of dy[m][co] * x[2 oh - 3 + r][2 ow - 3 + s][c]:
// D[co][slot] = dy^T . im2col(x) with the reduction over pixels, 16 per MFMA k-step.
// Both operands are pixel-strided, so both are read with ds_read_b64_tr_b16 (lane i
// of a 16-lane group gets column i of 4 consecutive pixel rows), as in conv_wgrad.hip:
//   * dy rows: the tile's 2 x 128 output pixels x 64 channels (+32 pad) in LDS;
//   * x "rows" are never materialised: the im2col row of pixel (h, ow), kernel row r,
//     is the 64 bytes at ow x 16 of input row 2 h + r of the same 4-channel image the
//     forward stages -- a per-lane address (stride-2 windows overlap, which is fine);
//   * each wave takes every 4th k-step of a tile and accumulates ALL 14 output blocks
//     (2 channel blocks x 7 kernel rows, 224 accumulators) over its workgroup's tiles;
//     the 4 waves are summed through LDS in a fixed order into row g of part
//     [G][64][224], and stem_wgrad_reduce sums the rows in order into the fp32
//     [64][7][7][3] gradient (the channels_last weight's memory order).  Deterministic.
constexpr int kSDY = 96;                       // dy LDS row: 64 channels + 32 pad (bf16)
constexpr int kTPix = kT * 128;                // pixel rows of a tile
constexpr int kDyBytes = kTPix * kSDY * 2;
constexpr int kWgBuf = kBufBytes + kDyBytes;
constexpr int kWgLds = 2 * kWgBuf;
static_assert(kWgLds >= 64 * 224 * 4, "wave reduction image fits");

typedef __attribute__((address_space(3))) bf16x4 lds_b4;
__device__ __forceinline__ bf16x4 str4(const uint8_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4*)(p));
}
__device__ __forceinline__ bf16x8 scat8(bf16x4 lo, bf16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__global__ __launch_bounds__(kStThreads) void stem_wgrad_kernel(const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ dy,
                                                                float* __restrict__ part, StemGeom g) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWgLds + 16];  // + a scratch slot for surplus pieces
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rowb = (g.W + 8) * 8;
  const int ohp = (g.OH + kT - 1) / kT;
  const int ntile = g.N * ohp;
  const int t_lo = (int)((int64_t)ntile * blockIdx.x / gridDim.x);
  const int t_hi = (int)((int64_t)ntile * (blockIdx.x + 1) / gridDim.x);
  for (int i = tid * 16; i < kWgLds; i += kStThreads * 16) *reinterpret_cast<u32x4*>(lds + i) = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();

  const int pp = g.W >> 1, npieces = kRowsIn * pp;
  Piece pc[kNP];
  u32x4 dv[8];  // the tile's dy: 256 rows x 8 16-byte chunks, 8 per thread
  auto load = [&](int t) {
    const int n = t / ohp, oh0 = (t - n * ohp) * kT;
#pragma unroll
    for (int u = 0; u < kNP; ++u) {
      int p = tid + u * kStThreads;
      p = p < npieces ? p : npieces - 1;
      const int q = p / pp, c2 = p - q * pp;
      int ih = 2 * oh0 - 3 + q;
      ih = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih);
      const uint32_t* src = reinterpret_cast<const uint32_t*>(x + (((int64_t)n * g.H + ih) * g.W + 2 * c2) * 3);
      pc[u].v[0] = src[0];
      pc[u].v[1] = src[1];
      pc[u].v[2] = src[2];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = tid + u * kStThreads, row = c >> 3, ch = c & 7;
      const int h = row >> 7;
      int ow = row & 127, oh = oh0 + h;
      ow = ow < g.OW ? ow : g.OW - 1;
      oh = oh < g.OH ? oh : g.OH - 1;
      dv[u] = *reinterpret_cast<const u32x4*>(dy + (((int64_t)n * g.OH + oh) * g.OW + ow) * 64 + ch * 8);
    }
  };
  auto store = [&](int t, int buf) {
    const int n = t / ohp, oh0 = (t - n * ohp) * kT;
    uint8_t* B = lds + buf * kWgBuf;
#pragma unroll
    for (int u = 0; u < kNP; ++u) {  // unconditional: see stem_fwd_kernel's store
      const int p = tid + u * kStThreads;
      const int q = p / pp, c2 = p - q * pp;
      const int ih = 2 * oh0 - 3 + q;
      const bool ok = ih >= 0 && ih < g.H;
      const uint32_t a0 = ok ? pc[u].v[0] : 0u, a1 = ok ? pc[u].v[1] : 0u, a2 = ok ? pc[u].v[2] : 0u;
      const u32x2 lo = {a0, a1 & 0xFFFFu};
      const u32x2 hi = {(a1 >> 16) | (a2 << 16), a2 >> 16};
      uint8_t* dst = p < npieces ? B + q * rowb + (3 + 2 * c2) * 8 : lds + kWgLds;
      *reinterpret_cast<u32x2*>(dst) = lo;
      *reinterpret_cast<u32x2*>(dst + 8) = hi;
    }
    uint8_t* D = B + kBufBytes;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = tid + u * kStThreads, row = c >> 3, ch = c & 7;
      const int h = row >> 7, ow = row & 127;
      const bool ok = ow < g.OW && oh0 + h < g.OH;  // pixels past the image: zero gradient rows
      *reinterpret_cast<u32x4*>(D + row * kSDY * 2 + ch * 16) = ok ? dv[u] : u32x4{0u, 0u, 0u, 0u};
    }
  };

  // transposed-read roles: group gq of 16 lanes, lane 4 q + p -> pixel row q, columns 4 p .. + 3
  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int cho = 16 * (gq & 1) + 4 * p4, rwo = 8 * (gq >> 1) + q4;
  f32x16 acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int kb = 0; kb < 7; ++kb) acc[i][kb] = f32x16{};

  auto compute = [&](int buf) {
    const uint8_t* B = lds + buf * kWgBuf;
    const uint8_t* D = B + kBufBytes;
#pragma unroll
    for (int u = 0; u < kTPix / 16 / 4; ++u) {
      const int ks = wave + 4 * u;
      const int t1 = 16 * ks + rwo, t2 = t1 + 4;  // this lane's two pixel rows
      bf16x8 fa[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i] = scat8(str4(D + (t1 * kSDY + 32 * i + cho) * 2), str4(D + (t2 * kSDY + 32 * i + cho) * 2));
      const int h1 = t1 >> 7, h2 = t2 >> 7;
      int w1 = t1 & 127, w2 = t2 & 127;
      w1 = w1 < g.OW ? w1 : g.OW - 1;  // (zero dy rows there: any in-image x will do)
      w2 = w2 < g.OW ? w2 : g.OW - 1;
      const uint8_t* x1 = B + 2 * h1 * rowb + 16 * w1 + 2 * cho;
      const uint8_t* x2 = B + 2 * h2 * rowb + 16 * w2 + 2 * cho;
#pragma unroll
      for (int kb = 0; kb < 7; ++kb) {
        const bf16x8 fb = scat8(str4(x1 + kb * rowb), str4(x2 + kb * rowb));
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][kb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb, acc[i][kb], 0, 0, 0);
      }
    }
  };

  if (t_lo < t_hi) {
    load(t_lo);
    store(t_lo, 0);
    __syncthreads();
    for (int t = t_lo; t < t_hi; ++t) {
      const int buf = (t - t_lo) & 1;
      load(t + 1 < t_hi ? t + 1 : t);  // unconditional: see stem_fwd_kernel
      asm volatile("" ::: "memory");    // keep the loads ahead of the tile's LDS reads / MFMAs
      compute(buf);
      store(t + 1 < t_hi ? t + 1 : t, buf ^ 1);
      __syncthreads();
    }
  }
  // the 4 waves' partials, summed in wave order: D[co][slot], lane -> slot 32 kb + (lane & 31),
  // accumulator e -> channel 32 i + (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  float* red = reinterpret_cast<float*>(lds);
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kb = 0; kb < 7; ++kb)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int co = 32 * i + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
            const int idx = co * 224 + 32 * kb + (lane & 31);
            red[idx] = (w == 0 ? 0.f : red[idx]) + acc[i][kb][e];
          }
    }
    __syncthreads();
  }
  float* dst = part + (int64_t)blockIdx.x * 64 * 224;
  for (int i = tid * 4; i < 64 * 224; i += kStThreads * 4)
    *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(red + i);
}

// out[co][r][s][c] (fp32, [64][7][7][3]) = sum over the G partial rows of
// part[g][co][32 r + 4 s + c].  A block owns 32 consecutive part columns; its 8 row
// groups each sum rows rg, rg + 8, ... (8 loads in flight), then the groups are added
// in order 0..7 through LDS (fixed order: deterministic).  The one-thread-per-output
// form walked all G = 256 rows 4 loads at a time: 64 dependent round trips, 23 us a
// step (profiles/r5_final/kernel_stats_rn50.csv).
constexpr int kRedCols = 32, kRedGroups = 256 / kRedCols;
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                               int G) {
  __shared__ float sh[kRedGroups][kRedCols];
  const int cl = threadIdx.x % kRedCols, rg = threadIdx.x / kRedCols;
  const int col = blockIdx.x * kRedCols + cl;  // < 64 * 224 (grid = 14336 / 32)
  const float* p = part + col;
  float a = 0.f;
  int k = rg;
  for (; k + 7 * kRedGroups < G; k += 8 * kRedGroups) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(k + u * kRedGroups) * 14336];
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  for (; k < G; k += kRedGroups) a += p[(int64_t)k * 14336];
  sh[rg][cl] = a;
  __syncthreads();
  if (rg != 0) return;
  for (int q = 1; q < kRedGroups; ++q) a += sh[q][cl];
  const int co = col / 224, j = col - co * 224, r = j >> 5, s = (j >> 2) & 7, c = j & 3;
  if (r < 7 && s < 7 && c < 3) out[co * 147 + r * 21 + s * 3 + c] = a;
}

int st_cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace

bool stem_ok(const StemGeom& g) {
  return g.N > 0 && g.H > 0 && g.W > 0 && g.W % 2 == 0 && g.W <= kMaxW && g.OH == (g.H - 1) / 2 + 1 &&
         g.OW == (g.W - 1) / 2 + 1 && g.OW <= 128 && (g.W >> 1) * kRowsIn <= kNP * kStThreads &&
         (int64_t)g.N * g.H * g.W * 3 < (1ll << 31) && (int64_t)g.N * g.OH * g.OW * 64 < (1ll << 40);
}

int stem_grid(const StemGeom& g) {
  const int ntile = g.N * ((g.OH + kT - 1) / kT);
  const int cu = st_cu_count();
  return ntile < cu ? ntile : cu;
}

bool launch_stem_wgrad(const uint16_t* x, const uint16_t* dy, float* part, float* dw, const StemGeom& g,
                       hipStream_t s) {
  if (!stem_ok(g)) return false;
  const int G = stem_grid(g);
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(G), dim3(kStThreads), 0, s, x, dy, part, g);
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(64 * 224 / kRedCols), dim3(256), 0, s, part, dw, G);
  return true;
}

bool launch_stem_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, const StemGeom& g,
                     hipStream_t s) {
  if (!stem_ok(g)) return false;
  const dim3 grid(stem_grid(g)), block(kStThreads);
  if (part)
    hipLaunchKernelGGL((stem_fwd_kernel<true>), grid, block, 0, s, x, w, y, part, g);
  else
    hipLaunchKernelGGL((stem_fwd_kernel<false>), grid, block, 0, s, x, w, y, part, g);
  return true;
}

}  // namespace rla
