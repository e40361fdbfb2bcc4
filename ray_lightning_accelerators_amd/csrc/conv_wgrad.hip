// Weight gradient of NHWC bf16 convolutions on the MFMA units (gfx950).
//
//   dW[co][r][s][ci] = sum over m = (n, oh, ow) of dy[m][co] * x[n][oh*sh - ph + r][ow*sw - pw + s][ci]
//
// i.e. for every filter tap (r, s) a GEMM  dy^T . x_shifted  whose reduction
// dimension is the huge N*OH*OW row index and whose output is the small
// [Cout, Cin] weight slice.  Why a kernel of our own (profiles/r3_rn50):
// MIOpen's NHWC wrw solvers cost ~80 us per ResNet-50 1x1 layer whatever its
// size (an fp32 workspace zero-fill, split-K atomics, a bf16 -> fp32 cast kernel;
// 2-6x the HBM floor of reading dy and x once), and hipBLASLt's dy^T . x with
// K = N*H*W = 401,408 runs at ~650 us.  The work is HBM-bound (arithmetic
// intensity Cout*Cin/(Cout+Cin) <= 128 flop/B against ~300 at the MFMA/HBM
// ridge), so the design goal is one read of dy and x at full bandwidth:
//
//   * grid = output tiles x taps x S row splits, in an XCD-aware order (the tiles of
//     one split share an XCD's L2); a workgroup (4 waves) owns a
//     [TCO x TCI] output tile (4 wave tiles of 64x64, or fewer wave tiles with
//     the reduction split across the waves) over a contiguous range of rows;
//   * rows stream through LDS in stages of KB rows: every thread loads 16-byte
//     row chunks of dy / x (coalesced: the row-major NHWC rows ARE the GEMM's k
//     axis), two stages ahead in registers, and writes them to a double-buffered
//     LDS image [row][channel] padded by 64 B per row;
//   * both MFMA operands are k-strided in that image (k = row), so they are read
//     with ds_read_b64_tr_b16 (hardware transpose: lane i of a 16-lane group gets
//     channel i of 4 consecutive rows); two reads form one 8-row fragment of
//     v_mfma_f32_32x32x16_bf16.  The 64-B pad puts the 4 rows of a 32-lane half
//     on disjoint 16-bank windows (conflict-free);
//   * S > 1: fp32 partial tiles [S][Cout][taps][Cin], summed in split order by a
//     small reduce kernel (deterministic; no atomics, no zero-fill).
//
// Output layout [Cout][KH][KW][Cin] = the channels_last weight's memory order,
// so the fp32 result IS the master gradient (no cast, no re-layout).
// Requires Cout % 64 == 0, Cin % 64 == 0 and 16-byte aligned bases (checked by
// the binding).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "kernels.h"

namespace rla {
namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_b4;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWgThreads = 256;
constexpr int kWgPad = 32;  // bf16 elements (64 B) of padding per LDS row

__device__ __forceinline__ bf16x4 tr4(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4*)(p));
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// source row of x for output row m and tap (r, s), clamped into the image (a
// padding tap loads a neighbouring pixel: a valid address near the real loads,
// not one hot dummy row); *pad is set when the tap falls in the zero padding
template <bool GEN>
__device__ __forceinline__ int64_t x_row(int64_t m, const WgradGeom& g, int r, int s, bool* pad) {
  *pad = false;
  if (!GEN) return m;
  // 32-bit index math (the binding bounds every row count below 2^29)
  const int mi = (int)m, ohw = g.OH * g.OW;
  const int n = mi / ohw;
  const int rem = mi - n * ohw;
  const int oh = rem / g.OW, ow = rem - oh * g.OW;
  int ih = oh * g.sh - g.ph + r, iw = ow * g.sw - g.pw + s;
  *pad = ih < 0 || ih >= g.H || iw < 0 || iw >= g.W;
  ih = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih);
  iw = iw < 0 ? 0 : (iw >= g.W ? g.W - 1 : iw);
  return (int64_t)((n * g.H + ih) * g.W + iw);
}

// PRE: x is the raw input of a deferred BatchNorm + ReLU (ops/bn.py DeferredApply; the
// forward conv applied it to its operands, conv1x1.hip / conv3x3.hip PRE): each valid
// x chunk is staged as bf16(relu(x * scale + shift)) -- bn_apply_kernel's exact
// expression -- so the gradient is bitwise the one of the materialised activation;
// zero-padding taps (GEN) stay zero.  A thread's x chunks keep their channel columns
// across stages: 16 coefficients per chunk in registers, loaded once.
template <int WA, int WB, bool GEN, int DEPTH = 2, bool PRE = false>
__global__ __launch_bounds__(kWgThreads) void wgrad_kernel(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ x, float* __restrict__ out,
                                                           WgradGeom g, int64_t M, int64_t rows_per_split,
                                                           int tiles_co, int tiles_ci, int splits,
                                                           const float* __restrict__ pre_ss = nullptr) {
  constexpr int NWT = WA * WB;          // wave tiles per workgroup tile
  constexpr int KS = 4 / NWT;           // waves sharing one wave tile (reduction split)
  constexpr int KB = KS == 4 ? 64 : 32;  // rows per stage: every wave gets >= 1 k-step of 16
  constexpr int TCO = 64 * WA, TCI = 64 * WB;
  constexpr int SA = TCO + kWgPad, SB = TCI + kWgPad;
  constexpr int NA = KB * TCO / 8 / kWgThreads, NB = KB * TCI / 8 / kWgThreads;
  constexpr int STAGE = KB * (SA + SB);  // bf16 elements per LDS buffer
  constexpr int KSTEPS = KB / 16 / KS;   // k-steps of 16 rows per wave per stage
  static_assert(NA >= 1 && NB >= 1 && KSTEPS >= 1, "tile / stage shape");
  static_assert(2 * STAGE * 2 >= (KS - 1) * NWT * 4 * 16 * 64 * 4, "LDS reuse for the reduction");
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int taps = g.KH * g.KW;
  // XCD-aware order (1-D grid): workgroups are dispatched round-robin over the 8
  // XCDs, so hardware block L runs on XCD L % 8.  Logical block q = xcd * per + L / 8
  // (per = blocks per XCD) gives each XCD a contiguous run of (split, tile) pairs:
  // every tile x tap of one row split runs on the SAME XCD at about the same time,
  // and their re-reads of the split's dy / x rows hit that XCD's L2 instead of
  // going to HBM / the shared MALL once per tile.
  const int ntile = tiles_co * tiles_ci * taps;
  const int total = ntile * splits, per = (total + 7) / 8;
  const int lq = (int)(blockIdx.x % 8u) * per + (int)(blockIdx.x / 8u);
  if (lq >= total) return;  // padding blocks of the last XCD
  const int split = lq / ntile;
  int b = lq - split * ntile;
  const int tci = b % tiles_ci;
  b /= tiles_ci;
  const int tco = b % tiles_co;
  const int tap = b / tiles_co;
  const int r = tap / g.KW, s = tap - (tap / g.KW) * g.KW;
  const int co0 = tco * TCO, ci0 = tci * TCI;
  const int64_t mb = (int64_t)split * rows_per_split;
  const int64_t me = mb + rows_per_split < M ? mb + rows_per_split : M;
  const int nst = (int)((me - mb + KB - 1) / KB);

  // this thread's 16-byte chunks of a stage: dy rows (TCO channels) and x rows (TCI),
  // in one of two register sets (stage k lives in set k & 1: two stages in flight)
  // Branch-free: out-of-range rows (past the split, or zero padding of x) load a
  // valid clamped row and are zeroed at the LDS store through a validity mask, so
  // the waitcnt pass sees straight-line loads and waits only for the older set.
  struct Set {
    u32x4 a[NA], b[NB];
    uint32_t ok;  // bit i: a[i] valid; bit NA + i: b[i] valid
  };
  static_assert(NA + NB <= 32, "validity mask");
  auto load = [&](Set& st, int64_t m0) {
    st.ok = 0u;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + i * kWgThreads, row = c / (TCO / 8), col = (c % (TCO / 8)) * 8;
      const int64_t m = m0 + row;
      const bool ok = m < me;
      st.a[i] = *reinterpret_cast<const u32x4*>(dy + (ok ? m : mb) * g.Cout + co0 + col);
      st.ok |= ok ? (1u << i) : 0u;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * kWgThreads, row = c / (TCI / 8), col = (c % (TCI / 8)) * 8;
      const int64_t m = m0 + row;
      bool pad;
      const int64_t xr = x_row<GEN>(m < me ? m : mb, g, r, s, &pad);
      const bool ok = m < me && !pad;
      st.b[i] = *reinterpret_cast<const u32x4*>(x + xr * g.Cin + ci0 + col);
      st.ok |= ok ? (1u << (NA + i)) : 0u;
    }
  };
  float pre_sc[PRE ? NB : 1][8], pre_sf[PRE ? NB : 1][8];
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * kWgThreads, col = (c % (TCI / 8)) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pre_sc[i][e] = pre_ss[2 * g.Cin + ci0 + col + e];
        pre_sf[i][e] = pre_ss[3 * g.Cin + ci0 + col + e];
      }
    }
  }
  auto store = [&](const Set& st, int buf) {
    __bf16* A = lds + buf * STAGE;
    __bf16* B = A + KB * SA;
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + i * kWgThreads, row = c / (TCO / 8), col = (c % (TCO / 8)) * 8;
      *reinterpret_cast<u32x4*>(A + row * SA + col) = (st.ok >> i) & 1u ? st.a[i] : z;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * kWgThreads, row = c / (TCI / 8), col = (c % (TCI / 8)) * 8;
      u32x4 v = st.b[i];
      if constexpr (PRE) {
#pragma unroll
        for (int wd = 0; wd < 4; ++wd)
          v[wd] = bn_relu_bf16x2(v[wd], (f32x2){pre_sc[i][2 * wd], pre_sc[i][2 * wd + 1]},
                                 (f32x2){pre_sf[i][2 * wd], pre_sf[i][2 * wd + 1]});
      }
      *reinterpret_cast<u32x4*>(B + row * SB + col) = (st.ok >> (NA + i)) & 1u ? v : z;
    }
  };

  // wave tile and reduction share of this wave
  const int wt = wave % NWT, ks = wave / NWT;
  const int wco = (wt / WB) * 64, wci = (wt % WB) * 64;
  // transposed-read lane roles: group gq of 16 lanes; lane 4q+p addresses row q, channels 4p..4p+3
  const int gq = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int cho = 16 * (gq & 1) + 4 * p;  // channel offset inside a 32-channel block
  const int rwo = 8 * (gq >> 1) + q;      // row offset inside a 16-row k-step

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;

  auto compute = [&](int buf) {
    const __bf16* A = lds + buf * STAGE;
    const __bf16* B = A + KB * SA;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) {
      const int rw = (kk * KS + ks) * 16 + rwo;
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const __bf16* pa = A + rw * SA + wco + 32 * i + cho;
        fa[i] = cat8(tr4(pa), tr4(pa + 4 * SA));
        const __bf16* pb = B + rw * SB + wci + 32 * i + cho;
        fb[i] = cat8(tr4(pb), tr4(pb + 4 * SB));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };
  // stage `it` from LDS buffer it & 1 while stages it + 1 (set nxt, landing) and
  // it + 2 (set cur, issued here: cur's stage went to LDS one step earlier) are in
  // flight; then stage it + 1 goes to the other buffer, read last before the
  // previous barrier
  // Every load and store of the loop is unconditional (a split with an odd stage
  // count runs one all-zero stage more): a load whose value were used only inside
  // an `if` would be sunk by the compiler next to that use -- the LDS store that
  // waits for it -- and the prefetch would be lost.
  // DEPTH register sets: stage k lives in set k % DEPTH, so DEPTH - 1 stages are
  // in flight while one is computed (2: four measured no faster -- equal on 1x1,
  // up to 20 % slower on the strided / 3x3 generic shapes, profiles/r3_wgrad/wgrad_probe_depth4.log)
  auto step = [&](int it, Set& cur, Set& nxt) {
    load(cur, mb + (int64_t)(it + DEPTH) * KB);  // past the split's end: masked, harmless
    __builtin_amdgcn_sched_barrier(0);  // loads stay ahead of the MFMAs
    compute(it & 1);
    __builtin_amdgcn_sched_barrier(0);
    store(nxt, (it + 1) & 1);  // stage it + 1 (past the end: zeros, never read)
    __syncthreads();
  };
  Set st[DEPTH];
  const int nstd = (nst + DEPTH - 1) / DEPTH * DEPTH;
  if (nstd > 0) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) load(st[d], mb + (int64_t)d * KB);
    store(st[0], 0);
  }
  __syncthreads();
  for (int it = 0; it < nstd; it += DEPTH) {  // unrolled by DEPTH: the register sets stay static
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) step(it + d, st[d], st[(d + 1) % DEPTH]);
  }

  // reduction split: waves ks > 0 hand their tiles to ks == 0 through LDS (fixed order)
  if constexpr (KS > 1) {
    float* red = reinterpret_cast<float*>(lds);  // every wave passed the loop's last barrier
    if (ks > 0) {
      float* d = red + ((ks - 1) * NWT + wt) * 4 * 16 * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int k = 0; k < 16; ++k) d[((i * 2 + j) * 16 + k) * 64 + lane] = acc[i][j][k];
    }
    __syncthreads();
    if (ks > 0) return;
#pragma unroll
    for (int o = 1; o < KS; ++o) {
      const float* d = red + ((o - 1) * NWT + wt) * 4 * 16 * 64;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int k = 0; k < 16; ++k) acc[i][j][k] += d[((i * 2 + j) * 16 + k) * 64 + lane];
    }
  }

  // D of 32x32x16: column = lane & 31 (ci), row = (k & 3) + 8 (k >> 2) + 4 (lane >> 5) (co)
  float* o = out + (int64_t)split * ((int64_t)g.Cout * taps * g.Cin);
  const int64_t rs = (int64_t)taps * g.Cin;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ci = ci0 + wci + 32 * j + (lane & 31);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int co = co0 + wco + 32 * i + (k & 3) + 8 * (k >> 2) + 4 * (lane >> 5);
        o[co * rs + (int64_t)tap * g.Cin + ci] = acc[i][j][k];
      }
    }
}

// out = sum over splits of part[s]: a block owns kRedCols float4 columns; thread
// group j (of 256 / kRedCols) sums splits j, j + G, j + 2G, ... and the group sums
// are combined in group order through LDS -- a fixed order (deterministic), with
// S / G independent loads per thread instead of a serial chain of S.
constexpr int kRedCols = 16;
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                           int64_t n, int S) {
  constexpr int G = 256 / kRedCols;
  __shared__ float4 sh[G][kRedCols];
  const int c = threadIdx.x % kRedCols, j = threadIdx.x / kRedCols;
  const int64_t i = ((int64_t)blockIdx.x * kRedCols + c) * 4;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i < n) {
    int k = j;
    for (; k + 3 * G < S; k += 4 * G) {  // 4 loads in flight
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(part + (int64_t)(k + u * G) * n + i);
#pragma unroll
      for (int u = 0; u < 4; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
    }
    for (; k < S; k += G) {
      const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)k * n + i);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  sh[j][c] = acc;
  __syncthreads();
  if (j != 0 || i >= n) return;
  for (int g = 1; g < G; ++g) {
    const float4 v = sh[g][c];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  *reinterpret_cast<float4*>(out + i) = acc;
}


// ---------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 (ResNet's bottleneck conv2): all nine taps of a 64x64
// [Cout x Cin] tile in one workgroup, from ONE load of each dy row and a halo
// tile of x, instead of the generic kernel's nine independent (tap) GEMMs that
// each re-read dy and x.  A stage is 64 dy rows = R whole output image rows of
// OWP (>= OW, multiple of 16) pixels; the x tile holds the R + 2 input rows they
// touch, each with one zero pixel of padding on both sides (OWP + 2 pixels), so
// tap (r, s) of output pixel (j, p) reads x-tile row (j + r) * (OWP + 2) + p + s:
// a plain row offset of the same LDS image (transposed reads at any row).  Wave
// r (0..2) accumulates the three taps (r, 0..2) = 3 x 64x64 fp32 in AGPRs; wave 3
// only helps load.  Rows outside the image (halo, p >= OW, rows past OH) are
// zeros, so no tap needs a mask.
// PRE: as wgrad_kernel's (a deferred BatchNorm + ReLU on x, staged in-image only)
template <int OWP, bool PRE = false>
__global__ __launch_bounds__(kWgThreads) void wgrad3x3_kernel(const uint16_t* __restrict__ dy,
                                                              const uint16_t* __restrict__ x, float* __restrict__ out,
                                                              WgradGeom g, int stages_per_split, int tiles_co,
                                                              int tiles_ci, int splits,
                                                              const float* __restrict__ pre_ss = nullptr) {
  constexpr int R = 64 / OWP, XP = OWP + 2, XROWS = (R + 2) * XP;
  constexpr int SA = 64 + kWgPad, SB = 64 + kWgPad;
  constexpr int NA = 64 * 8 / kWgThreads;                    // dy chunks per thread
  constexpr int NB = (XROWS * 8 + kWgThreads - 1) / kWgThreads;  // x chunks per thread
  constexpr int BROWS = NB * kWgThreads / 8;                  // x-tile rows incl. the unused tail
  static_assert(OWP % 16 == 0 && 64 % OWP == 0 && NA + NB <= 32, "3x3 stage shape");
  __shared__ __attribute__((aligned(16))) __bf16 lds[64 * SA + BROWS * SB];
  __bf16* A = lds;
  __bf16* B = lds + 64 * SA;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntile = tiles_co * tiles_ci, total = ntile * splits, per = (total + 7) / 8;
  const int lq = (int)(blockIdx.x % 8u) * per + (int)(blockIdx.x / 8u);  // XCD-aware (see wgrad_kernel)
  if (lq >= total) return;
  const int split = lq / ntile, tile = lq - split * ntile;
  const int co0 = (tile / tiles_ci) * 64, ci0 = (tile % tiles_ci) * 64;
  const int RB = (g.OH + R - 1) / R, T = g.N * RB;
  const int s0 = split * stages_per_split;
  const int s1 = s0 + stages_per_split < T ? s0 + stages_per_split : T;

  struct Set {
    u32x4 a[NA], b[NB];
    uint32_t ok;
  };
  // Masked chunks load a CLAMPED in-image address next to the valid ones (already
  // in cache): a shared dummy address (e.g. the tensor base) would have every CU
  // hammer one L2 channel with its halo / padding / tail chunks.
  auto load = [&](Set& st, int stage) {
    const bool live = stage < s1;
    const int sc = stage < T ? stage : T - 1;
    const int n = sc / RB, oh0 = (sc - (sc / RB) * RB) * R;
    st.ok = 0u;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + i * kWgThreads, row = c >> 3, col = (c & 7) * 8;
      const int j = row / OWP, pp = row - (row / OWP) * OWP;
      const bool ok = live && pp < g.OW && oh0 + j < g.OH;
      const int oh = oh0 + j < g.OH ? oh0 + j : g.OH - 1, ow = pp < g.OW ? pp : g.OW - 1;
      st.a[i] = *reinterpret_cast<const u32x4*>(dy + ((int64_t)(n * g.OH + oh) * g.OW + ow) * g.Cout + co0 + col);
      st.ok |= ok ? (1u << i) : 0u;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * kWgThreads, ri = c >> 3, col = (c & 7) * 8;
      const int rc = ri < XROWS ? ri : XROWS - 1;
      const int jr = rc / XP, q = rc - (rc / XP) * XP;
      const int ih = oh0 - 1 + jr, iw = q - 1;
      const bool ok = live && ri < XROWS && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const int ihc = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih), iwc = iw < 0 ? 0 : (iw >= g.W ? g.W - 1 : iw);
      st.b[i] = *reinterpret_cast<const u32x4*>(x + ((int64_t)(n * g.H + ihc) * g.W + iwc) * g.Cin + ci0 + col);
      st.ok |= ok ? (1u << (NA + i)) : 0u;
    }
  };
  // PRE: every x chunk of this thread holds channels ci0 + 8 (tid & 7) .. + 8
  float pre_sc[PRE ? 8 : 1], pre_sf[PRE ? 8 : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pre_sc[e] = pre_ss[2 * g.Cin + ci0 + (tid & 7) * 8 + e];
      pre_sf[e] = pre_ss[3 * g.Cin + ci0 + (tid & 7) * 8 + e];
    }
  }
  auto store = [&](const Set& st) {
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + i * kWgThreads, row = c >> 3, col = (c & 7) * 8;
      *reinterpret_cast<u32x4*>(A + row * SA + col) = (st.ok >> i) & 1u ? st.a[i] : z;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + i * kWgThreads, ri = c >> 3, col = (c & 7) * 8;
      u32x4 v = st.b[i];
      if constexpr (PRE) {
#pragma unroll
        for (int wd = 0; wd < 4; ++wd)
          v[wd] = bn_relu_bf16x2(v[wd], (f32x2){pre_sc[2 * wd], pre_sc[2 * wd + 1]},
                                 (f32x2){pre_sf[2 * wd], pre_sf[2 * wd + 1]});
      }
      *reinterpret_cast<u32x4*>(B + ri * SB + col) = (st.ok >> (NA + i)) & 1u ? v : z;
    }
  };

  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int cho = 16 * (gq & 1) + 4 * p4, rwo = 8 * (gq >> 1) + q4;
  const int r = wave;  // tap row of this wave (wave 3: loads only)
  f32x16 acc[3][2][2];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[t][i][j][k] = 0.f;

  // The 12 (k-step, tap) products of a stage as one stream: the next product's
  // fragments are read while this one's MFMAs run (one wave per SIMD: nothing else
  // hides the transposed reads' latency; round 5, as in conv3x3.hip).
  auto rd_a = [&](int kk, bf16x8 (&fa)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const __bf16* pa = A + (kk * 16 + rwo) * SA + 32 * i + cho;
      fa[i] = cat8(tr4(pa), tr4(pa + 4 * SA));
    }
  };
  auto rd_b = [&](int kk, int t, bf16x8 (&fb)[2]) {
    const int j = kk * 16 / OWP, p0 = kk * 16 - j * OWP;
    const int xb = (j + r) * XP + p0 + t + rwo;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const __bf16* pb = B + xb * SB + 32 * jj + cho;
      fb[jj] = cat8(tr4(pb), tr4(pb + 4 * SB));
    }
  };
  auto compute = [&]() {
    if (r >= 3) return;  // wave-uniform
    bf16x8 fa[2][2], fb[2][2];
    rd_a(0, fa[0]);
    rd_b(0, 0, fb[0]);
#pragma unroll
    for (int q = 0; q < 12; ++q) {
      const int kk = q / 3, t = q - (q / 3) * 3;
      if (q + 1 < 12) {
        const int kn = (q + 1) / 3, tn = (q + 1) - ((q + 1) / 3) * 3;
        if (tn == 0) rd_a(kn, fa[kn & 1]);
        rd_b(kn, tn, fb[(q + 1) & 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          acc[t][i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[kk & 1][i], fb[q & 1][jj], acc[t][i][jj], 0, 0, 0);
    }
  };
  // one LDS image, two register sets: stage `it` goes to LDS while stage it + 1 is
  // in flight; stage it + 2 is issued before this stage's MFMAs.  Loads and stores
  // unconditional (stages past the split are masked zeros) so none is sunk.
  auto step = [&](int it, Set& cur) {
    store(cur);
    __syncthreads();
    load(cur, it + 2);
    __builtin_amdgcn_sched_barrier(0);
    compute();
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };
  Set sa, sb;
  load(sa, s0);
  load(sb, s0 + 1);
  for (int it = s0; it < s1; it += 2) {
    step(it, sa);
    step(it + 1, sb);
  }

  if (r >= 3) return;
  float* o = out + (int64_t)split * ((int64_t)g.Cout * 9 * g.Cin);
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int ci = ci0 + 32 * jj + (lane & 31);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int co = co0 + 32 * i + (k & 3) + 8 * (k >> 2) + 4 * (lane >> 5);
          o[((int64_t)co * 9 + r * 3 + t) * g.Cin + ci] = acc[t][i][jj][k];
        }
      }
}

template <int WA, int WB>
void launch_tile(const uint16_t* dy, const uint16_t* x, float* out, const WgradGeom& g, int64_t M, int64_t rps,
                 int S, bool gen, hipStream_t st, const float* pre_ss) {
  const int tco = g.Cout / (64 * WA), tci = g.Cin / (64 * WB);
  const int total = tco * tci * g.KH * g.KW * S;
  const dim3 grid((unsigned)((total + 7) / 8 * 8)), block(kWgThreads);
  if (pre_ss && gen)
    hipLaunchKernelGGL((wgrad_kernel<WA, WB, true, 2, true>), grid, block, 0, st, dy, x, out, g, M, rps, tco, tci, S,
                       pre_ss);
  else if (pre_ss)
    hipLaunchKernelGGL((wgrad_kernel<WA, WB, false, 2, true>), grid, block, 0, st, dy, x, out, g, M, rps, tco, tci, S,
                       pre_ss);
  else if (gen)
    hipLaunchKernelGGL((wgrad_kernel<WA, WB, true>), grid, block, 0, st, dy, x, out, g, M, rps, tco, tci, S);
  else
    hipLaunchKernelGGL((wgrad_kernel<WA, WB, false>), grid, block, 0, st, dy, x, out, g, M, rps, tco, tci, S);
}

}  // namespace

bool wgrad3x3_ok(const WgradGeom& g) {
  return g.KH == 3 && g.KW == 3 && g.sh == 1 && g.sw == 1 && g.ph == 1 && g.pw == 1 && g.H == g.OH &&
         g.W == g.OW && g.OW <= 64;
}

int wgrad3x3_owp(int OW) { return OW <= 16 ? 16 : OW <= 32 ? 32 : 64; }

WgradPlan wgrad_plan(const WgradGeom& g, int splits, int algo) {
  WgradPlan p{};
  if (algo != 1 && wgrad3x3_ok(g)) {
    // halo kernel: stages of 64 / OWP whole output rows, 64x64 tiles
    p.kind = 1;
    p.wa = p.wb = 1;
    const int R = 64 / wgrad3x3_owp(g.OW);
    const int64_t T = (int64_t)g.N * ((g.OH + R - 1) / R);
    const int64_t tiles = (int64_t)(g.Cout / 64) * (g.Cin / 64);
    int64_t S = splits;
    if (S <= 0) {
      // one workgroup per CU (424 registers per lane: one wave per SIMD) in ONE round:
      // 359 workgroups ran as 256 + 103 (profiles/r3_wgrad/pmc_halo.log: 33% MFMA-busy
      // waves, the second round on 40% of the chip)
      S = 256 / tiles;
      if (S > T / 4) S = T / 4;       // >= 4 stages per split
      // fp32 partials (9 taps) at most ~4x the dy + x bytes (the generic kernel
      // re-reads those 9x; the autotuner picks between the two).  Round 5 split sweep
      // (profiles/r5_wsplit): at 7x7x512 the old 2x cap left S = 2 and 64 of 256 CUs
      // busy, 205 us; S = 4 (3x the input bytes in partials) runs 123 us
      const double in_bytes = 2.0 * (double)g.N * g.OH * g.OW * (g.Cout + (double)g.Cin);
      const int64_t max_part = (int64_t)(4.0 * in_bytes / (4.0 * 9.0 * g.Cout * g.Cin));
      if (S > max_part) S = max_part;
    }
    if (S < 1) S = 1;
    int64_t sps = (T + S - 1) / S;
    sps = (sps + 1) & ~(int64_t)1;  // even: the loop runs stages in pairs
    p.rows_per_split = sps;
    p.splits = (int)((T + sps - 1) / sps);
    return p;
  }
  p.kind = 0;
  // workgroup tile (in 64-channel wave tiles): 4 wave tiles when the weight is
  // big enough, with the larger side along the larger channel count
  if (g.Cout % 128 == 0 && g.Cin % 128 == 0) { p.wa = 2; p.wb = 2; }
  else if (g.Cout % 256 == 0) { p.wa = 4; p.wb = 1; }
  else if (g.Cin % 256 == 0) { p.wa = 1; p.wb = 4; }
  else if (g.Cout % 128 == 0) { p.wa = 2; p.wb = 1; }
  else if (g.Cin % 128 == 0) { p.wa = 1; p.wb = 2; }
  else { p.wa = 1; p.wb = 1; }
  const int64_t M = (int64_t)g.N * g.OH * g.OW;
  const int kb = p.wa * p.wb == 1 ? 64 : 32;
  const int64_t tiles = (int64_t)(g.Cout / (64 * p.wa)) * (g.Cin / (64 * p.wb)) * g.KH * g.KW;
  int64_t S = splits;
  if (S <= 0) {
    // ~512 workgroups (2 per CU, the loads of 8 waves in flight per CU) ...
    S = (512 + tiles - 1) / tiles;
    // ... at least 4 stages per split, and fp32 partials (written, then re-read by
    // the reduce) of at most the bytes the tiles read.  (Half, before the round-5
    // split sweep, profiles/r5_wsplit: that cap left the small-M layers under-filled
    // -- 7x7 512 <-> 2048 at S = 3, 41 us vs 34 at S = 8; 14x14 1024 -> 2048 / 2 at
    // S = 2, 92 us vs 71 at S = 4.)
    const int64_t max_rows = M / (4 * kb);
    if (S > max_rows) S = max_rows;
    const double in_bytes = 2.0 * (double)M * (g.Cout + (double)g.Cin) * g.KH * g.KW;  // per-tap tiles
    const double part_bytes = 4.0 * (double)g.Cout * g.Cin * g.KH * g.KW;
    const int64_t max_part = (int64_t)(in_bytes / part_bytes);
    if (S > max_part) S = max_part;
  }
  if (S < 1) S = 1;
  int64_t rps = (M + S - 1) / S;
  rps = (rps + kb - 1) / kb * kb;
  p.rows_per_split = rps;
  p.splits = (int)((M + rps - 1) / rps);
  if (p.splits < 1) p.splits = 1;
  return p;
}

void launch_wgrad(const uint16_t* dy, const uint16_t* x, float* out, float* part, const WgradGeom& g,
                  const WgradPlan& p, hipStream_t st, const float* pre_ss) {
  const int64_t M = (int64_t)g.N * g.OH * g.OW;
  if (p.kind == 1) {
    float* dst = p.splits > 1 ? part : out;
    const int tco = g.Cout / 64, tci = g.Cin / 64, total = tco * tci * p.splits;
    const dim3 grid((unsigned)((total + 7) / 8 * 8)), block(kWgThreads);
    const int sps = (int)p.rows_per_split, owp = wgrad3x3_owp(g.OW);
#define RLA_W3(O)                                                                                           \
  do {                                                                                                      \
    if (pre_ss)                                                                                             \
      hipLaunchKernelGGL((wgrad3x3_kernel<O, true>), grid, block, 0, st, dy, x, dst, g, sps, tco, tci, p.splits, \
                         pre_ss);                                                                           \
    else                                                                                                    \
      hipLaunchKernelGGL((wgrad3x3_kernel<O, false>), grid, block, 0, st, dy, x, dst, g, sps, tco, tci,      \
                         p.splits);                                                                         \
  } while (0)
    if (owp == 16)
      RLA_W3(16);
    else if (owp == 32)
      RLA_W3(32);
    else
      RLA_W3(64);
#undef RLA_W3
  } else {
  const bool gen = !(g.KH == 1 && g.KW == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0 && g.H == g.OH &&
                     g.W == g.OW);
  float* dst = p.splits > 1 ? part : out;
  const int key = p.wa * 10 + p.wb;
  switch (key) {
    case 22: launch_tile<2, 2>(dy, x, dst, g, M, p.rows_per_split, p.splits, gen, st, pre_ss); break;
    case 41: launch_tile<4, 1>(dy, x, dst, g, M, p.rows_per_split, p.splits, gen, st, pre_ss); break;
    case 14: launch_tile<1, 4>(dy, x, dst, g, M, p.rows_per_split, p.splits, gen, st, pre_ss); break;
    case 21: launch_tile<2, 1>(dy, x, dst, g, M, p.rows_per_split, p.splits, gen, st, pre_ss); break;
    case 12: launch_tile<1, 2>(dy, x, dst, g, M, p.rows_per_split, p.splits, gen, st, pre_ss); break;
    default: launch_tile<1, 1>(dy, x, dst, g, M, p.rows_per_split, p.splits, gen, st, pre_ss); break;
  }
  }
  if (p.splits > 1) {
    const int64_t n = (int64_t)g.Cout * g.KH * g.KW * g.Cin;
    const int64_t blocks = (n / 4 + kRedCols - 1) / kRedCols;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, out, n, p.splits);
  }
}

}  // namespace rla
