// 3x3 / stride 1 / pad 1 NHWC bf16 convolution on the MFMA units (gfx950):
//
//   y[n][oh][ow][co] = sum over r, s, ci of x[n][oh + r - 1][ow + s - 1][ci] * w[co][r][s][ci]
//
// ResNet-50's bottleneck conv2 (13 of its 16 3x3 layers are stride 1).  The same
// kernel is the layer's input gradient: dx = conv3x3(dy, w') with
// w'[ci][r][s][co] = w[co][2 - r][2 - s][ci] (ops/conv.py builds w').  Why a kernel
// of our own (profiles/r3_final/kernel_stats_rn50.csv): the library forward and
// data-gradient kernels of these layers run at ~300-550 TFLOP/s, and MIOpen's dgrad
// adds SubTensorOp / fill passes around them; every one of these layers is the
// same 29.6 GFLOP at batch 128, so the whole family is ~0.95 TFLOP per step.
//
// Implicit GEMM  D[co][m] = W[co][(tap, ci)] . X[(tap, ci)][m]  over m = output pixel:
//   * workgroup = 4 waves, tile = 256 consecutive output pixels x 64 output channels;
//     wave w owns pixels [64 w, 64 w + 64) x all 64 channels = 2 x 2 blocks of
//     v_mfma_f32_32x32x16_bf16 (A = weights: co x ci, B = pixels: ci x m);
//   * the reduction runs in chunks of 16 input channels (one MFMA k-step per tap);
//     a chunk's operands are staged in LDS: the x HALO image of the tile -- every
//     input row the 256 pixels touch, in a virtual padded layout [n][H + 2][W + 2]
//     whose zero rows / columns ARE the padding -- and the 9 taps x 64 channels of w.
//     Tap (r, s) of pixel (n, oh, ow) reads halo row (n (H + 2) + oh + r - v0),
//     column ow + s: every tap is a per-lane address into the SAME image, so x is
//     fetched once per chunk instead of once per tap (an im2col would read it 9x);
//   * LDS rows are 48 B (16 channels + 16 B pad): ds_read_b128 of 32 consecutive
//     pixels (or channels) lands on 16 distinct 16-B bank windows (3 is odd), i.e.
//     conflict-free (MI355X_MICROARCH.md, ds_read_b128 lane groups);
//   * two LDS buffers and two register sets: chunk k + 1 goes from registers to the
//     other buffer while chunk k is multiplied, chunk k + 3 is in flight from HBM/L2;
//     one barrier per chunk.  Loads are unconditional (masked chunks read a clamped
//     in-image address and store zeros) so the compiler cannot sink them;
//   * grid in an XCD-aware order: the output-channel tiles of one pixel tile and
//     neighbouring pixel tiles run on the same XCD, so the halo / weight re-reads hit
//     that XCD's L2.
// Epilogue: D of 32x32x16 gives a lane one pixel and 4 consecutive output channels
// per 4 accumulator values; a v_permlane32_swap between the two half-waves (same
// pixel) turns two 8-byte stores into one 16-byte store (round 5).
// Requires Cin % 16 == 0, Cout % 64 == 0, 16-byte aligned bases (checked by the binding).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace rla {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kCvThreads = 256;
constexpr int kTMMax = 512;     // output pixels per workgroup tile: 128 x JB (JB pixel blocks of 32 per wave)
constexpr int kTN = 64;         // output channels per workgroup tile
constexpr int kKC = 16;         // reduction channels per chunk (one k-step of 16)
constexpr int kRow = 24;        // bf16 per halo / weight row: 16 channels + 8 pad (48 B)
constexpr int kFRow = 96;       // FLIP weight rows: 64 output channels + 32 pad (wgrad's tr-read image)
constexpr int kWPieces = 9 * kTN * 2;  // 16-byte pieces of a chunk's weights (both layouts)
constexpr int kNW = (kWPieces + kCvThreads - 1) / kCvThreads;
constexpr int kMaxNX = 7;       // halo pieces per thread (host checks the shape fits)
// LDS buffer: halo rows for kMaxNX pieces per thread, then the weights (kNW pieces
// per thread in either layout); every thread's stores land in it unconditionally
// (surplus pieces go to unused rows), so no load is used only under a branch (the
// compiler would sink it to the use)
constexpr int kXElems = kMaxNX * kCvThreads / 2 * kRow;
constexpr int kWElems = (kNW * kCvThreads / 2 * kRow) > (kNW * kCvThreads / 8 * kFRow)
                            ? (kNW * kCvThreads / 2 * kRow) : (kNW * kCvThreads / 8 * kFRow);
constexpr int kBufElems = kXElems + kWElems;
static_assert(2 * kBufElems * 2 >= 4 * 32 * 2 * 65 * 4, "ST reduction image fits the halo buffers");
// Compile-time-shape instances pad every halo row by kHPad elements (160 B = 40 banks):
// the row stride is then 12 W dwords mod 64, so 32 consecutive output pixels that
// wrap into the next image row keep the bank sequence of one row (in the plain
// [W + 2] layout the wrap shifts it by 24 dwords and a ds_read_b128 lane group
// collides: modelled 1.3-1.9x the conflict-free LDS cycles of the pixel reads,
// profiles/r5_pmc).  Run-time-shape instances keep the unpadded layout.
constexpr int kHPad = 80;
__host__ __device__ constexpr int halo_rows_max(int nx, int wc) { return nx * kCvThreads / 2 / (wc + 2) + 1; }
__host__ __device__ constexpr int x_elems(int nx, int wc) {
  return wc == 0 ? kXElems
                 : (nx * kCvThreads / 2 * kRow + kHPad * halo_rows_max(nx, wc) > kXElems
                        ? nx * kCvThreads / 2 * kRow + kHPad * halo_rows_max(nx, wc) : kXElems);
}

__device__ __forceinline__ bf16x4 tr4(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(p));
}

template <int NX>
struct CvSet {
  u32x4 x[NX], w[kNW];
  uint32_t ok;  // bit i: x[i] valid (weights are always in range)
};

// FLIP (input gradient): w is the FORWARD weight [Cr][3][3][Co] of the layer whose
// input gradient this is -- Cr (= g.Cin here) its output channels, Co (= g.Cout)
// its input channels -- read as w'[co][t][k] = w[k][8 - t][co] with no re-layout
// kernel: a chunk's pieces are 8 consecutive co of one (k, tap) row, staged as
// [tap][k][co] and read as A fragments by transposed LDS reads (ds_read_b64_tr_b16).
//
// Persistent: one workgroup per CU, each walks its tiles' chunks as ONE stream -- the
// next tile's first chunks are in flight while this tile's last ones are multiplied
// and its results stored -- so the per-tile pipeline fill is paid once per workgroup.
// Work split (round 5): workgroup g owns output-channel block g % tiles_n and the
// (g / tiles_n)-th of wpb EQUAL contiguous pixel ranges of it, tiled by TM with a
// shorter last tile.  Whole tiles dealt over the CUs left the last round mostly idle
// on every ResNet shape: 784 tiles = 3.06 rounds of 256 at 56x56 and 28x28, 392 =
// 1.53 at 14x14, 200 tiles on 256 CUs at 7x7 -- a 22-24 % makespan loss.  With
// tiles_n = 8 (7x7) each XCD (block g runs on XCD g % 8) holds one weight block.
//
// ST (round 5, forward only): the next BatchNorm's batch statistics in the epilogue.
// A workgroup owns one 64-channel block, so each lane keeps the sums and sums of
// squares of its 32 channels' bf16-rounded outputs in registers over all its tiles;
// at the end the 4 waves x 32 pixel lanes are reduced through LDS in a fixed order
// into row `jr` of part [wpb][2][Cout] (bn_finalize's layout; deterministic), so
// the BatchNorm skips its own partial pass over y (one full read of the output).
//
// WC / CC (round 5): the image width and input channels as compile-time constants
// (0 = run time) for the shapes that matter (ResNet's 56/64, 28/128, 14/256, 7/512):
// each tap's halo offset (r (W + 2) + s) rows is then an immediate of the ds_read
// (one per-lane base per pixel block, set per tile, instead of a multiply-add per
// tap and block), and a stage's tile / chunk split is a shift.  Global loads take
// 32-bit byte offsets from the SGPR base (saddr form: no 64-bit address math).
// PRE (round 6, forward only): x is the raw input of a deferred BatchNorm + ReLU (ResNet's
// bn1 -> conv2, ops/bn.py DeferredApply): every in-image halo piece is staged as
// bf16(relu(x * scale + shift)) -- bn_apply_kernel's exact expression -- on its way from
// registers to LDS; the zero padding stays zero (the conv pads the ACTIVATION).  A
// thread's pieces all hold channel half (tid & 1) of the stage's 16-channel chunk, so
// each store reads 8 scales and 8 shifts from a per-workgroup LDS table.
constexpr int kPreMaxC = 512;
template <int NX, bool FLIP, int JB, int DEPTH, int WC = 0, int CC = 0, bool ST = false, bool PRE = false>
__global__ __launch_bounds__(kCvThreads) void conv3x3_kernel(const uint16_t* __restrict__ x,
                                                             const uint16_t* __restrict__ w,
                                                             uint16_t* __restrict__ y, Conv3x3Geom g,
                                                             float* __restrict__ part,
                                                             const float* __restrict__ pre_ss = nullptr,
                                                             int64_t* __restrict__ nbt_inc = nullptr) {
  static_assert(!(ST && FLIP), "statistics are a forward epilogue");
  static_assert(!(PRE && FLIP), "PRE is a forward variant");
  constexpr int XE = x_elems(NX, WC), BE = XE + kWElems;  // halo / whole buffer elements
  static_assert(2 * BE * 2 <= 160 * 1024, "two LDS buffers fit the CU's 160 KiB");
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * BE];
  // [channel][scale, shift] interleaved: one 16-byte read covers a word's two channels
  __shared__ __attribute__((aligned(16))) float pre_tab[PRE ? 2 * kPreMaxC : 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (WC) g.W = WC;
  if (CC) g.Cin = CC;
  if constexpr (PRE) {
    if (nbt_inc && blockIdx.x == 0 && tid == 0) nbt_inc[0] += 1;
    for (int i = tid; i < g.Cin; i += kCvThreads) {
      pre_tab[2 * i] = pre_ss[2 * g.Cin + i];
      pre_tab[2 * i + 1] = pre_ss[3 * g.Cin + i];
    }
    // visible to every thread before the first store (the prologue's barrier follows it)
  }
  const int WP = g.W + 2, HP = g.H + 2;
  const int RS = WC ? (WC + 2) * kRow + kHPad : WP * kRow;  // halo row stride (elements)
  // padded layout: LDS element offset of this thread's halo piece i (the same every chunk)
  uint32_t xlds[WC ? NX : 1];
  if constexpr (WC != 0) {
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int p = tid + i * kCvThreads, pix = p >> 1;
      const int vr = pix / WP, q = pix - vr * WP;
      xlds[i] = (uint32_t)(vr * RS + q * kRow + (p & 1) * 8);
    }
  }
  const int64_t M = (int64_t)g.N * g.H * g.W;
  const int hw = g.H * g.W;
  constexpr int TM = 128 * JB;
  const int tiles_n = g.Cout / kTN;
  if ((int)blockIdx.x >= g.wpb * tiles_n) return;  // (uniform)
  const int nblk = (int)blockIdx.x % tiles_n, jr = (int)blockIdx.x / tiles_n;
  const int64_t p_lo = M * jr / g.wpb, p_hi = M * (jr + 1) / g.wpb;  // this workgroup's pixels
  const int ntiles = (int)((p_hi - p_lo + TM - 1) / TM);
  if (ntiles == 0) return;
  const int nchunks = g.Cin / kKC;
  const int nst = ntiles * nchunks;
  const int xpieces = g.vrows * WP * 2;  // 16-byte pieces of a chunk's halo image

  // this workgroup's tile of stream stage `st` (clamped: stages past the end re-load the last one)
  auto tile_of = [&](int st, int* chunk) {
    const int sc = st < nst ? st : nst - 1;
    const int i = sc / nchunks;
    *chunk = sc - i * nchunks;
    return i;
  };
  // tile i: pixels [m0, m_end) (m_end - m0 <= TM; the last tile of the range is shorter)
  auto tile_org = [&](int tile, int64_t* m0, int* co0, int* v0, int64_t* m_end = nullptr) {
    *co0 = nblk * kTN;
    *m0 = p_lo + (int64_t)tile * TM;
    if (m_end) *m_end = *m0 + TM < p_hi ? *m0 + TM : p_hi;
    const int n0 = (int)(*m0 / hw), oh0 = (int)((*m0 - (int64_t)n0 * hw) / g.W);
    *v0 = n0 * HP + oh0;  // first virtual halo row (the padded layout [n][H + 2][W + 2])
  };

  // Load-side tile state: every thread's piece offsets (elements, without the
  // chunk's channel offset) and halo validity, computed once per tile -- the
  // per-chunk loads are then one add each.  (Recomputing the halo geometry per
  // chunk cost two runtime integer divisions per piece, ~1K VALU cycles a stage at
  // one wave per SIMD: the MFMAs ran at ~15 % of the step, profiles/r4_rn.)
  int ld_tile = -1;
  uint32_t xoff[NX], woff[kNW];  // byte offsets from x / w
  uint32_t xok = 0u;
  auto load_geom = [&](int tile) {
    int64_t m0;
    int co0, v0;
    tile_org(tile, &m0, &co0, &v0);
    xok = 0u;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int p = tid + i * kCvThreads;
      const int pc = p < xpieces ? p : xpieces - 1;
      const int pix = pc >> 1, h = pc & 1;
      const int vr = pix / WP, q = pix - vr * WP;
      const int v = v0 + vr;
      const int n = v / HP, ih = v - n * HP - 1, iw = q - 1;
      const bool ok = p < xpieces && n < g.N && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const int nc = n < g.N ? n : g.N - 1;
      const int ihc = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih), iwc = iw < 0 ? 0 : (iw >= g.W ? g.W - 1 : iw);
      xoff[i] = (uint32_t)(((nc * g.H + ihc) * g.W + iwc) * g.Cin + h * 8) * 2u;
      xok |= ok ? (1u << i) : 0u;
    }
#pragma unroll
    for (int i = 0; i < kNW; ++i) {
      const int p = tid + i * kCvThreads;
      const int pc = p < kWPieces ? p : kWPieces - 1;
      if (FLIP) {
        // piece = (tap, k, group of 8 co): w[ci0 + k][8 - tap][co0 + 8 grp]
        const int tap = pc >> 7, k = (pc >> 3) & 15, grp = pc & 7;
        woff[i] = (uint32_t)((k * 9 + (8 - tap)) * g.Cout + co0 + grp * 8) * 2u;
      } else {
        const int h = pc & 1, rest = pc >> 1, co = rest % kTN, tap = rest / kTN;
        woff[i] = (uint32_t)(((co0 + co) * 9 + tap) * g.Cin + h * 8) * 2u;
      }
    }
  };
  auto load = [&](CvSet<NX>& st, int stage) {
    int cc;
    const int tile = tile_of(stage, &cc);
    if (tile != ld_tile) {  // uniform: the stage stream crossed into a new tile
      load_geom(tile);
      ld_tile = tile;
    }
    const uint32_t ci0b = (uint32_t)(cc * kKC) * 2u;
    const uint32_t wstepb = FLIP ? ci0b * 9u * (uint32_t)g.Cout : ci0b;
    st.ok = xok;
    const char* xc = reinterpret_cast<const char*>(x);
    const char* wc = reinterpret_cast<const char*>(w);
#pragma unroll
    for (int i = 0; i < NX; ++i) st.x[i] = *reinterpret_cast<const u32x4*>(xc + (xoff[i] + ci0b));
#pragma unroll
    for (int i = 0; i < kNW; ++i) st.w[i] = *reinterpret_cast<const u32x4*>(wc + (woff[i] + wstepb));
  };
  auto store = [&](const CvSet<NX>& st, int buf, int chunk) {
    __bf16* X = lds + buf * BE;
    __bf16* Wt = X + XE;
    const u32x4 z = {0u, 0u, 0u, 0u};
    u32x4 xs[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) xs[i] = st.x[i];
    if constexpr (PRE) {
      // word by word (two channels), the coefficients read per word: the loop runs
      // between MFMA stages with every accumulator and fragment register live, so it
      // may hold only a few temporaries (16 coefficients at once spilled)
      const float* t = pre_tab + 2 * (chunk * kKC + (tid & 1) * 8);
#pragma unroll
      for (int wd = 0; wd < 4; ++wd) {
        const float4 c = *reinterpret_cast<const float4*>(t + 4 * wd);  // s0, f0, s1, f1
        const f32x2 sc = {c.x, c.z}, sf = {c.y, c.w};
#pragma unroll
        for (int i = 0; i < NX; ++i) xs[i][wd] = bn_relu_bf16x2(xs[i][wd], sc, sf);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {  // p >= xpieces: a row past the image, never read
      const int p = tid + i * kCvThreads;
      const uint32_t off = WC ? xlds[WC ? i : 0] : (uint32_t)((p >> 1) * kRow + (p & 1) * 8);
      *reinterpret_cast<u32x4*>(X + off) = (st.ok >> i) & 1u ? xs[i] : z;
    }
#pragma unroll
    for (int i = 0; i < kNW; ++i) {
      const int p = tid + i * kCvThreads;  // pieces past 9 taps land in unused rows
      if (FLIP)
        *reinterpret_cast<u32x4*>(Wt + (p >> 3) * kFRow + (p & 7) * 8) = st.w[i];
      else
        *reinterpret_cast<u32x4*>(Wt + (p >> 1) * kRow + (p & 1) * 8) = st.w[i];
    }
  };

  const int kg = (lane >> 5) * 8;  // k-group: channels 8 (lane / 32) .. + 7 of the chunk
  // transposed-read roles (FLIP A operand): group gq of 16 lanes, lane 4q+p -> row q, channels 4p..4p+3
  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int cho = 16 * (gq & 1) + 4 * p4, rwo = 8 * (gq >> 1) + q4;
  int bpos[JB];  // this lane's pixel of block j as an LDS element offset of tap (0, 0)
  auto set_tile = [&](int tile) {
    int64_t m0, m_end;
    int co0, v0;
    tile_org(tile, &m0, &co0, &v0, &m_end);
#pragma unroll
    for (int jb = 0; jb < JB; ++jb) {
      int64_t m = m0 + wave * (32 * JB) + jb * 32 + (lane & 31);
      if (m >= m_end) m = m_end - 1;  // past the tile: a duplicate, never stored
      const int n = (int)(m / hw), rem = (int)(m - (int64_t)n * hw);
      const int oh = rem / g.W, ow = rem - oh * g.W;
      bpos[jb] = (n * HP + oh - v0) * RS + ow * kRow + kg;
    }
  };

  f32x16 acc[2][JB];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < JB; ++j)
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[i][j][k] = 0.f;
  };

  // One wave per SIMD: nothing else hides an LDS read's latency, so tap t + 1's
  // fragments are read into the second register set while tap t's MFMAs run (round 5:
  // the straight form waited lgkmcnt(0) before every tap's MFMAs).  Not in the 512-pixel
  // statistics instances: their second fragment set spilled (172 B of scratch per lane
  // at 56x56, forward + statistics 65.6 -> 94.4 us).
  constexpr bool kPipe = !(ST && JB == 4);
  auto fetch = [&](const __bf16* X, const __bf16* Wt, int tap, bf16x8 (&fa)[2], bf16x8 (&fb)[JB]) {
    const int r = tap / 3, s = tap - (tap / 3) * 3;
    const int toff = r * RS + s * kRow;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (FLIP) {
        const __bf16* pa = Wt + (tap * 16 + rwo) * kFRow + i * 32 + cho;
        fa[i] = __builtin_shufflevector(tr4(pa), tr4(pa + 4 * kFRow), 0, 1, 2, 3, 4, 5, 6, 7);
      } else {
        fa[i] = *reinterpret_cast<const bf16x8*>(Wt + (tap * kTN + i * 32 + (lane & 31)) * kRow + kg);
      }
    }
#pragma unroll
    for (int j = 0; j < JB; ++j)  // toff: an immediate offset when WC is set
      fb[j] = *reinterpret_cast<const bf16x8*>(X + bpos[j] + toff);
  };
  auto compute = [&](int buf) {
    const __bf16* X = lds + buf * BE;
    const __bf16* Wt = X + XE;
    if constexpr (!kPipe) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int r = tap / 3, s = tap - (tap / 3) * 3;
        const int toff = r * RS + s * kRow;
        bf16x8 a[2], b[JB];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(Wt + (tap * kTN + i * 32 + (lane & 31)) * kRow + kg);
#pragma unroll
        for (int j = 0; j < JB; ++j) b[j] = *reinterpret_cast<const bf16x8*>(X + bpos[j] + toff);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < JB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      return;
    }
    bf16x8 fa[2][2], fb[2][JB];
    fetch(X, Wt, 0, fa[0], fb[0]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int cur = tap & 1;
      if (tap + 1 < 9) fetch(X, Wt, tap + 1, fa[cur ^ 1], fb[cur ^ 1]);
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of this tap's MFMAs
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
    }
  };

  // ST: this lane's channel sums [i][4 q + e] (channel i 32 + 8 q + 4 (lane >> 5) + e)
  float bs[2][16], bq[2][16];
  if constexpr (ST) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) bs[i][k] = bq[i][k] = 0.f;
  }

  // D[co][m]: lane -> pixel (lane & 31) of block j; accumulator k -> channel
  // (k & 3) + 8 (k >> 2) + 4 (lane >> 5) of block i
  auto epilogue = [&](int tile) {
    int64_t m0, m_end;
    int co0, v0;
    tile_org(tile, &m0, &co0, &v0, &m_end);
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int64_t m = m0 + wave * (32 * JB) + j * 32 + (lane & 31);
      // lanes l and l ^ 32 hold the same pixel (the swap stays in-pixel); one
      // v_permlane32_swap per dword of each channel-group pair (q, q + 1) gives lane
      // half (lane >> 5) channels 16 p + 8 (lane >> 5) .. + 8: 16-byte stores
      const bool ok = m < m_end;
      uint16_t* yo = y + (ok ? m : 0) * g.Cout + co0 + 8 * (lane >> 5);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        uint32_t v[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x4 b;
#pragma unroll
          for (int e = 0; e < 4; ++e) b[e] = (__bf16)acc[i][j][4 * q + e];
          if constexpr (ST) {
            if (ok) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float f = (float)b[e];  // the statistics of what BatchNorm reads
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

  // stage k of the stream: global -> register set k % DEPTH -> LDS buffer k & 1.  At
  // iteration `it` set (it + 1) % DEPTH holds stage it + 1 (issued DEPTH - 1
  // iterations earlier: the loads of DEPTH - 1 stages are in flight behind every
  // stage's MFMAs) and goes to the buffer the previous iteration finished reading;
  // the set is then reloaded with stage it + 1 + DEPTH.  One barrier per stage.
  auto step = [&](int it, int buf, CvSet<NX>& nxt) {
    int cc;
    const int tile = tile_of(it, &cc);
    if (cc == 0) {
      set_tile(tile);
      zero();
    }
    compute(buf);
    int ncc = 0;
    if constexpr (PRE) tile_of(it + 1, &ncc);  // the stored stage's chunk
    store(nxt, buf ^ 1, ncc);
    __syncthreads();
    load(nxt, it + 1 + DEPTH);
    if (cc == nchunks - 1) epilogue(tile);
  };
  CvSet<NX> sets[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(sets[d], d);
  if constexpr (PRE) __syncthreads();  // the coefficient table
  store(sets[0], 0, 0);
  __syncthreads();
  load(sets[0], DEPTH);
  for (int it = 0; it < nst; it += DEPTH) {  // unrolled by DEPTH: the register sets stay static
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (it + d >= nst) break;  // uniform
      step(it + d, d & 1, sets[(d + 1) % DEPTH]);
    }
  }
  if constexpr (ST) {
    // [wave][pixel lane][stat][64 channels], rows padded to 65 floats (lanes of one
    // write land on distinct banks); the halo buffers are dead after the last stage
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
    if (tid < 2 * kTN) {  // (stat, channel): 128 rows in a fixed order
      const int st = tid >> 6, c = tid & 63;
      float a = 0.f;
      for (int r = 0; r < 4 * 32; ++r) a += red[(2 * r + st) * kSR + c];
      part[((int64_t)jr * 2 + st) * g.Cout + nblk * kTN + c] = a;
    }
  }
}

}  // namespace

int conv3x3_vrows(const Conv3x3Geom& g) {
  // the most virtual halo rows any tile of the partition touches (g.wpb ranges of
  // M / wpb pixels, each cut into g.tm-pixel tiles from its own start)
  const int64_t M = (int64_t)g.N * g.H * g.W;
  const int hw = g.H * g.W, HP = g.H + 2, TM = g.tm;
  int best = 0;
  for (int j = 0; j < g.wpb; ++j) {
    const int64_t lo = M * j / g.wpb, hi = M * (j + 1) / g.wpb;
    for (int64_t m0 = lo; m0 < hi; m0 += TM) {
      const int64_t m1 = (m0 + TM < hi ? m0 + TM : hi) - 1;
      const int n0 = (int)(m0 / hw), oh0 = (int)((m0 % hw) / g.W);
      const int n1 = (int)(m1 / hw), oh1 = (int)((m1 % hw) / g.W);
      const int rows = (n1 * HP + oh1 + 2) - (n0 * HP + oh0) + 1;
      if (rows > best) best = rows;
    }
  }
  return best;
}

int conv3x3_pieces_per_thread(const Conv3x3Geom& g) {
  return (g.vrows * (g.W + 2) * 2 + kCvThreads - 1) / kCvThreads;
}

static int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

int conv3x3_wpb(int N, int H, int W, int Cout) {
  // one workgroup per CU: cu / tiles_n pixel ranges per output-channel block (at least one)
  const int tiles_n = Cout / kTN, cu = cu_count();
  const int64_t M = (int64_t)N * H * W;
  int64_t w = tiles_n > 0 ? cu / tiles_n : 1;
  if (w < 1) w = 1;
  if (w > (M + 31) / 32) w = (M + 31) / 32;  // ranges of at least 32 pixels
  return (int)w;
}

int conv3x3_pick_tm(int N, int H, int W, int Cout) {
  // 512-pixel tiles halve the weight / halo traffic per MFMA where a workgroup's range
  // holds at least 1.5 of them (ResNet-50: the 56x56 layers)
  const char* e = getenv("RLA_CONV3X3_TM");  // tests pin either tile size
  if (e && (e[0] == '2' || e[0] == '5')) return e[0] == '5' ? 512 : 256;
  const int64_t M = (int64_t)N * H * W;
  const int64_t per = M / conv3x3_wpb(N, H, W, Cout);
  return per >= 768 ? 512 : 256;
}

bool conv3x3_ok(const Conv3x3Geom& g) {
  // 32-bit element offsets into x, y and w (the kernel's per-tile piece tables)
  return g.N > 0 && g.H > 0 && g.W > 0 && g.Cin % kKC == 0 && g.Cout % kTN == 0 && g.vrows > 0 && g.wpb > 0 &&
         (g.tm == 256 || g.tm == 512) && conv3x3_pieces_per_thread(g) <= kMaxNX &&
         (int64_t)g.N * (g.H + 2) < (1ll << 30) &&
         (int64_t)g.N * g.H * g.W * (g.Cin > g.Cout ? g.Cin : g.Cout) < (1ll << 31) &&
         (int64_t)g.Cin * 9 * g.Cout < (1ll << 31);
}

// the compile-time-shape instance (WC, CC) when the layer is one of them and its halo
// needs exactly NX pieces per thread; false: use the run-time-shape kernel
struct C3Pre {
  const float* ss;
  int64_t* nbt;
};

template <int NX, bool FLIP, int JB, int DEPTH, int WC, int CC, bool ST, bool PRE>
static void launch_one(const uint16_t* x, const uint16_t* w, uint16_t* y, const Conv3x3Geom& g, hipStream_t st,
                       dim3 grid, float* part, const C3Pre& pre) {
  hipLaunchKernelGGL((conv3x3_kernel<NX, FLIP, JB, DEPTH, WC, CC, ST, PRE>), grid, dim3(kCvThreads), 0, st, x, w, y,
                     g, part, pre.ss, pre.nbt);
}

template <int NX, bool FLIP, int JB, int DEPTH, int WC, int CC, bool ST, bool PRE>
static bool launch_fixed(const uint16_t* x, const uint16_t* w, uint16_t* y, const Conv3x3Geom& g, hipStream_t st,
                         dim3 grid, float* part, const C3Pre& pre) {
  static const bool generic = getenv("RLA_CONV3X3_GENERIC") != nullptr;  // A/B switch: run-time-shape kernel
  if (generic || g.W != WC || g.Cin != CC || conv3x3_pieces_per_thread(g) > NX ||
      conv3x3_pieces_per_thread(g) < NX - 1)
    return false;
  launch_one<NX, FLIP, JB, DEPTH, WC, CC, ST, PRE>(x, w, y, g, st, grid, part, pre);
  return true;
}

template <bool FLIP, int JB, int DEPTH, bool ST, bool PRE>
static void launch_nx(const uint16_t* x, const uint16_t* w, uint16_t* y, const Conv3x3Geom& g, hipStream_t st,
                      dim3 grid, float* part, const C3Pre& pre) {
  // ResNet-50's stride-1 3x3 shapes (bottleneck conv2 forward; the input gradient of
  // the same layers reads dy with the same width and channel count).  Not with PRE:
  // those instances already hold every VGPR and AGPR, the transform's temporaries
  // spilled (732-1232 B of scratch per lane) -- PRE runs the run-time-shape kernel
  if constexpr (PRE) {
  } else if constexpr (JB == 4) {
    if (launch_fixed<7, FLIP, JB, DEPTH, 56, 64, ST, PRE>(x, w, y, g, st, grid, part, pre)) return;
    // 28x28: a workgroup's range is one whole image (784 pixels = a 512 + a 272 tile)
    if (launch_fixed<5, FLIP, JB, DEPTH, 28, 128, ST, PRE>(x, w, y, g, st, grid, part, pre)) return;
  } else {
    if (launch_fixed<4, FLIP, JB, DEPTH, 28, 128, ST, PRE>(x, w, y, g, st, grid, part, pre)) return;
    if (launch_fixed<4, FLIP, JB, DEPTH, 14, 256, ST, PRE>(x, w, y, g, st, grid, part, pre)) return;
    if (launch_fixed<4, FLIP, JB, DEPTH, 7, 512, ST, PRE>(x, w, y, g, st, grid, part, pre)) return;
  }
  switch (conv3x3_pieces_per_thread(g)) {
    case 1: case 2: case 3: case 4:
      launch_one<4, FLIP, JB, DEPTH, 0, 0, ST, PRE>(x, w, y, g, st, grid, part, pre);
      break;
    case 5:
      launch_one<5, FLIP, JB, DEPTH, 0, 0, ST, PRE>(x, w, y, g, st, grid, part, pre);
      break;
    case 6:
      launch_one<6, FLIP, JB, DEPTH, 0, 0, ST, PRE>(x, w, y, g, st, grid, part, pre);
      break;
    default:
      launch_one<7, FLIP, JB, DEPTH, 0, 0, ST, PRE>(x, w, y, g, st, grid, part, pre);
      break;
  }
}

bool conv3x3_pre_ok(const Conv3x3Geom& g) { return conv3x3_ok(g) && g.Cin <= kPreMaxC; }

bool launch_conv3x3(const uint16_t* x, const uint16_t* w, uint16_t* y, const Conv3x3Geom& g, bool flip,
                    hipStream_t st, float* part, const float* pre_ss, int64_t* nbt_inc) {
  if (!conv3x3_ok(g) || (flip && part) || (flip && pre_ss) || (pre_ss && !part) || (pre_ss && g.Cin > kPreMaxC))
    return false;
  // persistent: one workgroup per (pixel range, output-channel block) -- one per CU
  const dim3 grid((unsigned)(g.wpb * (g.Cout / kTN)));
  const C3Pre pre{pre_ss, nbt_inc};
  // 512-pixel tiles: twice the accumulators, so two register stages in flight.  A
  // deferred BatchNorm (pre_ss) comes with the statistics epilogue only (the ResNet path)
  if (g.tm == 512) {
    if (flip) launch_nx<true, 4, 2, false, false>(x, w, y, g, st, grid, nullptr, pre);
    else if (pre_ss) launch_nx<false, 4, 2, true, true>(x, w, y, g, st, grid, part, pre);
    else if (part) launch_nx<false, 4, 2, true, false>(x, w, y, g, st, grid, part, pre);
    else launch_nx<false, 4, 2, false, false>(x, w, y, g, st, grid, nullptr, pre);
  } else {
    if (flip) launch_nx<true, 2, 4, false, false>(x, w, y, g, st, grid, nullptr, pre);
    else if (pre_ss) launch_nx<false, 2, 4, true, true>(x, w, y, g, st, grid, part, pre);
    else if (part) launch_nx<false, 2, 4, true, false>(x, w, y, g, st, grid, part, pre);
    else launch_nx<false, 2, 4, false, false>(x, w, y, g, st, grid, nullptr, pre);
  }
  return true;
}

}  // namespace rla
