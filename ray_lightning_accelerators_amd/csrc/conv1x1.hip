// 1x1 / stride-1 NHWC bf16 convolution forward WITH the following BatchNorm's
// batch statistics in its epilogue (gfx950).
//
//   y[m][n] = sum_k x[m][k] * w[n][k]          (m = output pixel, NHWC rows)
//   part[b][0][n] = sum over block b's pixels of bf16(y[m][n])
//   part[b][1][n] = the same of bf16(y[m][n])^2
//
// Why: every BatchNorm forward starts with a pass that only READS the conv output
// to sum it (bn_partial_kernel<0>, 53 launches / ~570 us per ResNet-50 step,
// profiles/r4_rn/kernel_stats_rn50.csv).  The 1x1 layers (36 of the 53) are GEMMs
// whose output tile is in registers anyway: summing it there deletes that pass --
// the largest of them re-read 205 MB.  bn_finalize then reduces `part` exactly as it
// reduces the partial kernel's rows (same [blocks, 2, C] fp32 layout).
//
// Both operands are K-contiguous rows (x: [M][K], w: [N][K]), the per-lane layout of
// v_mfma_f32_32x32x16_bf16's A and B operands (lane l: row l & 31, k = 8 (l >> 5) .. +8).
//   * workgroup = 4 waves = 2 (channel halves) x 2 (pixel halves); a wave owns
//     TNW x 32 channels x 64 pixels (TNW x 2 MFMA blocks), the workgroup 64 TNW
//     channels x 128 pixels per tile, and walks `tiles_per_blk` consecutive pixel
//     tiles (the statistics accumulate in registers across them: one partial row per
//     workgroup column);
//   * operands reach LDS by DMA (global_load_lds_dwordx4): a (tile, 32-channel chunk)
//     stage is 128 x rows and 64 TNW w rows of 64 B, stored 16-B-unit-major
//     ([k unit][row]) so the fragment reads -- 32 consecutive rows of one k unit per
//     half-wave -- are contiguous 512-B ds_read_b128 runs (conflict-free).  A ring of
//     NS buffers: the DMA of NS - 2 stages is in flight behind every stage's
//     MFMAs, across tile boundaries; each stage is retired by a COUNTED vmcnt (the
//     DMA is inline asm, invisible to hipcc's wait bookkeeping, and hipcc would
//     otherwise drain every in-flight load at each epilogue's stores) and one raw
//     barrier (cdna_hip_programming.md, pipelining across barriers);
//   * K <= 128 (the ResNet-50 layers this kernel wins): the workgroup's whole weight
//     block stays in LDS, DMA'd once ahead of stage 0, and the ring carries x only
//     (6 stages with a 16 KB block, 4 with 32 KB);
//   * D of 32x32x16 gives a lane one pixel and 4 consecutive channels per 4
//     accumulators; the rounded values go straight into the lane's per-channel sum /
//     sum of squares, and one v_permlane32_swap per dword pair widens the stores to
//     16 bytes; one butterfly over the 32 pixel lanes and a fixed-order LDS add over
//     the two pixel-half waves at the end (deterministic);
//   * grid: workgroups sharing pixel tiles (same x, all channel columns) run on the
//     same XCD, so x is read from HBM once and re-read from that XCD's L2.
// Rows past M read a clamped row (never stored, excluded from the sums); stages past
// the end re-load the last one, so every iteration issues the same DMA count.
// Requires K % 32 == 0, N % 64 == 0, 16-byte aligned bases (binding checks).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "kernels.h"

namespace rla {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kC1Threads = 256;
constexpr int kC1LdsBytes = 65536;  // ring (+ resident weights) per workgroup: 2 workgroups per CU

// 16 bytes per lane, global -> LDS, lane-linear from the wave-uniform LDS byte
// address `lds`; M0 saved and restored in the same statement (LDS-DMA recipe)
__device__ __forceinline__ void c1_dma16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}

// BWD: the same GEMM as an input gradient (x = the conv's output gradient dy1 [M][K],
// w = its weight transposed [N = Cin][K = Cout]) whose epilogue is the PREVIOUS
// BatchNorm's backward partial pass: with da = bf16(dy1 . W) for block-output pixel m
// and channel c, d = (da + dy2) * (yb > 0) -- dy2 the folded residual gradient, yb
// that BatchNorm's (ReLU) output -- is written once (bf16) in place of da, and the
// partial row sums d and d * xb (xb the BatchNorm's input), bn_partial_kernel<1>'s
// layout.  da is never written or re-read (ops/conv.py, fuse_bn_dgrad).  dy2 / yb / xb
// for a tile are loaded at its first stage, two stages ahead of the epilogue.
//
// PRE: x is the raw input of a BatchNorm + ReLU whose apply pass was deferred to this
// conv (ResNet's bn2 -> conv3, ops/bn.py ``defer``): every x fragment becomes
// bf16(relu(x * scale + shift)) after its LDS read -- the exact expression of
// bn_apply_kernel, so y is bitwise the unfused conv of the applied activation -- and
// the activation is never written (one read + one write of [M, K] less per layer).
// pre_ss is bn_finalize's [4, K] (rows 2 / 3: scale / shift), staged once into LDS;
// nbt_inc: num_batches_tracked += 1 (the apply kernel's job when the BatchNorm's
// statistics came from a conv epilogue).
constexpr int kPreMaxK = 512;
template <int TNW, bool WRES, int NS, bool BWD = false, bool PRE = false>
__global__ __launch_bounds__(kC1Threads, 2) void conv1x1_stats_kernel(const uint16_t* __restrict__ x,
                                                                      const uint16_t* __restrict__ w,
                                                                      uint16_t* __restrict__ y, int64_t M, int K,
                                                                      int N, int gx, int tiles_per_blk,
                                                                      float* __restrict__ part,
                                                                      const uint16_t* __restrict__ dy2 = nullptr,
                                                                      const uint16_t* __restrict__ yb = nullptr,
                                                                      const uint16_t* __restrict__ xb = nullptr,
                                                                      const float* __restrict__ pre_ss = nullptr,
                                                                      int64_t* __restrict__ nbt_inc = nullptr) {
  static_assert(!BWD || TNW == 1, "the backward epilogue's prefetch is sized for 32-channel wave columns");
  static_assert(!(BWD && PRE), "PRE is a forward variant");
  constexpr int BN = 64 * TNW;                      // workgroup channels
  constexpr int kXBytes = 4 * 128 * 16;             // x part of a stage: [4 k units][128 rows] x 16 B
  constexpr int kStageBytes = kXBytes + (WRES ? 0 : 4 * BN * 16);
  constexpr int kXInst = 8 / 4, kWInst = WRES ? 0 : BN / 16 / 4;  // DMA instructions per wave per stage
  constexpr int kDma = kXInst + kWInst;
  // WRES: the workgroup's whole weight block [K / 8 units][BN rows] stays in LDS (DMA'd
  // once, ahead of stage 0) and the ring carries x only
  constexpr int kWResBytes = WRES ? kC1LdsBytes - NS * kStageBytes : 0;
  static_assert(NS * kStageBytes + kWResBytes <= kC1LdsBytes, "LDS budget (2 workgroups per CU)");
  __shared__ __attribute__((aligned(16))) uint8_t ring[NS * kStageBytes + kWResBytes];
  __shared__ float red[2][2][BN];
  __shared__ __attribute__((aligned(16))) float pre_tab[PRE ? 2 * kPreMaxK : 4];  // [scale | shift]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if constexpr (PRE) {
    if (nbt_inc && blockIdx.x == 0 && tid == 0) nbt_inc[0] += 1;
    for (int i = tid; i < K; i += kC1Threads) {
      pre_tab[i] = pre_ss[2 * K + i];
      pre_tab[kPreMaxK + i] = pre_ss[3 * K + i];
    }
    __syncthreads();  // ahead of every DMA: the loop's counted waits see DMA only
  }
  const int wn = wave & 1, wm = wave >> 1, r = lane & 31, h = lane >> 5;
  // XCD-aware (x, y): hardware block b runs on XCD b % 8; the gy column blocks of a
  // pixel range x all sit on XCD x % 8 (gx is a multiple of 8)
  const int gy = N / BN;
  const int xcd = (int)(blockIdx.x % 8u), slot = (int)(blockIdx.x / 8u);
  const int bx = xcd + 8 * (slot / gy), by = slot % gy;
  const int mt = (int)((M + 127) / 128);
  const int t0 = bx * tiles_per_blk;
  const int ntiles = mt - t0 < tiles_per_blk ? mt - t0 : tiles_per_blk;
  const int nb = by * BN;  // workgroup's first channel
  float* prow = part + (int64_t)bx * 2 * N + nb;
  if (ntiles <= 0) {  // padding column of the XCD deal: an all-zero partial row
    for (int c = tid; c < BN; c += kC1Threads) {
      prow[c] = 0.f;
      prow[N + c] = 0.f;
    }
    return;
  }
  const int nch = K >> 5;
  const int nst = ntiles * nch;
  const uint32_t ring0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ring;
  const uint32_t wres0 = ring0 + NS * kStageBytes;

  // DMA of stage st into ring buffer st % NS: wave-instruction g of the x part
  // covers k unit g / 2, rows 64 (g & 1) .. +64; of the w part k unit g / (BN / 64)
  auto issue = [&](int st) {
    const int sc = st < nst ? st : nst - 1;
    const int ti = sc / nch, k = (sc - ti * nch) * 32;
    const uint32_t buf = ring0 + (uint32_t)(st % NS) * kStageBytes;
#pragma unroll
    for (int u = 0; u < kXInst; ++u) {
      const int g = wave * kXInst + u;
      int64_t m = (int64_t)(t0 + ti) * 128 + (g & 1) * 64 + lane;
      m = m < M ? m : M - 1;
      c1_dma16(x + m * K + k + 8 * (g >> 1), __builtin_amdgcn_readfirstlane(buf + g * 1024));
    }
#pragma unroll
    for (int u = 0; u < kWInst; ++u) {
      const int g = wave * kWInst + u;
      const int row = (g % (BN / 64)) * 64 + lane;
      c1_dma16(w + (int64_t)(nb + row) * K + k + 8 * (g / (BN / 64)),
               __builtin_amdgcn_readfirstlane(buf + kXBytes + g * 1024));
    }
  };

  f32x16 acc[TNW][2];
  float ssum[TNW][16], ssq[TNW][16];
#pragma unroll
  for (int t = 0; t < TNW; ++t) {
#pragma unroll
    for (int e = 0; e < 16; ++e) ssum[t][e] = ssq[t][e] = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[t][j] = f32x16{};
  }

  auto compute = [&](int st) {
    const uint8_t* buf = ring + (st % NS) * kStageBytes;
    const int ti = st / nch, c = st - ti * nch;
    const uint8_t* wb = WRES ? ring + NS * kStageBytes + c * 4 * BN * 16 : buf + kXBytes;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ku = 2 * ks + h;
      bf16x8 fa[TNW], fb[2];
#pragma unroll
      for (int t = 0; t < TNW; ++t)
        fa[t] = *reinterpret_cast<const bf16x8*>(wb + (ku * BN + wn * 32 * TNW + 32 * t + r) * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(buf + (ku * 128 + wm * 64 + 32 * j + r) * 16);
      if constexpr (PRE) {  // channels 32 c + 8 ku .. +8 of both pixel fragments
        const float* sc = pre_tab + c * 32 + ku * 8;
        const float4 s0 = *reinterpret_cast<const float4*>(sc), s1 = *reinterpret_cast<const float4*>(sc + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(sc + kPreMaxK);
        const float4 h1 = *reinterpret_cast<const float4*>(sc + kPreMaxK + 4);
        const f32x2 s2[4] = {{s0.x, s0.y}, {s0.z, s0.w}, {s1.x, s1.y}, {s1.z, s1.w}};
        const f32x2 f2[4] = {{h0.x, h0.y}, {h0.z, h0.w}, {h1.x, h1.y}, {h1.z, h1.w}};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          u32x4 u = __builtin_bit_cast(u32x4, fb[j]);
#pragma unroll
          for (int wd = 0; wd < 4; ++wd) u[wd] = bn_relu_bf16x2(u[wd], s2[wd], f2[wd]);
          fb[j] = __builtin_bit_cast(bf16x8, u);
        }
      }
#pragma unroll
      for (int t = 0; t < TNW; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[t], fb[j], acc[t][j], 0, 0, 0);
    }
  };

  const int cw = nb + wn * 32 * TNW;  // wave's first channel
  // BWD: dy2 / yb / xb of a tile's [2 pixel blocks][2 channel halves] 16-byte chunks
  typedef u32x4 PreSet[3][2][2];
  auto prefetch = [&](PreSet& pre, int ti) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int64_t m = (int64_t)(t0 + ti) * 128 + wm * 64 + 32 * j + r;
      m = m < M ? m : M - 1;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int64_t off = m * N + cw + 16 * p + 8 * h;
        pre[0][j][p] = *reinterpret_cast<const u32x4*>(dy2 + off);
        pre[1][j][p] = *reinterpret_cast<const u32x4*>(yb + off);
        pre[2][j][p] = *reinterpret_cast<const u32x4*>(xb + off);
      }
    }
  };
  // D[n][m]: lane -> pixel r of block j; accumulator 4q + e -> channel 8q + 4h + e.
  // Stores: one v_permlane32_swap per dword of each channel-group pair (q, q + 1)
  // gives lane h channels 16p + 8h .. +8 -- one 16-byte store where the MFMA layout
  // gives two 8-byte ones (cdna_hip_programming.md, widened epilogue stores)
  auto epilogue = [&](int ti, const PreSet& pre) {
    const int64_t m0 = (int64_t)(t0 + ti) * 128 + wm * 64 + r;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t m = m0 + 32 * j;
      const bool ok = m < M;  // lanes l and l ^ 32 share the pixel: the swap stays in-pixel
      uint16_t* yo = y + (ok ? m : 0) * N + cw + 8 * h;
#pragma unroll
      for (int t = 0; t < TNW; ++t) {
        uint32_t v[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x4 b;
#pragma unroll
          for (int e = 0; e < 4; ++e) b[e] = (__bf16)acc[t][j][4 * q + e];
          if (!BWD && ok) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float f = (float)b[e];
              ssum[t][4 * q + e] += f;
              ssq[t][4 * q + e] += f * f;
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
          if (BWD) {  // channels cw + 16p + 8h .. +8 of pixel m: the BatchNorm backward partial
            const bf16x8 da = __builtin_bit_cast(bf16x8, o);
            const bf16x8 g2 = __builtin_bit_cast(bf16x8, pre[0][j][p]);
            const bf16x8 ym = __builtin_bit_cast(bf16x8, pre[1][j][p]);
            const bf16x8 xm = __builtin_bit_cast(bf16x8, pre[2][j][p]);
            bf16x8 dd;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float a = (float)ym[k] > 0.f ? (float)da[k] + (float)g2[k] : 0.f;
              dd[k] = (__bf16)a;
              if (ok) {
                const float f = (float)dd[k];
                ssum[0][8 * p + k] += f;
                ssq[0][8 * p + k] += f * (float)xm[k];
              }
            }
            if (ok) *reinterpret_cast<bf16x8*>(yo + 16 * p) = dd;
          } else if (ok) {
            *reinterpret_cast<u32x4*>(yo + 32 * t + 16 * p) = o;
          }
        }
      }
#pragma unroll
      for (int t = 0; t < TNW; ++t) acc[t][j] = f32x16{};
    }
  };

  if (WRES) {  // the weight block, ahead of stage 0 (retired by stage 0's counted wait)
    const int ng = (K / 8) * (BN / 64);
    for (int g = wave; g < ng; g += 4) {
      const int row = (g % (BN / 64)) * 64 + lane;
      c1_dma16(w + (int64_t)(nb + row) * K + 8 * (g / (BN / 64)), __builtin_amdgcn_readfirstlane(wres0 + g * 1024));
    }
  }
#pragma unroll
  for (int d = 0; d < NS - 1; ++d) issue(d);
  if constexpr (!BWD) {
    PreSet none;
    for (int st = 0; st < nst; ++st) {
      // stage st landed: the DMA issued after it (NS - 2 stages) may still fly;
      // then every wave's part is in and every wave has finished reading buffer st - 1
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((NS - 2) * kDma) : "memory");
      issue(st + NS - 1);
      const int ti = st / nch;
      compute(st);
      if (st - ti * nch == nch - 1) epilogue(ti, none);
    }
  } else {
    // BWD (round 6): the epilogue operands of tile t + 1 are loaded at tile t's first
    // stage into the other of two register sets (the tile loop is unrolled by two, so
    // both sets stay in fixed registers).  Loaded at the tile's own first stage, as
    // before, they were the youngest loads when the epilogue needed them, and the
    // compiler's in-order wait for them also drained the DMA ring issued behind them
    // -- and its conservative wait before re-filling the one set drained it again:
    // the 401408 x 64 -> 256 layers ran at ~3.6 TB/s (profiles/r6_full).  The counted
    // stage wait now also counts the 12 operand loads of every prefetch issued after
    // the stage's DMA (vmcnt is 6 bits: capped at 63, which only waits longer).
    constexpr int kPreLoads = 12;
    auto wait_stage = [&](int st) {
      int npf;  // prefetches issued after stage st's DMA
      if (st < NS - 1) {
        npf = 1 + (st >= 1 ? (st - 1) / nch + 1 : 0);  // the initial one + stages 0 .. st-1 starting a tile
      } else {
        const int lo = st - NS + 1, hi = st - 1;
        npf = hi / nch - (lo >= 1 ? (lo - 1) / nch : -1);
      }
#define RLA_C1_WAIT(N)                                                                                     \
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(                            \
                   (NS - 2) * kDma + (N) * kPreLoads > 63 ? 63 : (NS - 2) * kDma + (N) * kPreLoads)        \
               : "memory")
      switch (npf) {
        case 0: RLA_C1_WAIT(0); break;
        case 1: RLA_C1_WAIT(1); break;
        case 2: RLA_C1_WAIT(2); break;
        case 3: RLA_C1_WAIT(3); break;
        default: RLA_C1_WAIT(4); break;
      }
#undef RLA_C1_WAIT
    };
    PreSet pa, pb;
    prefetch(pa, 0);
    int st = 0;
    auto tile = [&](int ti, PreSet& cur, PreSet& nxt) {
      // the first stage outside the chunk loop: the prefetch is then not inside a loop
      // whose back-edge merge would make the compiler's waits for it conservative
      wait_stage(st);
      issue(st + NS - 1);
      prefetch(nxt, ti + 1 < ntiles ? ti + 1 : ti);  // past the end: a harmless re-load
      compute(st);
      ++st;
      for (int c = 1; c < nch; ++c, ++st) {
        wait_stage(st);
        issue(st + NS - 1);
        compute(st);
      }
      epilogue(ti, cur);
    };
    for (int ti = 0; ti < ntiles; ti += 2) {
      tile(ti, pa, pb);
      if (ti + 1 < ntiles) tile(ti + 1, pb, pa);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the workgroup's LDS

  // per-channel totals: butterfly over the 32 pixel lanes of each half-wave, then the
  // two pixel-half waves in a fixed order
#pragma unroll
  for (int t = 0; t < TNW; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float a = ssum[t][e], b = ssq[t][e];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
      }
      if (r == 0) {
        const int c = BWD ? wn * 32 + 16 * (e >> 3) + 8 * h + (e & 7)
                          : wn * 32 * TNW + 32 * t + 8 * (e >> 2) + 4 * h + (e & 3);
        red[wm][0][c] = a;
        red[wm][1][c] = b;
      }
    }
  __syncthreads();
  for (int c = tid; c < BN; c += kC1Threads) {
    prow[c] = red[0][0][c] + red[1][0][c];
    prow[N + c] = red[0][1][c] + red[1][1][c];
  }
}

int c1_cu_count() {
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

bool conv1x1_stats_ok(int64_t M, int K, int N) {
  return M > 0 && K >= 32 && K % 32 == 0 && N >= 64 && N % 64 == 0 && N <= 4096;
}

bool conv1x1_pre_ok(int64_t M, int K, int N) { return conv1x1_stats_ok(M, K, N) && K <= kPreMaxK; }

Conv1x1Plan conv1x1_stats_plan(int64_t M, int N) {
  Conv1x1Plan p;
  // 32-channel wave columns only where N needs them: choosing them to keep a K = 256 /
  // 512 weight block resident measured slower (profiles/r4_c1/c1stats_probe_v4_wide.log)
  p.tnw = N % 128 == 0 ? 2 : 1;
  p.gy = N / (64 * p.tnw);
  const int mt = (int)((M + 127) / 128);
  // ~2 resident workgroups per CU over the whole grid; gx a multiple of 8 (XCD deal)
  int want = 2 * c1_cu_count() / p.gy;
  if (want < 8) want = 8;
  if (want > mt) want = mt;
  p.tiles_per_blk = (mt + want - 1) / want;
  int gx = (mt + p.tiles_per_blk - 1) / p.tiles_per_blk;
  p.gx = (gx + 7) / 8 * 8;
  return p;
}

void launch_conv1x1_stats(const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t M, int K, int N,
                          const Conv1x1Plan& p, float* part, hipStream_t s, const float* pre_ss, int64_t* nbt_inc) {
  const dim3 grid(p.gx * p.gy), block(kC1Threads);
  // resident weights where they fit beside the x ring: 6 x-only stages (4 in flight)
  // with a 16 KB weight block, 4 stages with 32 KB; else x + w stream through 4 stages
  const int64_t wbytes = (int64_t)K * 64 * p.tnw * 2;
#define RLA_C1_LAUNCH(T, R, NS)                                                                                   \
  do {                                                                                                            \
    if (pre_ss)                                                                                                   \
      hipLaunchKernelGGL((conv1x1_stats_kernel<T, R, NS, false, true>), grid, block, 0, s, x, w, y, M, K, N, p.gx, \
                         p.tiles_per_blk, part, nullptr, nullptr, nullptr, pre_ss, nbt_inc);                     \
    else                                                                                                          \
      hipLaunchKernelGGL((conv1x1_stats_kernel<T, R, NS>), grid, block, 0, s, x, w, y, M, K, N, p.gx,             \
                         p.tiles_per_blk, part);                                                                  \
  } while (0)
  if (p.tnw == 2) {
    if (wbytes <= 16384)
      RLA_C1_LAUNCH(2, true, 6);
    else if (wbytes <= 32768)
      RLA_C1_LAUNCH(2, true, 4);
    else
      RLA_C1_LAUNCH(2, false, 4);
  } else {
    if (wbytes <= 16384)
      RLA_C1_LAUNCH(1, true, 6);
    else if (wbytes <= 32768)
      RLA_C1_LAUNCH(1, true, 4);
    else
      RLA_C1_LAUNCH(1, false, 4);
  }
#undef RLA_C1_LAUNCH
}

bool conv1x1_bn_bwd_ok(int64_t M, int K, int N) {
  return M > 0 && K >= 32 && K % 32 == 0 && K <= 128 && N >= 64 && N % 64 == 0 && N <= 4096;
}

void launch_conv1x1_bn_bwd(const uint16_t* dy1, const uint16_t* wt, uint16_t* d, int64_t M, int K, int N,
                           const uint16_t* dy2, const uint16_t* yb, const uint16_t* xb, float* part, int* rows,
                           hipStream_t s) {
  Conv1x1Plan p = conv1x1_stats_plan(M, N);
  if (p.tnw != 1) {  // 32-channel wave columns: the epilogue prefetch's register budget
    p.tnw = 1;
    p.gy = N / 64;
    const int mt = (int)((M + 127) / 128);
    int want = 2 * c1_cu_count() / p.gy;
    if (want < 8) want = 8;
    if (want > mt) want = mt;
    p.tiles_per_blk = (mt + want - 1) / want;
    const int gx = (mt + p.tiles_per_blk - 1) / p.tiles_per_blk;
    p.gx = (gx + 7) / 8 * 8;
  }
  *rows = p.gx;
  if (part == nullptr) return;  // size query
  hipLaunchKernelGGL((conv1x1_stats_kernel<1, true, 6, true>), dim3(p.gx * p.gy), dim3(kC1Threads), 0, s, dy1, wt, d,
                     M, K, N, p.gx, p.tiles_per_blk, part, dy2, yb, xb);
}

}  // namespace rla
