// Fused BatchNorm (+ReLU) (+residual add) over NHWC bf16 activations, gfx950.
//
// Why (profiles/r1_resnet50_v2): in PyTorch-ROCm ResNet-50 (bs 128, bf16,
// channels_last) MIOpen's NHWC batch norm (6 kernels per layer) plus the
// separate ReLU / residual-add / ReLU-backward elementwise kernels take ~9.5 of
// ~25.6 ms per step.  All of it is HBM-bound, so the win is fewer passes:
//   forward:  partial (read x) -> finalize ([C] only) -> apply (read x [+res], write y)
//   backward: partial (read x, y, dy) -> finalize -> apply (read x, y, dy, write dx [+dres])
// ReLU and the bottleneck's residual add live in `apply`; their backward (the
// mask comes from the saved output y) in the backward kernels; the running
// statistics and num_batches_tracked are updated by the small kernels, so no
// extra elementwise launches remain.
//
// Layout: [M, C] rows (NHWC = channels_last, M = N*H*W), C % 8 == 0, C <= 2048.
// A thread owns 8 consecutive channels (one 16-byte bf16x8 vector) and walks
// rows with stride rpi = 256 / (C/8); each wave therefore reads whole 128-byte
// row segments.  Per-block fp32 partial sums go to a [blocks, 2, C] workspace
// that the finalize kernel reduces in fp64.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.h"
#include "pool_gather.h"

namespace rla {
namespace {

typedef float f8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef uint16_t u8x16 __attribute__((ext_vector_type(8)));  // 8 raw bf16 = 16 bytes

__device__ __forceinline__ f8 ld8(const uint16_t* p) {
  const u8x16 raw = *reinterpret_cast<const u8x16*>(p);
  return __builtin_convertvector(__builtin_bit_cast(b8, raw), f8);
}

__device__ __forceinline__ void st8(uint16_t* p, f8 v) {
  *reinterpret_cast<u8x16*>(p) = __builtin_bit_cast(u8x16, __builtin_convertvector(v, b8));
}

// store v as bf16 and return the stored (rounded) values
__device__ __forceinline__ f8 st8r(uint16_t* p, f8 v) {
  const b8 b = __builtin_convertvector(v, b8);
  *reinterpret_cast<u8x16*>(p) = __builtin_bit_cast(u8x16, b);
  return __builtin_convertvector(b, f8);
}

__device__ __forceinline__ f8 splat(float v) {
  f8 r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = v;
  return r;
}

__device__ __forceinline__ f8 ld8f(const float* p) {  // 8 fp32 per-channel coefficients
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f8 r;
  r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
  r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
  return r;
}

// the forward's affine map; the backward recomputes the ReLU mask with this exact
// expression (one fused multiply-add per element) instead of re-reading y
__device__ __forceinline__ f8 bn_affine(f8 x, f8 sc, f8 sf) { return __builtin_elementwise_fma(x, sc, sf); }

__device__ __forceinline__ f8 relu_mask(f8 d, f8 y) {
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = y[k] > 0.f ? d[k] : 0.f;
  return d;
}

// ---------------------------------------------------------------- partial sums
// DY2 (backward): the incoming gradient is dy + dy2 -- the residual-branch gradient
// of the NEXT bottleneck (its bn3's dres), folded here instead of autograd adding
// the two into a new tensor first (ops/bn.py, fold_residual_grad)
// RECOMP (backward, ReLU without residual): the mask is x*scale+shift > 0 recomputed
// from the forward statistics `ss` ([4, C]: mean, invstd, scale, shift) -- y is not read
// WD (backward with a residual: the layer's dres IS the masked incoming gradient d):
// the partial pass writes d once, rounded to bf16, and sums the rounded values; the
// apply pass then reads x and d only (dx = A d + B x + C) -- 2 streams fewer than
// re-reading y, dy and dy2 there and writing dres again.
// L2 (two-level reduction, bn_plan's `group` > 1): the partial rows are stored
// write-through (sc1); one lane per block takes a ticket on its group's counter
// (agent scope, after every wave drained its stores); the block that draws the
// group's last ticket sums the group's rows in block order in fp64 (sc1 loads, the
// guide's write-through + ticket hand-off, MI355X_MICROARCH.md §visibility) into row
// `group index` of `l2` and resets the counter.  bn_finalize then reads a handful
// of fp64 rows instead of up to 512 fp32 rows -- its small-C launches were ONE
// block streaming 256 KB of partials (~5 us).  Deterministic:
// fixed order at both levels.
struct BnL2 {
  double* rows;   // [ceil(blocks / group), 2, C]
  int* cnt;       // [ceil(blocks / group)] zero-initialised tickets (reset by each last arriver)
  int group;      // blocks per group (1: no second level)
};

// POOL (backward of the ResNet stem's BatchNorm, whose output was max-pooled in the
// same pass, ops/bn.py `pool`): dy is gathered from the pooled gradient through the
// argmax bytes (pool_gather.h) instead of read from a materialised maxpool_bwd output.
template <int MODE, bool RELU, bool DY2 = false, bool RECOMP = false, bool WD = false, bool POOL = false>
__global__ __launch_bounds__(kBnThreads) void bn_partial_kernel(const uint16_t* __restrict__ x,
                                                                const uint16_t* __restrict__ y,
                                                                const uint16_t* __restrict__ dy, int64_t M, int C,
                                                                int64_t rows_per_blk, float* __restrict__ part,
                                                                int64_t* nbt, const uint16_t* __restrict__ dy2 = nullptr,
                                                                const float* __restrict__ ss = nullptr,
                                                                BnL2 l2 = BnL2{nullptr, nullptr, 1},
                                                                uint16_t* __restrict__ dout = nullptr,
                                                                PoolGrad pg = PoolGrad{}) {
  // forward: one input stream, so twice the rows in flight per thread
  constexpr int U = MODE == 0 ? 8 : 4;
  __shared__ float sh[2][kBnThreads * 8];
  const int G = C >> 3, rpi = kBnThreads / G, tid = threadIdx.x;
  const int g = tid % G, r0 = tid / G;
  if (MODE == 0 && nbt && blockIdx.x == 0 && tid == 0) nbt[0] += 1;  // torch: += 1 before the momentum
  f8 s = splat(0.f), q = splat(0.f);
  const int64_t rb = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t re = rb + rows_per_blk < M ? rb + rows_per_blk : M;
  if (r0 < rpi) {
    const int64_t col = (int64_t)g * 8, step = (int64_t)rpi * C;
    f8 sc, sf;
    if (RECOMP) {
      sc = ld8f(ss + 2 * C + col);
      sf = ld8f(ss + 3 * C + col);
    }
    int64_t r = rb + r0;
    const uint16_t* px = x + r * C + col;
    // U rows in flight per thread (x, and dy [/ y] in the backward)
    for (; r + (U - 1) * rpi < re; r += U * rpi, px += U * step) {
      f8 xv[U], dv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xv[u] = ld8(px + u * step);
        if (MODE == 1) {
          const int64_t off = (px - x) + u * step;
          dv[u] = POOL ? pool_grad8<f8, b8, u8x16>(pg, C, r + u * rpi, (int)col) : ld8(dy + off);
          if (DY2) dv[u] += ld8(dy2 + off);
          if (RELU && !RECOMP) dv[u] = relu_mask(dv[u], ld8(y + off));
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (MODE == 1 && RECOMP) dv[u] = relu_mask(dv[u], bn_affine(xv[u], sc, sf));
        if (MODE == 1 && WD) dv[u] = st8r(dout + (px - x) + u * step, dv[u]);
        if (MODE == 0) {
          s += xv[u];
          q += xv[u] * xv[u];
        } else {
          s += dv[u];
          q += dv[u] * xv[u];
        }
      }
    }
    for (; r < re; r += rpi, px += step) {
      const f8 xv = ld8(px);
      if (MODE == 0) {
        s += xv;
        q += xv * xv;
      } else {
        const int64_t off = px - x;
        f8 d = POOL ? pool_grad8<f8, b8, u8x16>(pg, C, r, (int)col) : ld8(dy + off);
        if (DY2) d += ld8(dy2 + off);
        if (RELU) d = relu_mask(d, RECOMP ? bn_affine(xv, sc, sf) : ld8(y + off));
        if (WD) d = st8r(dout + off, d);
        s += d;
        q += d * xv;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sh[0][r0 * C + g * 8 + k] = s[k];
      sh[1][r0 * C + g * 8 + k] = q[k];
    }
  }
  __syncthreads();
  float* out = part + (int64_t)blockIdx.x * 2 * C;
  for (int c = tid; c < C; c += kBnThreads) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rpi; ++r) {
      a += sh[0][r * C + c];
      b += sh[1][r * C + c];
    }
    if (l2.group > 1) {  // write-through: read by another block of this launch
      __hip_atomic_store(out + c, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(out + C + c, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      out[c] = a;
      out[C + c] = b;
    }
  }
  if (l2.group <= 1) return;
  __shared__ int sh_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drained
  __syncthreads();
  const int grp = (int)blockIdx.x / l2.group;
  const int g0 = grp * l2.group;
  const int gsz = (int)gridDim.x - g0 < l2.group ? (int)gridDim.x - g0 : l2.group;
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(l2.cnt + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh_last = t == gsz - 1;
    if (sh_last) __hip_atomic_store(l2.cnt + grp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!sh_last) return;
  const float* rows = part + (int64_t)g0 * 2 * C;
  double* dst = l2.rows + (int64_t)grp * 2 * C;
  for (int c = tid; c < 2 * C; c += kBnThreads) {
    double acc = 0.0;
    int k = 0;
    for (; k + 8 <= gsz; k += 8) {  // 8 loads in flight
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __hip_atomic_load(const_cast<float*>(rows + (int64_t)(k + u) * 2 * C + c), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (double)v[u];
    }
    for (; k < gsz; ++k)
      acc += (double)__hip_atomic_load(const_cast<float*>(rows + (int64_t)k * 2 * C + c), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    dst[c] = acc;
  }
}

// ---------------------------------------------------------------- finalize
// kFinCh channels per block x kFinSlices slices of the partial rows (1024 threads):
// each thread sums rows sl, sl + kFinSlices, ... of its channel, 8 in flight, in
// fp64; the slices are combined by a fixed-order LDS tree.  64 slices: the small-C
// layers' finalize (C = 64: 512 partial rows) is ONE round of 8 loads per thread
// over 4 blocks instead of four dependent rounds on one block (~5 us -> ~2 us a
// launch; 106 launches per ResNet-50 step, profiles/r4_rn).
constexpr int kFinCh = 16, kFinSlices = 1024 / kFinCh;

template <bool BWD, typename P = float>
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const P* __restrict__ part, int nparts, int C,
                                                           double count, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* running_mean,
                                                           float* running_var, const int64_t* nbt, float momentum,
                                                           float eps, const float* __restrict__ mean_in,
                                                           const float* __restrict__ invstd_in,
                                                           float* __restrict__ out, int nbt_pending = 0) {
  __shared__ double sh[2][kFinSlices][kFinCh];
  const int cl = threadIdx.x % kFinCh, sl = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  // the per-channel inputs of the final step, issued ahead of the partial rows: they
  // land in the same memory round trip instead of a second one after the LDS tree
  // (round 6; ~105 finalize launches per ResNet-50 step, each latency-bound)
  float g = 1.f, bt = 0.f, rm = 0.f, rv = 0.f, mi = 0.f, is = 0.f;
  int64_t nb = 1;
  if (sl == 0 && c < C) {
    if (gamma) g = gamma[c];
    if (!BWD) {
      if (beta) bt = beta[c];
      if (running_mean) {
        rm = running_mean[c];
        rv = running_var[c];
        if (nbt) nb = nbt[0];
      }
    } else {
      mi = mean_in[c];
      is = invstd_in[c];
    }
  }
  double a = 0.0, b = 0.0;
  if (c < C) {
    const int64_t rs = 2 * (int64_t)C;
    const P* q = part + c;
    int p = sl;
    for (; p + 7 * kFinSlices < nparts; p += 8 * kFinSlices) {
      P v[16];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[2 * u] = q[(p + u * kFinSlices) * rs];
        v[2 * u + 1] = q[(p + u * kFinSlices) * rs + C];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a += v[2 * u];
        b += v[2 * u + 1];
      }
    }
    for (; p < nparts; p += kFinSlices) {
      a += q[p * rs];
      b += q[p * rs + C];
    }
  }
  sh[0][sl][cl] = a;
  sh[1][sl][cl] = b;
  __syncthreads();
#pragma unroll
  for (int st = kFinSlices / 2; st >= 1; st >>= 1) {
    if (sl < st) {
      sh[0][sl][cl] += sh[0][sl + st][cl];
      sh[1][sl][cl] += sh[1][sl + st][cl];
    }
    __syncthreads();
  }
  if (sl != 0 || c >= C) return;
  a = sh[0][0][cl];
  b = sh[1][0][cl];
  if (!BWD) {
    const double mean = a / count;
    double var = b / count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = g * invstd;
    out[c] = (float)mean;
    out[C + c] = invstd;
    out[2 * C + c] = sc;
    out[3 * C + c] = bt - (float)mean * sc;
    if (running_mean) {
      // momentum < 0: cumulative moving average, factor 1 / num_batches_tracked
      const float mom = momentum >= 0.f ? momentum : 1.f / (float)(nbt ? nb + nbt_pending : 1);
      const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
      running_mean[c] = (1.f - mom) * rm + mom * (float)mean;
      running_var[c] = (1.f - mom) * rv + mom * (float)unbiased;
    }
  } else {
    const float mean = mi, istd = is;
    const float dbeta = (float)a;
    const float dgamma = (float)((b - (double)mean * a) * (double)istd);
    const float A = g * istd;
    const float B = -A * istd * dgamma / (float)count;
    out[c] = dgamma;
    out[C + c] = dbeta;
    out[2 * C + c] = A;
    out[3 * C + c] = B;
    out[4 * C + c] = -A * dbeta / (float)count - B * mean;
  }
}

// ---------------------------------------------------------------- elementwise
template <bool RELU, bool RES>
__global__ __launch_bounds__(kBnThreads) void bn_apply_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ res,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, int64_t M, int C,
                                                              uint16_t* __restrict__ y, int64_t* nbt_inc) {
  const int G = C >> 3, rpi = kBnThreads / G, tid = threadIdx.x;
  const int g = tid % G, r0 = tid / G;
  // the statistics came from a conv epilogue (no partial kernel ran): num_batches_tracked
  // += 1 here, after the finalize that already used the incremented value
  if (nbt_inc && blockIdx.x == 0 && tid == 0) nbt_inc[0] += 1;
  if (r0 >= rpi) return;
  const f8 sc = ld8f(scale + g * 8), sf = ld8f(shift + g * 8);
  const int64_t col = (int64_t)g * 8, rstride = (int64_t)gridDim.x * rpi;
  int64_t r = (int64_t)blockIdx.x * rpi + r0;
  for (; r + rstride < M; r += 2 * rstride) {  // two rows in flight
    const int64_t o0 = r * C + col, o1 = (r + rstride) * C + col;
    f8 v0 = ld8(x + o0), v1 = ld8(x + o1);
    f8 a0, a1;
    if (RES) {
      a0 = ld8(res + o0);
      a1 = ld8(res + o1);
    }
    v0 = bn_affine(v0, sc, sf);
    v1 = bn_affine(v1, sc, sf);
    if (RES) {
      v0 += a0;
      v1 += a1;
    }
    if (RELU) {
      v0 = relu_mask(v0, v0);
      v1 = relu_mask(v1, v1);
    }
    st8(y + o0, v0);
    st8(y + o1, v1);
  }
  if (r < M) {
    const int64_t o = r * C + col;
    f8 v = bn_affine(ld8(x + o), sc, sf);
    if (RES) v += ld8(res + o);
    if (RELU) v = relu_mask(v, v);
    st8(y + o, v);
  }
}

template <bool RELU, bool DRES, bool DY2 = false, bool RECOMP = false, bool POOL = false>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_apply_kernel(const uint16_t* __restrict__ x,
                                                                  const uint16_t* __restrict__ y,
                                                                  const uint16_t* __restrict__ dy,
                                                                  const float* __restrict__ coef, int64_t M, int C,
                                                                  uint16_t* __restrict__ dx,
                                                                  uint16_t* __restrict__ dres,
                                                                  const uint16_t* __restrict__ dy2 = nullptr,
                                                                  const float* __restrict__ ss = nullptr,
                                                                  PoolGrad pg = PoolGrad{}) {
  const int G = C >> 3, rpi = kBnThreads / G, tid = threadIdx.x;
  const int g = tid % G, r0 = tid / G;
  if (r0 >= rpi) return;
  const f8 A = ld8f(coef + 2 * C + g * 8), B = ld8f(coef + 3 * C + g * 8), Cc = ld8f(coef + 4 * C + g * 8);
  f8 sc, sf;
  if (RECOMP) {
    sc = ld8f(ss + 2 * C + g * 8);
    sf = ld8f(ss + 3 * C + g * 8);
  }
  const int64_t col = (int64_t)g * 8, rstride = (int64_t)gridDim.x * rpi;
  for (int64_t r = (int64_t)blockIdx.x * rpi + r0; r < M; r += rstride) {
    const int64_t o = r * C + col;
    f8 d = POOL ? pool_grad8<f8, b8, u8x16>(pg, C, r, (int)col) : ld8(dy + o);
    if (DY2) d += ld8(dy2 + o);
    const f8 xv = ld8(x + o);
    if (RELU) d = relu_mask(d, RECOMP ? bn_affine(xv, sc, sf) : ld8(y + o));
    st8(dx + o, A * d + B * xv + Cc);
    if (DRES) st8(dres + o, d);
  }
}

int apply_grid(int64_t M, int C) {
  const int rpi = kBnThreads / (C >> 3);
  int64_t b = (M + rpi - 1) / rpi;
  if (b > 2048) b = 2048;  // 8 blocks per CU; each thread then walks ~M/(2048*rpi) rows
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

BnPlan bn_plan(int64_t M, int C) {
  const int rpi = kBnThreads / (C >> 3);
  // >= 16 row iterations per thread, at most 512 blocks (2 per CU: 8 waves with 4-8
  // rows in flight each keep HBM busy).  Round 3 also capped the partial table at
  // 128K floats for the finalize's sake -- which left the wide layers on a fraction
  // of the chip (C = 2048: 64 blocks on 256 CUs); the 64-slice finalize reads up to
  // 512 rows in one round, so every width now gets the full grid.
  int64_t blocks = (M + (int64_t)rpi * 16 - 1) / ((int64_t)rpi * 16);
  if (blocks > 512) blocks = 512;
  if (blocks < 1) blocks = 1;
  BnPlan p;
  p.rows_per_blk = (M + blocks - 1) / blocks;
  p.blocks = (int)((M + p.rows_per_blk - 1) / p.rows_per_blk);
  if (p.blocks < 1) p.blocks = 1;
  // second level: groups whose rows (group x 2C fp32) one block sums in ~1 us
  // (<= 32 KB); only where the finalize would otherwise stream many rows
  // Off by default (RLA_BN_L2=1 turns it on): the tickets' agent-scope atomics and the
  // last arriver's fp64 pass lengthened every partial launch by ~5 us while saving
  // ~1 us of finalize (profiles/r4_rn: forward partials 609 -> 900 us per step)
  static const bool l2_on = [] {
    const char* e = getenv("RLA_BN_L2");
    return e && e[0] == '1';
  }();
  int g = 4096 / C;
  if (g > p.blocks) g = p.blocks;
  p.group = l2_on && p.blocks > 16 && g > 1 ? g : 1;
  p.groups = (p.blocks + p.group - 1) / p.group;
  return p;
}

void launch_bn_partial(const uint16_t* x, const uint16_t* y, const uint16_t* dy, int64_t M, int C, int mode,
                       bool relu, const BnPlan& plan, float* part, int64_t* nbt, hipStream_t s, const uint16_t* dy2,
                       const float* ss, BnLevel2 lv, uint16_t* dout, const PoolGrad* pool) {
  const dim3 grid(plan.blocks), block(kBnThreads);
  const BnL2 L{lv.rows, lv.tickets, lv.rows ? plan.group : 1};
  if (pool) {  // the stem: ReLU mask recomputed from the forward stats, dy gathered through the pool
    hipLaunchKernelGGL((bn_partial_kernel<1, true, false, true, false, true>), grid, block, 0, s, x, y, dy, M, C,
                       plan.rows_per_blk, part, nullptr, nullptr, ss, L, nullptr, *pool);
    return;
  }
  if (mode == 1 && dout) {  // residual layer: d written here (y-mask or none)
    if (relu && dy2)
      hipLaunchKernelGGL((bn_partial_kernel<1, true, true, false, true>), grid, block, 0, s, x, y, dy, M, C,
                         plan.rows_per_blk, part, nullptr, dy2, nullptr, L, dout);
    else if (relu)
      hipLaunchKernelGGL((bn_partial_kernel<1, true, false, false, true>), grid, block, 0, s, x, y, dy, M, C,
                         plan.rows_per_blk, part, nullptr, nullptr, nullptr, L, dout);
    else if (dy2)
      hipLaunchKernelGGL((bn_partial_kernel<1, false, true, false, true>), grid, block, 0, s, x, y, dy, M, C,
                         plan.rows_per_blk, part, nullptr, dy2, nullptr, L, dout);
    else
      hipLaunchKernelGGL((bn_partial_kernel<1, false, false, false, true>), grid, block, 0, s, x, y, dy, M, C,
                         plan.rows_per_blk, part, nullptr, nullptr, nullptr, L, dout);
    return;
  }
  if (mode == 1 && relu && ss) {
    if (dy2)
      hipLaunchKernelGGL((bn_partial_kernel<1, true, true, true>), grid, block, 0, s, x, y, dy, M, C,
                         plan.rows_per_blk, part, nullptr, dy2, ss, L);
    else
      hipLaunchKernelGGL((bn_partial_kernel<1, true, false, true>), grid, block, 0, s, x, y, dy, M, C,
                         plan.rows_per_blk, part, nullptr, nullptr, ss, L);
    return;
  }
  if (mode == 1 && dy2) {
    if (relu)
      hipLaunchKernelGGL((bn_partial_kernel<1, true, true>), grid, block, 0, s, x, y, dy, M, C, plan.rows_per_blk,
                         part, nullptr, dy2, nullptr, L);
    else
      hipLaunchKernelGGL((bn_partial_kernel<1, false, true>), grid, block, 0, s, x, y, dy, M, C, plan.rows_per_blk,
                         part, nullptr, dy2, nullptr, L);
    return;
  }
  if (mode == 0)
    hipLaunchKernelGGL((bn_partial_kernel<0, false>), grid, block, 0, s, x, y, dy, M, C, plan.rows_per_blk, part,
                       nbt, nullptr, nullptr, L);
  else if (relu)
    hipLaunchKernelGGL((bn_partial_kernel<1, true>), grid, block, 0, s, x, y, dy, M, C, plan.rows_per_blk, part,
                       nullptr, nullptr, nullptr, L);
  else
    hipLaunchKernelGGL((bn_partial_kernel<1, false>), grid, block, 0, s, x, y, dy, M, C, plan.rows_per_blk, part,
                       nullptr, nullptr, nullptr, L);
}

void launch_bn_finalize(const float* part, int nparts, int C, double count, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, const int64_t* nbt,
                        float momentum, float eps, float* stats, hipStream_t s, int nbt_pending) {
  hipLaunchKernelGGL((bn_finalize_kernel<false>), dim3((C + kFinCh - 1) / kFinCh), dim3(1024), 0, s, part, nparts, C, count,
                     gamma, beta, running_mean, running_var, nbt, momentum, eps, nullptr, nullptr, stats, nbt_pending);
}

void launch_bn_bwd_finalize(const float* part, int nparts, int C, double count, const float* gamma,
                            const float* mean, const float* invstd, float* coef, hipStream_t s) {
  hipLaunchKernelGGL((bn_finalize_kernel<true>), dim3((C + kFinCh - 1) / kFinCh), dim3(1024), 0, s, part, nparts, C, count,
                     gamma, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, mean, invstd, coef);
}

void launch_bn_finalize64(const double* part, int nparts, int C, double count, const float* gamma,
                          const float* beta, float* running_mean, float* running_var, const int64_t* nbt,
                          float momentum, float eps, float* stats, hipStream_t s) {
  hipLaunchKernelGGL((bn_finalize_kernel<false, double>), dim3((C + kFinCh - 1) / kFinCh), dim3(1024), 0, s, part, nparts, C,
                     count, gamma, beta, running_mean, running_var, nbt, momentum, eps, nullptr, nullptr, stats);
}

void launch_bn_bwd_finalize64(const double* part, int nparts, int C, double count, const float* gamma,
                              const float* mean, const float* invstd, float* coef, hipStream_t s) {
  hipLaunchKernelGGL((bn_finalize_kernel<true, double>), dim3((C + kFinCh - 1) / kFinCh), dim3(1024), 0, s, part, nparts, C,
                     count, gamma, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, mean, invstd, coef);
}

void launch_bn_apply(const uint16_t* x, const uint16_t* res, const float* scale, const float* shift, int64_t M,
                     int C, bool relu, uint16_t* y, hipStream_t s, int64_t* nbt_inc) {
  const dim3 grid(apply_grid(M, C)), block(kBnThreads);
  if (relu && res)
    hipLaunchKernelGGL((bn_apply_kernel<true, true>), grid, block, 0, s, x, res, scale, shift, M, C, y, nbt_inc);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<true, false>), grid, block, 0, s, x, res, scale, shift, M, C, y, nbt_inc);
  else if (res)
    hipLaunchKernelGGL((bn_apply_kernel<false, true>), grid, block, 0, s, x, res, scale, shift, M, C, y, nbt_inc);
  else
    hipLaunchKernelGGL((bn_apply_kernel<false, false>), grid, block, 0, s, x, res, scale, shift, M, C, y, nbt_inc);
}

void launch_bn_bwd_apply(const uint16_t* x, const uint16_t* y, const uint16_t* dy, const float* coef, int64_t M,
                         int C, bool relu, uint16_t* dx, uint16_t* dres, hipStream_t s, const uint16_t* dy2,
                         const float* ss, const PoolGrad* pool) {
  const dim3 grid(apply_grid(M, C)), block(kBnThreads);
  if (pool) {
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false, false, true, true>), grid, block, 0, s, x, y, dy, coef, M, C,
                       dx, dres, nullptr, ss, *pool);
    return;
  }
  if (relu && ss && !dres) {  // no residual: the mask is recomputed from x and the forward stats
    if (dy2)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false, true, true>), grid, block, 0, s, x, y, dy, coef, M, C, dx,
                         dres, dy2, ss);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false, false, true>), grid, block, 0, s, x, y, dy, coef, M, C,
                         dx, dres, nullptr, ss);
    return;
  }
  if (dy2) {  // the folded residual gradient; ResNet's bn3 (relu, its own dres) is the user
    if (relu && dres)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<true, true, true>), grid, block, 0, s, x, y, dy, coef, M, C, dx, dres,
                         dy2);
    else if (relu)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false, true>), grid, block, 0, s, x, y, dy, coef, M, C, dx,
                         dres, dy2);
    else if (dres)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<false, true, true>), grid, block, 0, s, x, y, dy, coef, M, C, dx,
                         dres, dy2);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<false, false, true>), grid, block, 0, s, x, y, dy, coef, M, C, dx,
                         dres, dy2);
    return;
  }
  if (relu && dres)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true, true>), grid, block, 0, s, x, y, dy, coef, M, C, dx, dres);
  else if (relu)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false>), grid, block, 0, s, x, y, dy, coef, M, C, dx, dres);
  else if (dres)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<false, true>), grid, block, 0, s, x, y, dy, coef, M, C, dx, dres);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<false, false>), grid, block, 0, s, x, y, dy, coef, M, C, dx, dres);
}

}  // namespace rla
