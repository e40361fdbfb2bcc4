// Fused MNIST-MLP training step, v3: layer 1 pipelined across steps, every
// weight-gradient epilogue spread over many CUs.
//
// v2 (a head + W1 kernel pair, retired) measured 25 us/step on MI355X; 10 of its head kernel's
// 17 us went to staging the X batch (50 KB gathered through the sample index)
// plus the 784-deep layer-1 GEMM on ONE CU, and 4.4 us to the small-parameter
// gradient/Adam epilogue on that same CU (profiles/r1_first/mlp_phases_v2.json).
// v3 keeps only the inherently serial chain on the one-workgroup head and moves
// everything else to a wide tail launch:
//
//   head(t)   one workgroup per 32 batch rows (the per-sample chain is row-
//             independent): H1 = relu(H1pre[t] + b1) (4 KB read instead of X + W1),
//             layers 2/3, log_softmax/NLL/accuracy, dH2, dH1.  Hands the
//             transposed activations / deltas (H1^T, H2^T, dH2^T, dZ^T, dH1^T;
//             bf16, [rows][Bp]) to the tail through HBM and zeroes its rows of
//             the other H1pre slot.  With several row blocks, each writes its
//             (sum NLL, #correct, #rows) to `head_part` and tail block 0 reduces
//             them in block order (deterministic) into the stats ring.
//   tail(t)   blocks [0, 49): one 16-pixel W1 column tile each: dW1 tile =
//             X[t]_tile^T dH1 (MFMA; X^T by ds_read_b64_tr_b16), Adam on the
//             tile, then gather X[t+1]'s tile (u8 -> bf16) and add
//             X[t+1]_tile . W1_tile^T into H1pre[t+1] (17.15 fixed-point int32 atomics,
//             49 adders per element) -- layer 1 is linear in W1 and this block
//             holds the freshly updated tile in registers.  The X tile is parked
//             in `xring` for tail(t+1)'s dW1.
//             blocks [49, ...): one wave per 16x16 dW2 / dW3 tile or 64 biases:
//             MFMA over the batch from the head's transposes, Adam, bf16 shadow
//             (row-major + transposed) refresh.
//
// World size > 1 splits the tail: GRAD (all gradients -> `grads`, gather
// X[t+1]) before the allreduce, ADAM (W1 tiles: Adam + the next-step partial;
// extra blocks: flat Adam over every other parameter) after it.  PRIME computes
// H1pre for the pending batch from the current weights (after init / load /
// broadcast).
//
// Device state (graph-replay safe): counters[0] optimizer step, [1] cursor of
// the NEXT batch, [2] cursor the last head consumed, [3] ring slot the next head
// reads, [4] which of the two `order` epoch buffers counters[1] indexes.
// H1pre is stored in MFMA-fragment order (element (b, m) at
// (((b/16 * L1/16 + m/16) * 4 + b%4) * 64 + (b%16/4) * 16 + m%16) so every atomic
// wave-instruction covers 256 contiguous bytes.  The integer atomics are
// associative, so H1pre (and the step) does not depend on arrival order.
#include "common.h"
#include "kernels.h"
#include "mlp_common.h"
#include "comm/xgmi.h"

namespace rla {
namespace {

using namespace mlp;
using comm::kDpMaxBlocks;
using comm::kXgmiFlagBytes;
using comm::kXgmiMaxRanks;

constexpr int kThreads = 512;
constexpr int kWaves = 8;
constexpr int kDZS = 40;
constexpr int kXSS = 24;   // LDS row stride of a 16-pixel X slice (bf16)
constexpr int kBMax = 256;
constexpr int kCnt = 5;  // counters: [0, 5) current state, [5, 10) the head's advanced copy
constexpr int kHeadRows = 32;  // batch rows per head workgroup

enum TailMode { kFused = 0, kGrad = 1, kAdam = 2, kPrime = 3, kFusedDP = 4 };

// rows of the `act` hand-off buffer ([rows][Bp] bf16)
template <int L1, int L2>
struct Act {
  static constexpr int H1T = 0, H2T = L1, DH2T = L1 + L2, DZT = L1 + 2 * L2, ROWS = L1 + 2 * L2 + 16;
};

template <int BC, int L1, int L2>
struct Cfg3 {
  static constexpr int H1S = L1 + 8, H2S = L2 + 8, TS = BC + 8;
  static constexpr int MT = BC / 16, TN1 = L1 / 16, TN2 = L2 / 16;
  static constexpr size_t oH1 = 0;
  static constexpr size_t oH1T = oH1 + (size_t)BC * H1S * 2;
  static constexpr size_t oH2 = oH1T + (size_t)L1 * TS * 2;
  static constexpr size_t oZ = oH2 + (size_t)BC * H2S * 2;
  static constexpr size_t odZ = oZ + (size_t)BC * 16 * 4;
  static constexpr size_t odZT = odZ + (size_t)BC * kDZS * 2;
  static constexpr size_t oY = odZT + (size_t)16 * TS * 2;
  static constexpr size_t oMisc = oY + (size_t)BC * 4;
  static constexpr size_t oBias = oMisc + 64;
  // K-split partial sums (fp32), reduced in fixed group order: layer 3 [KG3][BC][16],
  // dH1 [KG1][BC][L1]
  // K splits only where a wave would chain >= 4 k-steps (L2 >= 128); below that
  // the unsplit maps below were measured faster (profiles/r2_c11)
  static constexpr int KS3 = L2 / 32, KG3 = KS3 >= 4 ? 4 : 1;
  static constexpr int KSH = L2 / 32, KG1A = 8 / TN1, KG1 = KSH < 4 ? 1 : (KSH < KG1A ? KSH : KG1A);
  static constexpr size_t oPart = oBias + (((size_t)(L1 + L2 + 16) * 4 + 15) / 16) * 16;
  static constexpr size_t szPart3 = KG3 > 1 ? (size_t)KG3 * BC * 16 * 4 : 0;
  static constexpr size_t szPart1 = KG1 > 1 ? (size_t)KG1 * BC * L1 * 4 : 0;
  static constexpr size_t total = oPart + (szPart3 > szPart1 ? szPart3 : szPart1);
};

template <int BC, int L1, int L2>
constexpr bool fits3() {
  return Cfg3<BC, L1, L2>::total + 256 <= 160 * 1024;
}

__device__ __forceinline__ __bf16 relu_bf(float x) { return (__bf16)fmaxf(x, 0.f); }

// H1pre partial sums travel as 12.20 fixed point in int32: the 49 tile
// contributions are added with integer atomics, which are associative, so the sum
// (and the whole step) is bitwise reproducible whatever order the atomics land in.
// Resolution 2^-20 (9.5e-7; H1's bf16 rounding right after is 4.9e-4 at 0.1).  Each
// tile's 16-pixel partial saturates at +-32 (an average |w| of 2 over pixels in
// [0, 1]), so the 49-term sum stays inside +-1568 and can never wrap.  32-bit words
// halve the bytes every head pass loads and every atomic moves against round 5's
// 32.32 int64 (same box: 7.81 vs 8.08 us/step steady, profiles/r6_h1copies).
// Cost: a pre-activation within ~1e-6 of zero can take the other side of the ReLU
// than an fp32 sum would (tests/test_mlp3.py models the rounding in its emulation).
constexpr float kFix = 1048576.0f;  // 2^20
constexpr float kFixSat = 33554432.0f;  // 2^25 = 32.0 in fixed point
__device__ __forceinline__ unsigned f32_to_fixed(float x) {
  return (unsigned)__float2int_rn(fminf(fmaxf(x * kFix, -kFixSat), kFixSat));
}
__device__ __forceinline__ float fixed_to_f32(int q) { return (float)q * (1.0f / 1048576.0f); }

// H1pre copies per ring slot: the 49 W1 tiles' layer-1 partials are spread over G
// copies (tile kt adds into copy kt % G) and the head sums the copies as it loads
// them (integer adds: exact, order-free).  Device-scope atomics to ONE address
// serialise at ~12 ns each (MI355X_MICROARCH.md "fanin"), so 49 tiles adding into the
// same 8-byte word drained ~0.6 us after the tiles were done (measured: plain stores
// in place of the atomics cut the step 8.38 -> 7.87 us, profiles/r6_h1copies); two
// copies halve every chain.  One copy at L1 = 128 (the head's loads would double).
template <int L1>
struct H1Copies {
  static constexpr int G = L1 <= 64 ? 2 : 1;
};

// Gather one 16-pixel tile of batch (ob, cursor) as bf16 rows into xring slot
// `dst_slot` (rows >= B zero); block kt == 0 also stages that batch's labels
// into yring (-1 for padded rows), so no kernel chases the sample index on
// its critical path.  Runs as extra workgroups of the head launch (for the
// NEXT batch, concurrently with the head's serial chain) or in PRIME.
__device__ __forceinline__ void gather_tile(const MLP3Args& a, int kt, int64_t ob, int64_t cursor,
                                            int64_t dst_slot, int nthreads) {
  const int tid = threadIdx.x;
  const int B = a.B, Bp = (B + 31) / 32 * 32;
  const int64_t* idx = a.order + ob * a.order_stride + cursor * B;
  __bf16* dst = reinterpret_cast<__bf16*>(a.xring) + (dst_slot * kTiles + kt) * (int64_t)Bp * 16;
  for (int b = tid; b < Bp; b += nthreads) {
    bf16x8 lo = zero8(), hi = zero8();
    if (b < B) u8x16_to_bf16(*reinterpret_cast<const uint4*>(a.x_u8 + idx[b] * kD + kt * 16), lo, hi);
    *reinterpret_cast<bf16x8*>(dst + b * 16) = lo;
    *reinterpret_cast<bf16x8*>(dst + b * 16 + 8) = hi;
  }
  if (kt == 0)
    for (int b = tid; b < Bp; b += nthreads) a.yring[dst_slot * Bp + b] = b < B ? (int)a.labels[idx[b]] : -1;
}

// Step state read through the constant address space (scalar loads, lgkmcnt): a
// step's kernels write the counters only after every reader of the launch is
// done with them (head: at its end; one-launch: after all blocks' acks), and a
// vector load here made the compiler wait on vmcnt ahead of independent loads.
__device__ __forceinline__ int64_t ld_state(const int64_t* p, int i) {
  return ((const __attribute__((address_space(4))) int64_t*)(p))[i];
}

// Diagnostic stamp (probe builds only pass a.stamps): latest end over many blocks.
__device__ __forceinline__ void stamp_max(const MLP3Args& a, int k) {
  if (a.stamps && threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned long long*>(a.stamps + k),
              (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// One-launch step bookkeeping (mlp3_one_kernel): counters[kSeq] counts its
// launches; hand[kHandAck] accumulates one acknowledgement per block per launch
// (monotonic: launch `seq` is complete at (seq + 1) * gridDim.x); hand[kHandErr]
// is set when a bounded wait expires.
constexpr int kSeq = 10;
constexpr int kHandAck = 0, kHandErr = 16, kHandWords = 32;

// ---------------------------------------------------------------------------
// Head kernel (blocks [0, nchunks): one 8-wave workgroup per BC batch rows;
// blocks [nchunks, nchunks + 49): next-batch gather)
// ---------------------------------------------------------------------------
// MULTI = false (B <= 32): ONE row block, its index and the block-role branch
// compile-time constants -- the runtime form (row block = blockIdx.x, branch on
// a kernarg-derived chunk count) measured 0.7 us slower per step at the
// default 32-64 / batch-32 config (profiles/r2_c11, A/B on one box).
//
// REP = true: the serial chain as replicated by EVERY block of the one-launch
// step (mlp3_one_kernel, B <= 32): nothing goes to global memory, the transposed
// activations / deltas stay in this block's LDS (H1^T, dZ^T and the extra
// H2^T / dH2^T / dH1^T images at OneLds offsets) for the block's own tail role;
// no H1pre zeroing (invariant: the slot the tiles accumulate into is zero at a
// step's start), no state advance (block 0 does it after every block's ack).
// REP: the one-launch tile's loads of the NEXT batch (pixels of sample `si`, tile
// `kt`, and its label), issued by head_body right after its acknowledgement (its
// vmcnt(0) has resolved the sample index; the rest of the head pass reads LDS
// only) by the one wave that uses them, so the round trip hides under the head pass.
struct RepPre {
  bool active;  // wave-uniform: the PreWave of a W1 tile block
  int64_t si;
  int kt;
  uint4 xn;
  int64_t yn;
  uint32_t raw;  // LDS byte address of the DMA landing area (kPreRawBytes), PreWave::hidden
};

struct NoHook {
  __device__ void operator()() const {}
};

// The next batch's pixels / labels, fetched during the head pass by LDS-DMA
// (global_load_lds: no destination VGPR) from a tile wave that has no W1 column
// (PreWave): the compiler does not see these loads, so none of the counted waits it
// places for its own loads -- and no register it reuses next to a pending load's
// destination -- can wait for their HBM round trip inside the head pass.  With
// plain loads (rounds 2-4, wave 0) the softmax waited vmcnt(0) for the label load (a
// register-pair hazard on its destination) and with it for every prologue load.
// The consumer, the same wave, waits vmcnt(0) itself (it has no stores in flight).
// M0 is saved and restored in the same statement (LDS-DMA recipe, as conv1x1.hip).
__device__ __forceinline__ void dma_lds16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}
__device__ __forceinline__ void dma_lds4(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}
constexpr int kPreRawBytes = 64 * 16 + 64 * 4;  // pixels (16 B per lane) + labels (4 B per lane)
template <int L1>
struct PreWave {
  // a tile wave without a W1 column (no Adam stores before the consumer), when there is one
  static constexpr bool hidden = L1 / 16 < kWaves;
  static constexpr int wave = hidden ? kWaves - 1 : 0;
};

// REP: `hook` issues the block's PRIVATE prologue loads (Adam state of its W1 tile,
// the parked X tile, the next sample index) right after the head's loads of SHARED
// state, so they are the youngest kRepHookLoads vector loads of every wave and the
// acknowledgement waits for the shared ones only (vmcnt(kRepHookLoads)).  Issued in
// the kernel prologue instead (rounds 2-4), they were older than the head's loads,
// and the ack's vmcnt(0) waited for their HBM round trips: every tile block's head
// pass ended ~1.2 us after block 0's (profiles/r4_dp/dp_phases_wire16.log).
constexpr int kRepHookLoads = 6;

template <int BC, int L1, int L2, bool MULTI, bool REP, class Hook = NoHook>
__device__ __forceinline__ void head_body(const MLP3Args& a, char* smem, RepPre* pre = nullptr,
                                          const Hook& hook = Hook{}) {
  using C = Cfg3<BC, L1, L2>;
  using O = Off<L1, L2>;
  using A = Act<L1, L2>;
  static_assert(!REP || (!MULTI && BC == 32), "one-launch head: one 32-row block");
  __bf16* sH1 = (__bf16*)(smem + C::oH1);
  __bf16* sH1T = (__bf16*)(smem + C::oH1T);
  __bf16* sH2 = (__bf16*)(smem + C::oH2);
  float* sZ = (float*)(smem + C::oZ);
  __bf16* sdZ = (__bf16*)(smem + C::odZ);
  __bf16* sdZT = (__bf16*)(smem + C::odZT);
  int* sY = (int*)(smem + C::oY);
  float* misc = (float*)(smem + C::oMisc);
  float* sBias = (float*)(smem + C::oBias);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const __bf16* SH = reinterpret_cast<const __bf16*>(a.shadow);
  const float* P = a.params;

  const int nchunks = MULTI ? (a.B + BC - 1) / BC : 1;
  const int c = MULTI ? (int)blockIdx.x : 0;  // this workgroup's batch rows [c * BC, c * BC + BC)
  const bool stamp_ok = a.stamps && tid == 0 && c == 0 && (!REP || blockIdx.x == 0);

  // device counters: uniform scalar loads, no LDS broadcast round trip
  const int64_t t = ld_state(a.counters, 0) + 1;
  const int64_t cursor = ld_state(a.counters, 1);
  const int64_t slot = ld_state(a.counters, 3);
  const int64_t ob = ld_state(a.counters, 4);
  const int Bp = (a.B + 31) / 32 * 32;
  __bf16* ACT = reinterpret_cast<__bf16*>(a.act);
  __bf16* DH1T = reinterpret_cast<__bf16*>(a.dh1t);
  // REP: LDS images of H2^T / dH2^T / dH1^T ([rows][TS] bf16) after the head's own region
  __bf16* sH2T = (__bf16*)(smem + C::total);
  __bf16* sDH2T = sH2T + L2 * C::TS;
  __bf16* sDH1T = sDH2T + L2 * C::TS;

  // Every load of the head's inputs is issued unconditionally (invalid lanes read
  // a clamped in-bounds address and select zero afterwards) and LDS is written
  // only after the last load is in flight: a load in a divergent branch, or an
  // LDS write of a just-loaded value ahead of the others, makes the compiler wait
  // for it (vmcnt(0)) before issuing anything else -- a full memory round trip each.
  constexpr int NBIAS = L1 + L2 + kNC;
  float bias_v;
  {
    const int bt = tid < NBIAS ? tid : 0;
    const int64_t bgi = bt < L1 ? O::B1 + bt : (bt < L1 + L2 ? O::B2 + (bt - L1) : O::B3 + (bt - L1 - L2));
    bias_v = P[bgi];
  }
  if (tid == 0) {
    misc[0] = 0.f; misc[1] = 0.f; misc[2] = 0.f;
    if (stamp_ok) a.stamps[0] = __builtin_amdgcn_s_memrealtime();
  }
  // the tail of this step accumulates the next step's H1pre into the other slot;
  // in fragment order this block's rows are one contiguous BC * L1 range
  if constexpr (!REP) {
#pragma unroll
    for (int cp = 0; cp < H1Copies<L1>::G; ++cp) {
      uint4* z = reinterpret_cast<uint4*>(a.h1pre + ((slot ^ 1) * H1Copies<L1>::G + cp) * (int64_t)Bp * L1 +
                                          (int64_t)c * BC * L1);
      for (int i = tid; i < BC * L1 / 4; i += kThreads) z[i] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  const float invB = 1.f / (float)a.B;
  constexpr int KS2 = L1 / 32, KS3 = C::KS3, KSH = C::KSH;
  constexpr int MT = C::MT;
  // Wave work maps (8 waves).  Layer 2 / dH2: wave w owns output column tiles
  // nt = w + 8j (j < NTW2) for BOTH row tiles, so each weight fragment feeds MT
  // MFMAs.  Layer 3: (row tile, K group) per wave, KG3 groups of KPG3 k-steps.
  // dH1: (column tile, K group) per wave, KG1 groups of KPG1 k-steps.  K-split
  // partials are summed in fixed group order through LDS -> deterministic.
  // narrow layer 2 (TN2 * MT <= 8 tiles): one (column, row) tile per wave instead,
  // so all 8 waves work (measured faster at 32-64 than column-per-wave)
  constexpr bool ROW2 = C::TN2 * MT <= kWaves;
  constexpr int NTW2 = ROW2 ? 1 : (C::TN2 + kWaves - 1) / kWaves;
  constexpr int MTW2 = ROW2 ? 1 : MT;  // row tiles per wave in layer 2 / dH2
  const int nt_base = ROW2 ? w % C::TN2 : w;
  const int mt_base = ROW2 ? w / C::TN2 : 0;
  const bool l2_active = ROW2 ? (w < C::TN2 * MT) : true;
  constexpr int KG3 = C::KG3, KPG3 = KS3 / KG3;
  constexpr int KG1 = C::KG1, KPG1 = KSH / KG1;
  static_assert(MT * KG3 <= kWaves && C::TN1 * KG1 <= kWaves, "wave maps");
  float* sPart = (float*)(smem + C::oPart);

  // LDS [rows][TS] -> act rows [dst_row][Bp] at columns [row0, row0 + BC) (< Bp)
  auto copy_rows = [&](const __bf16* src, int nrows, int dst_row, int row0) {
    constexpr int CPR = BC / 8;
    for (int e = tid; e < nrows * CPR; e += kThreads) {
      const int r = e / CPR, col = (e - r * CPR) * 8;
      if (row0 + col < Bp)
        *reinterpret_cast<bf16x8*>(ACT + (int64_t)(dst_row + r) * Bp + row0 + col) = ld8(src + r * C::TS + col);
    }
  };

  {
    const int row0 = c * BC;

    // Labels and H1pre of BOTH ring slots are loaded before the barrier and
    // selected after it: none of these loads waits for the counters read.
    constexpr int NQ = (BC * L1 / 4 + kThreads - 1) / kThreads;
    constexpr int G = H1Copies<L1>::G;
    int4 qs[NQ][2][G];  // [item][slot][copy]: 4 consecutive int32 words
    bool qok[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int f4 = tid + k * kThreads;
      const int mtl = (f4 * 4 >> 8) / C::TN1;
      // rows past round_up(B, 32) exist only in the last chunk's LDS image
      qok[k] = f4 < BC * L1 / 4 && row0 + mtl * 16 < Bp;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int cp = 0; cp < G; ++cp) {
          const int* src = a.h1pre + (qok[k] ? (s * G + cp) * (int64_t)Bp * L1 + (int64_t)row0 * L1 + f4 * 4 : 0);
          qs[k][s][cp] = *reinterpret_cast<const int4*>(src);
        }
    }
    // labels of both ring slots (staged by the previous step; -1 past B)
    const bool yok = tid < BC && row0 + tid < Bp;
    const int yt = yok ? row0 + tid : 0;
    const int y0 = a.yring[yt], y1 = a.yring[Bp + yt];
    // ---- every weight fragment this wave needs, issued right behind the H1pre /
    // label loads the first barrier waits for (the in-order vmcnt lets the
    // fragments stay in flight across it): one L2 round trip in total ----
    bf16x8 w2f[NTW2][KS2];
    bf16x8 w3tf[NTW2];
    // clamped address + select: the load itself is never conditional
    auto ld8z = [&](bool ok, int64_t off) { const bf16x8 v = ld8(SH + (ok ? off : 0)); return ok ? v : zero8(); };
#pragma unroll
    for (int j = 0; j < NTW2; ++j) {
      const int nt = nt_base + kWaves * j;
      const bool ok = l2_active && nt < C::TN2;
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks)
        w2f[j][ks] = ld8z(ok, O::W2 + (int64_t)(nt * 16 + r16) * L1 + ks * 32 + 8 * g);
      w3tf[j] = ld8z(ok && g < 2, O::W3T + (int64_t)(nt * 16 + r16) * 16 + 8 * g);
    }
    const int mt3 = w % MT, kg3 = w / MT;
    bf16x8 w3f[KPG3];
#pragma unroll
    for (int i = 0; i < KPG3; ++i)
      w3f[i] = ld8z(kg3 < KG3 && r16 < kNC, O::W3 + (int64_t)r16 * L2 + (kg3 * KPG3 + i) * 32 + 8 * g);
    // dH1 with a short K (KG1 == 1) and few tiles: one (column, row) tile per wave
    constexpr bool ROW1 = KG1 == 1 && C::TN1 * MT <= kWaves;
    constexpr int MTW1 = ROW1 ? 1 : MT;
    const int ct1 = w % C::TN1, kg1 = ROW1 ? (w < C::TN1 * MT ? 0 : 1) : w / C::TN1;
    const int mt1_base = ROW1 ? w / C::TN1 : 0;
    bf16x8 w2tf[KPG1];
#pragma unroll
    for (int i = 0; i < KPG1; ++i)
      w2tf[i] = ld8z(kg1 < KG1, O::W2T + (int64_t)(ct1 * 16 + r16) * L2 + (kg1 * KPG1 + i) * 32 + 8 * g);
    if constexpr (REP) {
      asm volatile("" ::: "memory");  // the hook's loads stay younger than every load above
      hook();
      asm volatile("" ::: "memory");
    }
    // LDS writes last: their waits cover only the earliest loads (in-order vmcnt)
    if (tid < NBIAS) sBias[tid] = bias_v;
    if (tid < BC) sY[tid] = yok ? (slot ? y1 : y0) : -1;
    __syncthreads();  // sBias ready

    // ---- H1 = relu(H1pre + b1); H1pre chunk is contiguous in fragment order ----
    {
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const int f4 = tid + k * kThreads;
        if (f4 >= BC * L1 / 4) continue;
        if (!qok[k])
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int cp = 0; cp < G; ++cp) qs[k][s][cp] = make_int4(0, 0, 0, 0);
        const int f = f4 * 4;
        const int ln = f & 63, i = (f >> 6) & 3, blk = f >> 8;
        const int ct = blk % C::TN1, mtl = blk / C::TN1;
        const int b = mtl * 16 + 4 * (ln >> 4) + i, m = ct * 16 + (ln & 15);
        // both slots converted, the RESULT selected: selecting the loaded pairs
        // made the compiler index qs at run time (qs in scratch, and a wait on
        // the H1pre loads right at issue, ahead of the weight-fragment loads)
        bf16x4 hs[2];
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          int q[4] = {qs[k][sl][0].x, qs[k][sl][0].y, qs[k][sl][0].z, qs[k][sl][0].w};
#pragma unroll
          for (int cp = 1; cp < G; ++cp) {  // two's-complement adds: exact while the true sum fits
            q[0] += qs[k][sl][cp].x;
            q[1] += qs[k][sl][cp].y;
            q[2] += qs[k][sl][cp].z;
            q[3] += qs[k][sl][cp].w;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) hs[sl][k] = relu_bf(fixed_to_f32(q[k]) + sBias[m + k]);
        }
        const bf16x4 h = slot ? hs[1] : hs[0];
        *reinterpret_cast<bf16x4*>(sH1 + b * C::H1S + m) = h;
#pragma unroll
        for (int k = 0; k < 4; ++k) sH1T[(m + k) * C::TS + b] = h[k];
      }
    }
    __syncthreads();
    if (stamp_ok) a.stamps[1] = __builtin_amdgcn_s_memrealtime();
    if constexpr (!REP) copy_rows(sH1T, L1, A::H1T, row0);

    // ---------------- layer 2: H2 = relu(H1 W2^T + b2) ----------------
#pragma unroll
    for (int j = 0; j < NTW2; ++j) {
      const int nt = nt_base + kWaves * j;
      if (!l2_active || nt >= C::TN2) continue;
      const int n = nt * 16 + r16;
      const float bias = sBias[L1 + n];
#pragma unroll
      for (int mi = 0; mi < MTW2; ++mi) {
        const int mt = mt_base + mi;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS2; ++ks)
          acc = mfma16(ld8(sH1 + (mt * 16 + r16) * C::H1S + ks * 32 + 8 * g), w2f[j][ks], acc);
        bf16x4 t4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const __bf16 h = relu_bf(acc[i] + bias);
          sH2[(mt * 16 + 4 * g + i) * C::H2S + n] = h;
          t4[i] = h;
        }
        if constexpr (REP) *reinterpret_cast<bf16x4*>(sH2T + n * C::TS + mt * 16 + 4 * g) = t4;
        else if (row0 + mt * 16 < Bp)
          *reinterpret_cast<bf16x4*>(ACT + (int64_t)(A::H2T + n) * Bp + row0 + mt * 16 + 4 * g) = t4;
      }
    }
    __syncthreads();

    // ---------------- layer 3 (logits), K split over waves ----------------
    if (kg3 < KG3) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < KPG3; ++i)
        acc = mfma16(ld8(sH2 + (mt3 * 16 + r16) * C::H2S + (kg3 * KPG3 + i) * 32 + 8 * g), w3f[i], acc);
      if (r16 < kNC) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = (mt3 * 16 + 4 * g + i) * 16 + r16;
          if constexpr (KG3 == 1) sZ[e] = acc[i] + sBias[L1 + L2 + r16];
          else sPart[kg3 * BC * 16 + e] = acc[i];
        }
      }
    }
    __syncthreads();
    if constexpr (KG3 > 1) {
      for (int e = tid; e < BC * 16; e += kThreads) {
        const int j = e & 15;
        if (j >= kNC) continue;
        float z = 0.f;
#pragma unroll
        for (int k = 0; k < KG3; ++k) z += sPart[k * BC * 16 + e];
        sZ[e] = z + sBias[L1 + L2 + j];
      }
      __syncthreads();
    }
    if (stamp_ok) a.stamps[2] = __builtin_amdgcn_s_memrealtime();
    if constexpr (REP) {
      // One-launch acknowledgement, as early as it is safe: the rest of the head
      // pass reads LDS only, so once every wave's global loads (state, H1pre,
      // labels, weight fragments, biases, the block's own prologue loads) have
      // landed, nothing of this step's state is read by this block any more.  The
      // writers of that state (small blocks: weights / biases; block 0: counters,
      // the consumed H1pre slot) then wait for every block's LOADS instead of every
      // block's whole head pass.  (The weight fragments of dH2 / dH1 were issued
      // in the prologue ~1.5 us earlier: this wait costs little.)
      // The wait as the BUILTIN (not inline asm), so the compiler's own wait bookkeeping
      // sees it; it waits for every load older than the hook's (all shared state).
      // gfx9 encoding: vmcnt in bits 3:0, expcnt 7 (bits 6:4), lgkmcnt 15 (bits 11:8).
      asm volatile("" ::: "memory");
      static_assert(kRepHookLoads < 16, "vmcnt immediate");
      __builtin_amdgcn_s_waitcnt(0x0F70 | kRepHookLoads);  // vmcnt(kRepHookLoads): the hook's loads may fly on
      asm volatile("" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add(reinterpret_cast<long long*>(a.hand + kHandAck), 1ll, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      if (pre->active) {
        if constexpr (PreWave<L1>::hidden) {
          // lane l: the 16 pixels of row (l & 31) -> raw + 16 l; dword (l & 1) of the
          // label of row (l >> 1) -> raw + 1024 + 4 l (row r's int64 at raw + 1024 + 8 r)
          const int64_t sr = __shfl(pre->si, lane >> 1, 64);
          dma_lds16(a.x_u8 + pre->si * kD + pre->kt * 16, pre->raw);
          dma_lds4(reinterpret_cast<const char*>(a.labels + sr) + 4 * (lane & 1), pre->raw + 1024u);
        } else {
          pre->xn = *reinterpret_cast<const uint4*>(a.x_u8 + pre->si * kD + pre->kt * 16);
          pre->yn = a.labels[pre->si];
        }
      }
    }

    // ---------------- log_softmax / NLL / accuracy / dZ (one row per lane) -------------
    if (w < (BC + 63) / 64) {
      const int r = w * 64 + lane;
      float loss = 0.f, correct = 0.f, cnt = 0.f;
      bf16x8 d8[2];
      d8[0] = zero8();
      d8[1] = zero8();
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
        for (int q = 0; q < 2; ++q) *reinterpret_cast<bf16x8*>(sdZ + r * kDZS + 8 * q) = d8[q];
        *reinterpret_cast<bf16x8*>(sdZ + r * kDZS + 16) = zero8();
        *reinterpret_cast<bf16x8*>(sdZ + r * kDZS + 24) = zero8();
#pragma unroll
        for (int j = 0; j < 16; ++j) sdZT[j * C::TS + r] = (j < kNC) ? d8[j >> 3][j & 7] : (__bf16)0.f;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        loss += __shfl_xor(loss, off, 64);
        correct += __shfl_xor(correct, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
      }
      if (lane == 0) {
        atomicAdd(&misc[0], loss);
        atomicAdd(&misc[1], correct);
        atomicAdd(&misc[2], cnt);
      }
    }
    __syncthreads();
    if constexpr (!REP) copy_rows(sdZT, 16, A::DZT, row0);

    // ---------------- dH2 = (dZ W3) * (H2 > 0), in place over H2 ----------------
#pragma unroll
    for (int j = 0; j < NTW2; ++j) {
      const int nt = nt_base + kWaves * j;
      if (!l2_active || nt >= C::TN2) continue;
      const int n = nt * 16 + r16;
#pragma unroll
      for (int mi = 0; mi < MTW2; ++mi) {
        const int mt = mt_base + mi;
        const f32x4 acc = mfma16(ld8(sdZ + (mt * 16 + r16) * kDZS + 8 * g), w3tf[j], f32x4{0.f, 0.f, 0.f, 0.f});
        bf16x4 t4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __bf16* hp = sH2 + (mt * 16 + 4 * g + i) * C::H2S + n;
          const __bf16 d = ((float)(*hp) > 0.f) ? (__bf16)acc[i] : (__bf16)0.f;
          *hp = d;
          t4[i] = d;
        }
        if constexpr (REP) *reinterpret_cast<bf16x4*>(sDH2T + n * C::TS + mt * 16 + 4 * g) = t4;
        else if (row0 + mt * 16 < Bp)
          *reinterpret_cast<bf16x4*>(ACT + (int64_t)(A::DH2T + n) * Bp + row0 + mt * 16 + 4 * g) = t4;
      }
    }
    __syncthreads();

    // ---------------- dH1 = (dH2 W2) * (H1 > 0) -> dh1t, K split over waves ----------------
    if (kg1 < KG1) {
      const int m = ct1 * 16 + r16;
#pragma unroll
      for (int mi = 0; mi < MTW1; ++mi) {
        const int mt = mt1_base + mi;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < KPG1; ++i)
          acc = mfma16(ld8(sH2 + (mt * 16 + r16) * C::H2S + (kg1 * KPG1 + i) * 32 + 8 * g), w2tf[i], acc);
        if constexpr (KG1 == 1) {
          bf16x4 t4;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const __bf16 hv = sH1[(mt * 16 + 4 * g + i) * C::H1S + m];
            t4[i] = ((float)hv > 0.f) ? (__bf16)acc[i] : (__bf16)0.f;
          }
          if constexpr (REP) *reinterpret_cast<bf16x4*>(sDH1T + m * C::TS + mt * 16 + 4 * g) = t4;
          else if (row0 + mt * 16 < Bp)
            *reinterpret_cast<bf16x4*>(DH1T + (int64_t)m * Bp + row0 + mt * 16 + 4 * g) = t4;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) sPart[(kg1 * BC + mt * 16 + 4 * g + i) * L1 + m] = acc[i];
        }
      }
    }
    if constexpr (KG1 > 1) {
      __syncthreads();
      // fixed-order reduction of the K groups; 4 consecutive rows per item (one bf16x4 store)
      for (int e = tid; e < L1 * (BC / 4); e += kThreads) {
        const int m = e % L1, q = e / L1;
        bf16x4 t4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = 4 * q + i;
          float v = 0.f;
#pragma unroll
          for (int k = 0; k < KG1; ++k) v += sPart[(k * BC + b) * L1 + m];
          const __bf16 hv = sH1[b * C::H1S + m];
          t4[i] = ((float)hv > 0.f) ? (__bf16)v : (__bf16)0.f;
        }
        if constexpr (REP) *reinterpret_cast<bf16x4*>(sDH1T + m * C::TS + 4 * q) = t4;
        else if (row0 + 4 * q < Bp) *reinterpret_cast<bf16x4*>(DH1T + (int64_t)m * Bp + row0 + 4 * q) = t4;
      }
    }
    __syncthreads();
    if (stamp_ok) a.stamps[3] = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (REP) return;  // loss stats stay in misc[0..3); block 0 publishes them
  if (tid == 0 && nchunks > 1) {
    // several row blocks: partial sums for tail block 0's ordered reduction
    a.head_part[c * 4 + 0] = misc[0];
    a.head_part[c * 4 + 1] = misc[1];
    a.head_part[c * 4 + 2] = misc[2];
  }
  if (tid == 0 && c == 0) {
    // the advanced state goes to the NEXT copy: this launch's gather blocks are
    // still reading the current one (the tail publishes it, see mlp3_tail_kernel).
    int64_t* cn = a.counters + kCnt;
    cn[0] = a.advance_step ? t : t - 1;
    cn[2] = cursor;
    int64_t nc = cursor + 1, nob = ob;
    if (nc >= a.n_batches) { nc = 0; nob ^= 1; }
    cn[1] = nc;
    cn[4] = nob;
    cn[3] = slot ^ 1;
    if (a.stats && nchunks == 1) {
      const int s = (int)((t - 1) % (a.stats_ring > 0 ? a.stats_ring : 1));
      float* st = a.stats + s * 4;
      st[0] = misc[0] * invB;
      st[1] = misc[1];
      st[2] = misc[2];
      st[3] = (float)t;
    }
    if (a.stamps) a.stamps[4] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int BC, int L1, int L2, bool MULTI>
__global__ __launch_bounds__(kThreads) void mlp3_head_kernel(MLP3Args a) {
  __shared__ __attribute__((aligned(16))) char smem[Cfg3<BC, L1, L2>::total];
  const int nchunks = MULTI ? (a.B + BC - 1) / BC : 1;
  if ((int)blockIdx.x >= nchunks) {  // the NEXT batch's tiles, for this step's tail (xring / yring slot ^ 1)
    int64_t nc = a.counters[1] + 1, nob = a.counters[4];
    if (nc >= a.n_batches) { nc = 0; nob ^= 1; }
    gather_tile(a, (int)blockIdx.x - nchunks, nob, nc, a.counters[3] ^ 1, kThreads);
    stamp_max(a, 5);
    return;
  }
  head_body<BC, L1, L2, MULTI, false>(a, smem);
}

// ---------------------------------------------------------------------------
// Tail kernel pieces
// ---------------------------------------------------------------------------
template <int L1, int L2>
struct SmallTasks {
  static constexpr int TN1 = L1 / 16, TN2 = L2 / 16;
  static constexpr int NT_W2 = TN1 * TN2, NT_W3 = TN2, NTILE = NT_W2 + NT_W3;
  static constexpr int NBIAS = L1 + L2 + kNC, NBW = (NBIAS + 63) / 64;
  static constexpr int NTASK = NTILE + NBW;
  static constexpr int NBLK = (NTASK + TN1 - 1) / TN1;  // tail blocks have TN1 waves
};

// One wave's share of the small parameters: a 16x16 tile of dW2 or dW3 (4
// values per lane), or 64 biases (1 per lane).  small_compute produces the
// gradient values (+ prefetched Adam state); small_finalize applies Adam (or
// stores gradients).  The fused data-parallel tail exchanges the values over
// xGMI between the two halves.
struct SmallRes {
  float v[4], pv[4], mv[4], vv[4];
  int64_t gi[4];
  bool valid[4];
  int kind;  // 0 W2 tile, 1 W3 tile, 2 bias, -1 idle lane / wave
  int rowv, colv;
};

// LDS images of the one-launch block's own head pass ([rows][ts] bf16, batch-contiguous rows)
struct RepLds {
  const __bf16 *h1t, *h2t, *dh2t, *dzt, *dh1t;
  int ts;
};

// REP (the one-launch step): called twice -- L == nullptr: task setup + Adam
// prefetch only (before the block's head pass); then with L: the gradient from
// this block's LDS images instead of act / dh1t (r keeps the first call's state)
template <int L1, int L2, bool REP = false>
__device__ __forceinline__ void small_compute(const MLP3Args& a, bool prefetch_adam, int task, SmallRes& r,
                                              const RepLds* L = nullptr) {
  const bool setup = !REP || L == nullptr, compute = !REP || L != nullptr;
  using O = Off<L1, L2>;
  using A = Act<L1, L2>;
  using S = SmallTasks<L1, L2>;
  const int lane = threadIdx.x & 63, r16 = lane & 15, g = lane >> 4;
  const int Bp = (a.B + 31) / 32 * 32;
  const __bf16* ACT = reinterpret_cast<const __bf16*>(a.act);
  const __bf16 *arow_l = nullptr, *brow_l = nullptr;  // REP: LDS rows of the two MFMA operands
  if (setup) {
    r.kind = -1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r.v[i] = r.pv[i] = r.mv[i] = r.vv[i] = 0.f;
      r.gi[i] = 0;
      r.valid[i] = false;
    }
  }
  if (task < S::NTILE) {
    const __bf16 *arow, *brow;
    if (task < S::NT_W2) {  // dW2[n][m] = sum_b dH2[b][n] H1[b][m]
      const int nt = task % S::TN2, ct = task / S::TN2;
      if (setup) {
        r.kind = 0;
        r.rowv = nt * 16 + 4 * g;
        r.colv = ct * 16 + r16;
      }
      arow = ACT + (int64_t)(A::DH2T + nt * 16 + r16) * Bp;
      brow = ACT + (int64_t)(A::H1T + ct * 16 + r16) * Bp;
      if constexpr (REP) {
        arow_l = L->dh2t + (nt * 16 + r16) * L->ts;
        brow_l = L->h1t + (ct * 16 + r16) * L->ts;
      }
      if (setup)
#pragma unroll
        for (int i = 0; i < 4; ++i) { r.gi[i] = O::W2 + (int64_t)(r.rowv + i) * L1 + r.colv; r.valid[i] = true; }
    } else {  // dW3[j][n] = sum_b dZ[b][j] H2[b][n]
      const int nt = task - S::NT_W2;
      if (setup) {
        r.kind = 1;
        r.rowv = 4 * g;
        r.colv = nt * 16 + r16;
      }
      arow = ACT + (int64_t)(A::DZT + r16) * Bp;
      brow = ACT + (int64_t)(A::H2T + nt * 16 + r16) * Bp;
      if constexpr (REP) {
        arow_l = L->dzt + r16 * L->ts;
        brow_l = L->h2t + (nt * 16 + r16) * L->ts;
      }
      if (setup)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          r.valid[i] = (r.rowv + i) < kNC;
          r.gi[i] = O::W3 + (int64_t)(r.valid[i] ? r.rowv + i : 0) * L2 + r.colv;
        }
    }
    if (setup && prefetch_adam)
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // unconditional: gi is in bounds for invalid rows too (row 0)
        r.pv[i] = a.params[r.gi[i]]; r.mv[i] = a.exp_avg[r.gi[i]]; r.vv[i] = a.exp_avg_sq[r.gi[i]];
      }
    if (!compute) return;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (REP) {
      acc = mfma16(ld8(arow_l + 8 * g), ld8(brow_l + 8 * g), acc);  // Bp = 32: one k-step
    } else {
      for (int ks = 0; ks < Bp / 32; ++ks) {
        const int b0 = ks * 32 + 8 * g;
        acc = mfma16(ld8(arow + b0), ld8(brow + b0), acc);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = acc[i];
  } else {  // 64 biases per wave: row sums of dH1^T / dH2^T / dZ^T
    const int e = (task - S::NTILE) * 64 + lane;
    if (e >= S::NBIAS) return;
    const __bf16* row;
    if (e < L1) {
      row = REP ? L->dh1t + e * L->ts : reinterpret_cast<const __bf16*>(a.dh1t) + (int64_t)e * Bp;
      r.gi[0] = O::B1 + e;
    } else if (e < L1 + L2) {
      row = REP ? L->dh2t + (e - L1) * L->ts : ACT + (int64_t)(A::DH2T + e - L1) * Bp;
      r.gi[0] = O::B2 + (e - L1);
    } else {
      row = REP ? L->dzt + (e - L1 - L2) * L->ts : ACT + (int64_t)(A::DZT + e - L1 - L2) * Bp;
      r.gi[0] = O::B3 + (e - L1 - L2);
    }
    if (setup) {
      r.kind = 2;
      r.valid[0] = true;
      if (prefetch_adam) { r.pv[0] = a.params[r.gi[0]]; r.mv[0] = a.exp_avg[r.gi[0]]; r.vv[0] = a.exp_avg_sq[r.gi[0]]; }
    }
    if (!compute) return;
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

    // 32 rows per group: four independent 16-byte loads in flight before any add
    // (a one-load-per-iteration loop made this wave the tail kernel's straggler)
    for (int b0 = 0; b0 < Bp; b0 += 32) {
      bf16x8 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = ld8(row + b0 + 8 * q);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) s8[j] += (float)v[q][j];
    }
    r.v[0] = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  }
}

template <int L1, int L2>
__device__ __forceinline__ void small_finalize(const MLP3Args& a, bool adam, const SmallRes& r, const AdamScal& o) {
  using O = Off<L1, L2>;
  if (r.kind < 0) return;
  __bf16* SHW = reinterpret_cast<__bf16*>(a.shadow);
  bf16x4 sh4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sh4[i] = (__bf16)0.f;
    if (!r.valid[i]) continue;
    if (adam) {
      float m_ = r.mv[i], v_ = r.vv[i];
      const float p_ = adam1(r.pv[i], r.v[i], m_, v_, o);
      a.params[r.gi[i]] = p_;
      a.exp_avg[r.gi[i]] = m_;
      a.exp_avg_sq[r.gi[i]] = v_;
      SHW[r.gi[i]] = (__bf16)p_;
      sh4[i] = (__bf16)p_;
    } else {
      a.grads[r.gi[i]] = r.v[i];
    }
  }
  if (adam && r.kind == 0) *reinterpret_cast<bf16x4*>(SHW + O::W2T + (int64_t)r.colv * L2 + r.rowv) = sh4;
  if (adam && r.kind == 1) *reinterpret_cast<bf16x4*>(SHW + O::W3T + (int64_t)r.colv * 16 + r.rowv) = sh4;
}

// Owner protocol: r.v[] already holds the new fp32 weights (from the owner's Adam or
// its all-gather); store them and the bf16 shadows, and m / v where this rank owns
// the task (r.mv / r.vv advanced by the owner's Adam).
template <int L1, int L2>
__device__ __forceinline__ void small_store(const MLP3Args& a, const SmallRes& r, bool store_mv) {
  using O = Off<L1, L2>;
  if (r.kind < 0) return;
  __bf16* SHW = reinterpret_cast<__bf16*>(a.shadow);
  bf16x4 sh4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sh4[i] = (__bf16)0.f;
    if (!r.valid[i]) continue;
    a.params[r.gi[i]] = r.v[i];
    if (store_mv) {
      a.exp_avg[r.gi[i]] = r.mv[i];
      a.exp_avg_sq[r.gi[i]] = r.vv[i];
    }
    SHW[r.gi[i]] = (__bf16)r.v[i];
    sh4[i] = (__bf16)r.v[i];
  }
  if (r.kind == 0) *reinterpret_cast<bf16x4*>(SHW + O::W2T + (int64_t)r.colv * L2 + r.rowv) = sh4;
  if (r.kind == 1) *reinterpret_cast<bf16x4*>(SHW + O::W3T + (int64_t)r.colv * 16 + r.rowv) = sh4;
}

// ---------------------------------------------------------------------------
// In-kernel xGMI exchange of the fused data-parallel tail (kind StepDP): every
// block pushes its gradient values into the peers' receive areas (at their arena
// index), raises its per-(slot, block, rank) generation flag on every rank,
// waits for the same block of every other rank, and sums the W contributions in
// fixed rank order -- the allreduce happens inside the optimizer epilogue.
// Protocol and memory rules as in csrc/comm/xgmi_allreduce.hip (aux region).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t* dp_flag(char* region, int slot, int blk, int src) {
  return reinterpret_cast<uint32_t*>(region) + ((size_t)slot * kDpMaxBlocks + blk) * kXgmiMaxRanks + src;
}
__device__ __forceinline__ float* dp_data(char* region, int slot, int src, int64_t stride) {
  return reinterpret_cast<float*>(region + kXgmiFlagBytes) + ((int64_t)slot * kXgmiMaxRanks + src) * stride;
}

// all threads of the block; returns the receive slot; *fail set on a poll timeout
__device__ __forceinline__ int dp_begin(const MLP3Args& a, uint32_t* sh_gen) {
  if (threadIdx.x == 0) *sh_gen = a.dp_gen[blockIdx.x] + 1u;
  __syncthreads();
  return (int)(*sh_gen & 1u);
}

__device__ __forceinline__ void dp_signal_and_wait(const MLP3Args& a, uint32_t gen, int slot, int* sh_fail) {
  if (a.dp_lite) {
    // One wave fences (guide's producer/consumer form, system scope): every wave
    // drains its pushes, the block barrier orders them before wave 0's release
    // fence and flag stores; wave 0 polls, ONE acquire, barrier, then everyone
    // reads.  The all-threads form below paid a system fence per wave, twice.
    const int tid = threadIdx.x, blk = blockIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < 64) {
      if (tid == 0) *sh_fail = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid < a.dp_world)
        __hip_atomic_store(dp_flag(a.dp_regions[tid], slot, blk, a.dp_rank), gen, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      if (tid < a.dp_world) {
        uint32_t* f = dp_flag(a.dp_regions[a.dp_rank], slot, blk, tid);
        int64_t spins = 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != gen) {
          if (++spins > a.dp_spin) {
            *sh_fail = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
      a.dp_gen[blk] = gen;
      if (*sh_fail) __hip_atomic_store(a.dp_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  __threadfence_system();
  __syncthreads();
  const int tid = threadIdx.x, blk = blockIdx.x;
  if (tid == 0) *sh_fail = 0;
  if (tid < a.dp_world)
    __hip_atomic_store(dp_flag(a.dp_regions[tid], slot, blk, a.dp_rank), gen, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (tid < a.dp_world) {
    uint32_t* f = dp_flag(a.dp_regions[a.dp_rank], slot, blk, tid);
    int64_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != gen) {
      if (++spins > a.dp_spin) {
        *sh_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __threadfence_system();
  __syncthreads();
  if (tid == 0) {
    a.dp_gen[blk] = gen;
    if (*sh_fail) __hip_atomic_store(a.dp_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ void dp_push1(const MLP3Args& a, int slot, int64_t idx, float v) {
  for (int r = 0; r < a.dp_world; ++r)
    __builtin_nontemporal_store(v, dp_data(a.dp_regions[r], slot, a.dp_rank, a.dp_stride) + idx);
}

// ---- tagged granules (dp_lite == 2, default): every value travels as ONE 8-byte
// {generation, fp32 bits} word, written by one system-scope store and read by
// system-scope loads.  A reader accepts a word only when its tag is this step's
// generation, so no flag, no release fence and no acquire fence are needed (an
// aligned 8-byte store is never torn); the double-buffered slots and the
// monotonic per-block generation keep the previous steps' words from matching.
// Twice the bytes of the flag form, ~1 us less latency per exchange on one GPU.
__device__ __forceinline__ unsigned long long* dp_gran(char* region, int slot, int src, int64_t stride) {
  // stride floats per (slot, src) area -> stride / 2 granules
  return reinterpret_cast<unsigned long long*>(region + kXgmiFlagBytes) + ((int64_t)slot * kXgmiMaxRanks + src) * (stride / 2);
}

__device__ __forceinline__ void dp_push_gran(const MLP3Args& a, int slot, int64_t idx, float v, uint32_t gen) {
  const unsigned long long w = ((unsigned long long)gen << 32) | (unsigned long long)__float_as_uint(v);
  for (int r = 0; r < a.dp_world; ++r)
    __hip_atomic_store(dp_gran(a.dp_regions[r], slot, a.dp_rank, a.dp_stride) + idx, w, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// fixed rank-order sum of the W granules of value idx; sets *fail on a poll timeout
__device__ __forceinline__ float dp_sum_gran(const MLP3Args& a, int slot, int64_t idx, uint32_t gen, int* fail) {
  float s = 0.f;
  for (int r = 0; r < a.dp_world; ++r) {
    unsigned long long* p = dp_gran(a.dp_regions[a.dp_rank], slot, r, a.dp_stride) + idx;
    unsigned long long w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    int64_t spins = 0;
    while ((uint32_t)(w >> 32) != gen) {
      if (++spins > a.dp_spin) {
        *fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    s += __uint_as_float((uint32_t)w);
  }
  return s;
}

// block epilogue of a granule exchange: publish the generation, report timeouts
__device__ __forceinline__ void dp_gran_end(const MLP3Args& a, uint32_t gen, int fail, int* sh_fail) {
  if (threadIdx.x == 0) *sh_fail = 0;
  __syncthreads();
  if (fail) *sh_fail = 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    a.dp_gen[blockIdx.x] = gen;
    if (*sh_fail) __hip_atomic_store(a.dp_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__device__ __forceinline__ float dp_sum1(const MLP3Args& a, int slot, int64_t idx) {
  float s = 0.f;
  for (int r = 0; r < a.dp_world; ++r)
    s += __builtin_nontemporal_load(dp_data(a.dp_regions[a.dp_rank], slot, r, a.dp_stride) + idx);
  return s;
}

// ---------------------------------------------------------------------------
// Wave-positioned exchange protocols of the one-launch data-parallel step
// (a.dp_proto 1 "packed", 2 "owner"; layout in comm/xgmi.h).  The unit of
// exchange is one wave: 64 lanes x 4 values (a 16x16 gradient tile, 64 biases, or
// a W1 tile's 16-neuron slice), at unit = block * 8 + wave.
//
// Cost model per step, world N, P parameters (4P bytes of fp32 gradient), per link:
//   round-2 granules  (N-1 peers) x 8P bytes out, 8P per link     one hop
//   packed one-shot   4P per link (two values per 8-B granule)    one hop
//   owner             4P/N (reduce-scatter) + 8P/N (all-gather)   two hops
// At the default 32-64 model (P = 27,882) and N = 8: 223 / 112 / 42 KB per link.
// Which wins depends on the link's small-write bandwidth against its one-way
// latency (break-even ~ (70 KB / bandwidth) = one extra hop) -- measured per job:
// bench.py times both at start-up and keeps the faster (scripts/dp_overhead_probe.py
// prices the in-kernel part with loopback ranks).
//
// Packed granule: {bits(v0) rounded to a multiple of 4 ulp | tag, bits(v1)}; the
// 2-bit tag ((gen >> 1) & 3) is this step's: a slot (gen & 1) is rewritten every
// second step, so its stale granules carry the previous tag (gen - 2).  Regions are
// re-armed (all bits set: tag 3; generations 0) whenever a job starts using them,
// so the first tag-3 step (gen 6) finds slot 0 already rewritten at gen 4.  An
// aligned 8-byte store is not torn, so no flag and no fence: a reader accepts a
// granule exactly when its tag matches.  Gradient values lose at most 2 ulp of
// fp32 (2^-22 relative) on the wire; every rank sums the SAME granules in fixed
// rank order (its own from registers, rounded identically), so replicas stay
// bitwise equal.
// ---------------------------------------------------------------------------
typedef unsigned long long u64;

// v0's wire form: rounded to a multiple of 4 ulp, never carried into the exponent
// (a mantissa within 2 ulp of all-ones truncates: FLT_MAX stays finite), non-finite
// values kept non-finite -- an infinity keeps a zero mantissa above the tag bits
// (the reader masks them off), a NaN gets its quiet bit so the tag cannot turn it
// into an infinity.
__device__ __forceinline__ uint32_t pk_round(float v) {
  const uint32_t b = __float_as_uint(v), man = b & 0x7fffffu;
  uint32_t r = man >= 0x7ffffeu ? b : b + 2u;
  if ((b & 0x7f800000u) == 0x7f800000u) r = man ? (b | 0x400000u) : b;
  return r & ~3u;
}
__device__ __forceinline__ u64 pk2(float v0, float v1, uint32_t tag) {
  return ((u64)__float_as_uint(v1) << 32) | (u64)(pk_round(v0) | tag);
}
__device__ __forceinline__ float pk_lo(u64 w) { return __uint_as_float((uint32_t)w & ~3u); }
__device__ __forceinline__ float pk_hi(u64 w) { return __uint_as_float((uint32_t)(w >> 32)); }

// Wire layout (round 4): each lane's share of a unit is CONTIGUOUS -- packed /
// reduce-scatter area: lane l's two granules {g0, g1} at u64 [2l, 2l + 1] of the
// unit's 1 KB; all-gather area: its four {gen, fp32} granules at u64 [4l, 4l + 3]
// of 2 KB -- so a lane moves 16 B per instruction (buffer_load / store_dwordx4 sc0
// sc1) instead of 8 B: half the poll and push instructions, and 16-B system-scope
// accesses run at the full rate where 8-B ones ran at 0.54-0.70x of it
// (MI355X_MICROARCH.md, the visibility table).  Each 8-B granule still carries its
// own tag / generation, so a 16-B access torn between its halves is harmless.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// byte offsets inside a region
__device__ __forceinline__ uint32_t dp_pk_off(int slot, int src, int unit) {
  return (uint32_t)(kXgmiFlagBytes + ((((int64_t)slot * kXgmiMaxRanks + src) * comm::kDpMaxUnits + unit) * 128) * 8);
}
__device__ __forceinline__ uint32_t dp_ag_off(int slot, int unit) {
  return (uint32_t)(kXgmiFlagBytes + (comm::kDpPackedGranules + ((int64_t)slot * comm::kDpMaxUnits + unit) * 256) * 8);
}
constexpr uint32_t kDpSrcBytes = (uint32_t)comm::kDpMaxUnits * 128 * 8;  // bytes per source rank of a slot
static_assert((int64_t)kXgmiFlagBytes + (comm::kDpPackedGranules + comm::kDpGatherGranules) * 8 < (1ll << 31),
              "32-bit buffer offsets");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dp_rsrc(char* region) {
  // raw buffer over the whole region (gfx9 dword3); offsets stay below 2^31
  return __builtin_amdgcn_make_buffer_rsrc(region, 0, 0x7fffffff, 0x00020000);
}
constexpr int kSysPolicy = 1 | 16;  // sc0 | sc1: system scope (peer memory over xGMI)
__device__ __forceinline__ void st_sys2(__amdgpu_buffer_rsrc_t r, uint32_t off, u64 a, u64 b) {
  const u32x4_t v = {(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kSysPolicy);
}
__device__ __forceinline__ void ld_sys2(__amdgpu_buffer_rsrc_t r, uint32_t off, u64& a, u64& b) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSysPolicy);
  a = (u64)v[0] | ((u64)v[1] << 32);
  b = (u64)v[2] | ((u64)v[3] << 32);
}

// Polls of the wave-positioned protocols are compiled for a rank CLASS NW (the
// world size rounded up to 2, 4 or 8: one kernel instance each), so every loop
// below is unrolled over compile-time indices and every load is unconditional: a
// per-element "load if i < n" on a run-time n made hipcc branch around each load
// and wait vmcnt(0) per element (profiles/r4_dp: the round-3 instance that took a
// run-time world size).  Peer slots k < NW - 1 that the actual world does not have
// re-read our own source slot (a valid address) and are never checked.
constexpr int kDpPeerGran = 2 * (kXgmiMaxRanks - 1);

// peer slot k (0..NW-2) -> its rank: the ranks in order, ours skipped
__device__ __forceinline__ int dp_peer(int k, int me) { return k < me ? k : k + 1; }

// issue the 2 (NW - 1) peer granules of (slot, unit) in our own region: granule 2k + h
// is half h of peer k's contribution
// (src0: byte offset of source rank 0's area of this slot / unit, plus this lane's 16 B)
template <int NW>
__device__ __forceinline__ void dp_peer_issue(u64 (&w)[2 * (NW - 1)], __amdgpu_buffer_rsrc_t mine, uint32_t src0,
                                              int me, int W) {
#pragma unroll
  for (int k = 0; k < NW - 1; ++k) {
    const int s = dp_peer(k, me);
    ld_sys2(mine, src0 + (uint32_t)(s < W ? s : me) * kDpSrcBytes, w[2 * k], w[2 * k + 1]);
  }
}

// Wait until every real peer's two granules carry this step's tag (or the bound
// expires: *fail).  Re-polls re-issue all of them (unconditional, still one round
// trip; a matched granule is not rewritten before this wave's own next step).
template <int NW>
__device__ __forceinline__ void dp_peer_wait(const MLP3Args& a, u64 (&w)[2 * (NW - 1)], __amdgpu_buffer_rsrc_t mine,
                                             uint32_t src0, int me, int W, uint32_t tag, int* fail) {
  int64_t spins = 0;
  while (true) {
    bool all = true;
#pragma unroll
    for (int k = 0; k < NW - 1; ++k)
      if (dp_peer(k, me) < W) all = all && ((uint32_t)w[2 * k] & 3u) == tag && ((uint32_t)w[2 * k + 1] & 3u) == tag;
    if (all) return;
    if (++spins > a.dp_spin) {
      *fail = 1;
      return;
    }
    __builtin_amdgcn_s_sleep(1);
    dp_peer_issue<NW>(w, mine, src0, me, W);
  }
}

// Fixed-rank-order sum of every rank's packed contribution to this lane's 4 values
// (ours from registers, rounded as on the wire), times `scale`.
template <int NW>
__device__ __forceinline__ void dp_packed_sum(const u64 (&w)[2 * (NW - 1)], int me, int W, u64 g0, u64 g1,
                                              float (&v)[4], float scale) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
  for (int s = 0; s < NW; ++s) {
    if (s >= W) break;
    // rank s is peer slot s (below us) or s - 1 (above): both compile-time indices
    const int lo = s < NW - 1 ? s : 0, hi = s > 0 ? s - 1 : 0;
    u64 a0 = g0, a1 = g1;
    if (s < me) { a0 = w[2 * lo]; a1 = w[2 * lo + 1]; }
    else if (s > me) { a0 = w[2 * hi]; a1 = w[2 * hi + 1]; }
    s0 += pk_lo(a0); s1 += pk_hi(a0); s2 += pk_lo(a1); s3 += pk_hi(a1);
  }
  v[0] = s0 * scale; v[1] = s1 * scale; v[2] = s2 * scale; v[3] = s3 * scale;
}

__device__ __forceinline__ void dp_push_packed(char* region, int slot, int src, int unit, u64 g0, u64 g1) {
  st_sys2(dp_rsrc(region), dp_pk_off(slot, src, unit) + 16u * (threadIdx.x & 63), g0, g1);
}

// this rank's contribution to every peer (loopback: into every peer's source slot
// of our own region)
template <int NW>
__device__ __forceinline__ void dp_push_all(const MLP3Args& a, int slot, int unit, u64 g0, u64 g1) {
  const int me = a.dp_rank, W = a.dp_world;
#pragma unroll
  for (int r = 0; r < NW; ++r)
    if (r < W && r != me) dp_push_packed(a.dp_loop ? a.dp_regions[me] : a.dp_regions[r], slot, a.dp_loop ? r : me,
                                         unit, g0, g1);
}

// "packed" one-shot: push this wave's 4 values to every peer, sum all ranks' in
// fixed order; v[] becomes the sum times `scale`.  Whole-wave call.
template <int NW>
__device__ __forceinline__ void dp_packed_exchange(const MLP3Args& a, int unit, uint32_t gen, float (&v)[4],
                                                   float scale, int* fail) {
  const int slot = (int)(gen & 1u), me = a.dp_rank, W = a.dp_world;
  if (W == 1) {  // (uniform) nothing to exchange
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= scale;
    return;
  }
  const uint32_t tag = (gen >> 1) & 3u;
  const u64 g0 = pk2(v[0], v[1], tag), g1 = pk2(v[2], v[3], tag);
  const __amdgpu_buffer_rsrc_t mine = dp_rsrc(a.dp_regions[me]);
  const uint32_t src0 = dp_pk_off(slot, 0, unit) + 16u * (threadIdx.x & 63);
  u64 w[2 * (NW - 1)];
  // first polls before the pushes: gfx950 counts loads AND stores in one in-order
  // vmcnt, so pushes issued first would make the first wait cover their remote
  // completion too.  Loopback reads its own pushes: polls after them.
  if (!a.dp_loop) dp_peer_issue<NW>(w, mine, src0, me, W);
  dp_push_all<NW>(a, slot, unit, g0, g1);
  if (a.dp_loop) dp_peer_issue<NW>(w, mine, src0, me, W);
  dp_peer_wait<NW>(a, w, mine, src0, me, W, tag, fail);
  dp_packed_sum<NW>(w, me, W, g0, g1, v, scale);
}

// "owner": the task's gradient goes to its owner rank only (reduce-scatter, one
// hop: 1 / N of the one-shot bytes), the owner sums every rank's contribution,
// runs `adam(v)` (v: summed gradient in, new fp32 weights out; it also advances
// the caller's m / v registers) and publishes the weights to every other rank as
// {gen, fp32} granules (all-gather, the second hop); the others wait for them.
// On return v[] holds the new weights on every rank; true on the owner (whose
// m / v registers are then the ones to store).  Loopback: a wave whose task
// another (absent) rank owns plays that owner itself.
template <int NW, typename AdamFn>
__device__ __forceinline__ bool dp_owner_step(const MLP3Args& a, int unit, int owner, uint32_t gen, float (&v)[4],
                                              float scale, int* fail, AdamFn adam) {
  const int lane = threadIdx.x & 63, slot = (int)(gen & 1u), me = a.dp_rank, W = a.dp_world;
  if (W == 1) {  // (uniform) every task is ours and there is nothing to exchange
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= scale;
    adam(v);
    return true;
  }
  const uint32_t tag = (gen >> 1) & 3u;
  const bool own = owner == me;
  const u64 g0 = pk2(v[0], v[1], tag), g1 = pk2(v[2], v[3], tag);
  const __amdgpu_buffer_rsrc_t mine = dp_rsrc(a.dp_regions[me]);
  const uint32_t agsrc = dp_ag_off(slot, unit) + 32u * lane;
  u64 wa[4];
  auto ag_issue = [&]() {
    ld_sys2(mine, agsrc, wa[0], wa[1]);
    ld_sys2(mine, agsrc + 16u, wa[2], wa[3]);
  };
  if (!own && !a.dp_loop) ag_issue();  // first polls before the push
  if (!own) dp_push_packed(a.dp_regions[owner], slot, me, unit, g0, g1);
  if (own || a.dp_loop) {
    if (own) {
      const uint32_t src0 = dp_pk_off(slot, 0, unit) + 16u * lane;
      u64 w[2 * (NW - 1)];
      if (a.dp_loop) dp_push_all<NW>(a, slot, unit, g0, g1);
      dp_peer_issue<NW>(w, mine, src0, me, W);
      dp_peer_wait<NW>(a, w, mine, src0, me, W, tag, fail);
      dp_packed_sum<NW>(w, me, W, g0, g1, v, scale);
    } else {  // loopback stand-in of the owner: W identical contributions
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      for (int s = 0; s < W; ++s) { s0 += pk_lo(g0); s1 += pk_hi(g0); s2 += pk_lo(g1); s3 += pk_hi(g1); }
      v[0] = s0 * scale; v[1] = s1 * scale; v[2] = s2 * scale; v[3] = s3 * scale;
    }
    adam(v);
    const u64 tg = (u64)gen << 32;
#pragma unroll
    for (int r = 0; r < NW; ++r) {
      if (r >= W || (own ? r == me : r != owner)) continue;  // loopback stand-in: publish once, to ourselves
      const __amdgpu_buffer_rsrc_t dr = dp_rsrc(a.dp_regions[r]);
      const uint32_t off = dp_ag_off(slot, unit) + 32u * lane;
      st_sys2(dr, off, tg | (u64)__float_as_uint(v[0]), tg | (u64)__float_as_uint(v[1]));
      st_sys2(dr, off + 16u, tg | (u64)__float_as_uint(v[2]), tg | (u64)__float_as_uint(v[3]));
    }
    if (own) return true;
  }
  if (a.dp_loop) ag_issue();
  int64_t spins = 0;
  while (true) {
    bool all = true;
#pragma unroll
    for (int i = 0; i < 4; ++i) all = all && (uint32_t)(wa[i] >> 32) == gen;
    if (all) break;
    if (++spins > a.dp_spin) {
      *fail = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    ag_issue();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = __uint_as_float((uint32_t)wa[i]);
  return false;
}

// One-launch DP: this launch's generation, read with the step state at kernel start
// (the kernel boundary's cache invalidation covers it), so no block
// waits on a dependent global load and a barrier before its exchange; the end
// needs no barrier either (every thread holds the same value; timeouts go straight
// to the host-mapped error word).
__device__ __forceinline__ uint32_t dp_gen_now(const MLP3Args& a) {
  // a SCALAR load, issued with the step-state loads (ld_state) it is waited for
  // together with.  (Round 3 used a vector load here; hipcc proves the value
  // uniform, moves it to an SGPR with v_readfirstlane and waits vmcnt(0) for it
  // right at kernel start, ahead of every prefetch: +0.7-1 us on the head pass of
  // every exchange-capable instance, profiles/r4_dp.)
  return ((const __attribute__((address_space(4))) uint32_t*)(a.dp_gen))[blockIdx.x] + 1u;
}
__device__ __forceinline__ void dp_end_nosync(const MLP3Args& a, uint32_t gen, int fail) {
  if (threadIdx.x == 0) a.dp_gen[blockIdx.x] = gen;
  if (fail) __hip_atomic_store(a.dp_err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Owner of a task of the one-launch step: W1 tile kt -> task kt; small-parameter
// task t -> kTiles + t; round robin over the ranks (mirrored by
// parallel/mlp_engine.py dp_owner_mask for optimizer-state consolidation).
__device__ __forceinline__ int dp_task_owner(const MLP3Args& a, int task) { return task % a.dp_world; }

// ADAM mode: flat Adam over every non-W1 parameter (after the allreduce).
template <int L1, int L2>
__device__ __forceinline__ void small_adam_flat(const MLP3Args& a, const AdamScal& o, int blk, int nblk) {
  using O = Off<L1, L2>;
  __bf16* SHW = reinterpret_cast<__bf16*>(a.shadow);
  for (int64_t i = O::B1 + (int64_t)blk * blockDim.x + threadIdx.x; i < O::NP; i += (int64_t)nblk * blockDim.x) {
    float m = a.exp_avg[i], v = a.exp_avg_sq[i];
    const float p = adam1(a.params[i], a.grads[i] * a.grad_scale, m, v, o);
    a.params[i] = p;
    a.exp_avg[i] = m;
    a.exp_avg_sq[i] = v;
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
}

// Multi-block head (B > 32): its per-block (sum NLL, #correct, #rows), summed in
// block order into the stats ring.  Run by one lane of the tail's LAST block at
// the END of its work: placed at the tail's start, this branch cost the default
// step ~0.7 us (it delayed the issue of every block's initial loads).
__device__ __forceinline__ void tail_head_stats(const MLP3Args& a, const int64_t* cn) {
  float l = 0.f, k = 0.f, n = 0.f;
  for (int cb = 0; cb < (a.B + kHeadRows - 1) / kHeadRows; ++cb) {
    l += a.head_part[cb * 4 + 0];
    k += a.head_part[cb * 4 + 1];
    n += a.head_part[cb * 4 + 2];
  }
  const int64_t t = cn[0];
  float* st = a.stats + (int)((t - 1) % (a.stats_ring > 0 ? a.stats_ring : 1)) * 4;
  st[0] = l / (float)a.B;
  st[1] = k;
  st[2] = n;
  st[3] = (float)t;
}

template <int L1, int L2>
__global__ __launch_bounds__(64 * (L1 / 16)) void mlp3_tail_kernel(MLP3Args a, int mode) {
  constexpr int TN1 = L1 / 16;
  constexpr int NT = 64 * TN1;
  __shared__ __attribute__((aligned(16))) __bf16 sX[kBMax * kXSS];
  __shared__ __attribute__((aligned(16))) __bf16 sXn[kBMax * kXSS];
  __shared__ __attribute__((aligned(16))) __bf16 sW[L1 * kXSS];
  __shared__ AdamScal sh_o;
  const int tid = threadIdx.x, lane = tid & 63, ct = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const bool dp = mode == kFusedDP;
  const bool do_grad = mode == kFused || mode == kGrad || dp;
  const bool do_adam = mode == kFused || mode == kAdam || dp;
  const bool do_fwd = mode != kGrad;
  if (a.stamps && blockIdx.x == 0 && tid == 0) a.stamps[8] = __builtin_amdgcn_s_memrealtime();
  // every block reads the head's NEXT copy (never written in this launch);
  // block 0 publishes it as the current state for the next head
  const int64_t* cn = a.counters + kCnt;
  if (blockIdx.x == 0 && tid < kCnt) a.counters[tid] = cn[tid];
  // Adam's step scalars need the step counter (a load) and two double-precision
  // pows: issued here, computed by lane 0 only AFTER its block's own loads are in
  // flight -- computed first, they delayed wave 0's loads (and the block) by a
  // full round trip plus the pows.
  const int64_t t_step = cn[0];  // already advanced by the head kernel
  const float lr_now = a.lr_ptr ? a.lr_ptr[0] : a.lr;
  auto scalars = [&]() {
    if (tid == 0 && do_adam)
      adam_scalars(sh_o, t_step, lr_now, a.beta1, a.beta2, a.eps, a.weight_decay, a.adamw);
  };
  if ((int)blockIdx.x >= kTiles) {  // small parameters (block-uniform branch)
    const int sblk = (int)blockIdx.x - kTiles;
    if (mode == kFused || mode == kFusedDP || mode == kAdam) {
      // the H1pre slot the head consumed (cn[3] ^ 1) is zero for the step after
      // this one to accumulate into (the one-launch step relies on it)
      const int Bp = (a.B + 31) / 32 * 32;
      constexpr int G = H1Copies<L1>::G;
      uint4* z = reinterpret_cast<uint4*>(a.h1pre + (cn[3] ^ 1) * G * (int64_t)Bp * L1);
      const int nz = G * Bp * L1 / 4, nsb = (int)gridDim.x - kTiles;
      for (int i = sblk * NT + tid; i < nz; i += nsb * NT) z[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (mode == kAdam) {
      scalars();
      __syncthreads();
      small_adam_flat<L1, L2>(a, sh_o, sblk, (int)gridDim.x - kTiles);
      stamp_max(a, 11);
      return;
    }
    SmallRes r;
    small_compute<L1, L2>(a, mode != kGrad, sblk * TN1 + ct, r);
    scalars();
    __syncthreads();
    if (mode == kFusedDP) {
      __shared__ uint32_t sh_dgen;
      __shared__ int sh_dfail;
      const int dslot = dp_begin(a, &sh_dgen);
      const float scale = a.grad_scale;
      if (a.dp_lite == 2) {
        const uint32_t gen = sh_dgen;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r.valid[i]) dp_push_gran(a, dslot, r.gi[i], r.v[i], gen);
        int fail = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r.valid[i]) r.v[i] = dp_sum_gran(a, dslot, r.gi[i], gen, &fail) * scale;
        dp_gran_end(a, gen, fail, &sh_dfail);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r.valid[i]) dp_push1(a, dslot, r.gi[i], r.v[i]);
        dp_signal_and_wait(a, sh_dgen, dslot, &sh_dfail);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r.valid[i]) r.v[i] = dp_sum1(a, dslot, r.gi[i]) * scale;
      }
    }
    small_finalize<L1, L2>(a, mode != kGrad, r, sh_o);
    if (blockIdx.x == gridDim.x - 1 && tid == 0 && a.stats && a.B > kHeadRows) tail_head_stats(a, cn);
    stamp_max(a, 11);
    return;
  }
  const int kt = blockIdx.x;
  const int B = a.B;
  const int Bp = (B + 31) / 32 * 32;
  const int m = ct * 16 + r16, pix = kt * 16 + 4 * g;
  const int64_t gidx = (int64_t)m * kD + pix;

  // ---- loads that need no device state: Adam state, allreduced grads, current W1 ----
  F4 p4{}, m4{}, v4{}, g4{};
  if (do_adam) {
    p4 = *reinterpret_cast<const F4*>(a.params + gidx);
    m4 = *reinterpret_cast<const F4*>(a.exp_avg + gidx);
    v4 = *reinterpret_cast<const F4*>(a.exp_avg_sq + gidx);
  }
  if (mode == kAdam) g4 = *reinterpret_cast<const F4*>(a.grads + gidx);
  bf16x4 w4;
  if (mode == kPrime) w4 = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(a.shadow) + gidx);

  const int64_t slot = cn[3];
  const int64_t tile_elems = (int64_t)Bp * 16;
  __bf16* XR = reinterpret_cast<__bf16*>(a.xring);
  __bf16* xr_next = XR + (slot * kTiles + kt) * tile_elems;

  // ---- X slices: this step's (parked by the previous tail) and the next step's ----
  if (mode != kPrime) {
    // Both ring slots are loaded unconditionally and selected afterwards, so the
    // loads do not wait for the counters read (one memory round trip, not two).
    // cur = X[t] (parked by the previous step), next = X[t+1] (the head launch's
    // gather blocks); slot = cn[3] is where next lives.
    const __bf16* t0 = XR + (int64_t)kt * tile_elems;
    const __bf16* t1 = XR + (int64_t)(kTiles + kt) * tile_elems;
    for (int b = tid; b < Bp; b += NT) {
      const bf16x8 a0 = ld8(t0 + b * 16), a1 = ld8(t0 + b * 16 + 8);
      const bf16x8 c0 = ld8(t1 + b * 16), c1 = ld8(t1 + b * 16 + 8);
      const bool next_is_0 = slot == 0;
      if (do_grad) {
        *reinterpret_cast<bf16x8*>(sX + b * kXSS) = next_is_0 ? c0 : a0;
        *reinterpret_cast<bf16x8*>(sX + b * kXSS + 8) = next_is_0 ? c1 : a1;
      }
      if (do_fwd) {
        *reinterpret_cast<bf16x8*>(sXn + b * kXSS) = next_is_0 ? a0 : c0;
        *reinterpret_cast<bf16x8*>(sXn + b * kXSS + 8) = next_is_0 ? a1 : c1;
      }
    }
  } else {  // PRIME: no head ran, gather the pending batch here
    const int64_t* idx = a.order + cn[4] * a.order_stride + cn[1] * B;
    if (kt == 0)
      for (int b = tid; b < Bp; b += NT) a.yring[slot * Bp + b] = b < B ? (int)a.labels[idx[b]] : -1;
    for (int b = tid; b < Bp; b += NT) {
      bf16x8 lo = zero8(), hi = zero8();
      if (b < B) u8x16_to_bf16(*reinterpret_cast<const uint4*>(a.x_u8 + idx[b] * kD + kt * 16), lo, hi);
      *reinterpret_cast<bf16x8*>(sXn + b * kXSS) = lo;
      *reinterpret_cast<bf16x8*>(sXn + b * kXSS + 8) = hi;
      *reinterpret_cast<bf16x8*>(xr_next + b * 16) = lo;
      *reinterpret_cast<bf16x8*>(xr_next + b * 16 + 8) = hi;
    }
  }
  scalars();
  __syncthreads();
  if (a.stamps && kt == 0 && tid == 0) a.stamps[9] = __builtin_amdgcn_s_memrealtime();

  // ---- dW1 tile: D[pixel pix+i][neuron m] = sum_b X[b][pix+i] dH1[b][m] ----
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (do_grad) {
    const __bf16* dh = reinterpret_cast<const __bf16*>(a.dh1t) + (int64_t)m * Bp;
    const int q = r16 >> 2, pp = r16 & 3;
    for (int ks = 0; ks < Bp / 32; ++ks) {
      const int b0 = ks * 32 + 8 * g;
      const bf16x4 lo = tr_read(sX + (b0 + q) * kXSS + 4 * pp);
      const bf16x4 hi = tr_read(sX + (b0 + 4 + q) * kXSS + 4 * pp);
      const bf16x8 afrag = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      acc = mfma16(afrag, ld8(dh + b0), acc);
    }
  }
  if (mode == kGrad) {
    F4 gg{{acc[0], acc[1], acc[2], acc[3]}};
    *reinterpret_cast<F4*>(a.grads + gidx) = gg;
    return;
  }
  if (dp) {  // allreduce of this tile inside the epilogue (xGMI push / flag / fixed-order sum)
    __shared__ uint32_t sh_dgen;
    __shared__ int sh_dfail;
    const int dslot = dp_begin(a, &sh_dgen);
    if (a.dp_lite == 2) {
      const uint32_t gen = sh_dgen;
#pragma unroll
      for (int i = 0; i < 4; ++i) dp_push_gran(a, dslot, gidx + i, acc[i], gen);
      int fail = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = dp_sum_gran(a, dslot, gidx + i, gen, &fail) * a.grad_scale;
      dp_gran_end(a, gen, fail, &sh_dfail);
    } else {
      typedef float v4f __attribute__((ext_vector_type(4)));
      const v4f mine = {acc[0], acc[1], acc[2], acc[3]};
      for (int r = 0; r < a.dp_world; ++r)
        __builtin_nontemporal_store(mine, reinterpret_cast<v4f*>(dp_data(a.dp_regions[r], dslot, a.dp_rank,
                                                                         a.dp_stride) + gidx));
      dp_signal_and_wait(a, sh_dgen, dslot, &sh_dfail);
      v4f s = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < a.dp_world; ++r)
        s += __builtin_nontemporal_load(
            reinterpret_cast<const v4f*>(dp_data(a.dp_regions[a.dp_rank], dslot, r, a.dp_stride) + gidx));
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = s[i] * a.grad_scale;
    }
  }
  if (do_adam) {
    const AdamScal o = sh_o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float gr = (mode == kAdam) ? g4.v[i] * a.grad_scale : acc[i];
      p4.v[i] = adam1(p4.v[i], gr, m4.v[i], v4.v[i], o);
      w4[i] = (__bf16)p4.v[i];
    }
    *reinterpret_cast<F4*>(a.params + gidx) = p4;
    *reinterpret_cast<F4*>(a.exp_avg + gidx) = m4;
    *reinterpret_cast<F4*>(a.exp_avg_sq + gidx) = v4;
    *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.shadow) + gidx) = w4;
  }
  // ---- next step's layer-1 partial: H1pre[b][m] += sum_{16 px} X'[b][px] W1[m][px] ----
  *reinterpret_cast<bf16x4*>(sW + m * kXSS + 4 * g) = w4;
  __syncthreads();
  if (do_fwd) {
    constexpr int G = H1Copies<L1>::G;
    unsigned* h1 =
        reinterpret_cast<unsigned*>(a.h1pre + (slot * G + kt % G) * (int64_t)Bp * L1);
    const bf16x8 bfrag = (g < 2) ? ld8(sW + (ct * 16 + r16) * kXSS + 8 * g) : zero8();
    for (int mt = 0; mt < Bp / 16; ++mt) {
      const bf16x8 afrag = (g < 2) ? ld8(sXn + (mt * 16 + r16) * kXSS + 8 * g) : zero8();
      const f32x4 d = mfma16(afrag, bfrag, f32x4{0.f, 0.f, 0.f, 0.f});
      unsigned* dst = h1 + (int64_t)((mt * TN1 + ct) * 4) * 64 + lane;
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(dst + i * 64, f32_to_fixed(d[i]));
    }
  }
  if (a.stamps && kt == 0 && tid == 0) a.stamps[10] = __builtin_amdgcn_s_memrealtime();
  stamp_max(a, 11);
}

// ---------------------------------------------------------------------------
// One-launch step (kind Step1; world size 1, B <= 32).  The head's serial chain
// (H1 -> layers 2/3 -> loss -> dH2 -> dH1, ~4 us, latency-bound on one CU) is
// REPLICATED: every block of the launch runs it on its own CU from the same
// inputs (bitwise-identical results: fixed reduction orders), keeps H1^T / H2^T /
// dZ^T / dH2^T / dH1^T in its LDS and goes straight on to its own tail role --
//   block 0          loss stats + the state advance,
//   blocks [1, 50)   one W1 column tile each (dW1, Adam, X[t+1] gather, H1pre[t+1] partial),
//   the rest         the small parameters (one dW2 / dW3 tile or 64 biases per wave).
// No activation crosses a CU, so the two-launch step's kernel boundary and its
// tail's load phase (the tile's Adam state, X tiles and the next batch's gather
// are issued before the head pass) leave the critical path.
//
// Ordering (the only cross-block traffic): every block reads the state
// (counters, H1pre, labels, weights) and then adds one acknowledgement to
// hand[kHandAck] (monotonic).  Whoever overwrites something another block reads
// -- the small blocks (weights / biases), block 0 (counters, the consumed H1pre
// slot) -- first waits for launch `seq`'s (seq + 1) * gridDim.x acks.  The W1
// tiles write nothing another block reads (the head reads H1pre, not W1) and
// never wait.  Invariant kept by every step kind: the H1pre slot the tiles add
// into (slot ^ 1) is zero when a step starts (block 0 / the two-launch tail
// zero the consumed slot; prime zeroes both).
// ---------------------------------------------------------------------------
template <int L1, int L2>
struct One {
  using C = Cfg3<32, L1, L2>;
  static constexpr int NTASK = SmallTasks<L1, L2>::NTASK;
  static constexpr int NSMALL = (NTASK + kWaves - 1) / kWaves;
  // after the head's region: H2^T, dH2^T, dH1^T images, then the tile's X / W1 slices + Adam scalars
  static constexpr size_t oImg = C::total;
  static constexpr size_t oTile = oImg + (size_t)(2 * L2 + L1) * C::TS * 2;
  static constexpr size_t oRaw = oTile + (size_t)(2 * 32 + L1) * kXSS * 2 + 64;  // PreWave DMA area
  static constexpr size_t lds = oRaw + kPreRawBytes;
};
static_assert(One<128, 256>::lds <= 160 * 1024, "one-launch LDS budget");

// lane 0 waits for launch `seq`'s acknowledgements, then the whole block proceeds
__device__ __forceinline__ void one_wait_acks(const MLP3Args& a, int64_t seq, int* sh_fail) {
  if (threadIdx.x == 0) {
    const long long target = (long long)(seq + 1) * (long long)gridDim.x;
    const long long* ack = reinterpret_cast<const long long*>(a.hand + kHandAck);
    int64_t n = 0;
    *sh_fail = 0;
    while (__hip_atomic_load(ack, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++n > a.hand_spin) {
        *sh_fail = 1;
        __hip_atomic_store(a.hand + kHandErr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // data-parallel step: also the comm engine's host-mapped error word, which the
        // Trainer / bench check at every epoch end without a device sync
        if (a.dp_err) __hip_atomic_store(a.dp_err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  // Why relaxed atomics suffice for this hand-off: it orders READS
  // before WRITES (write-after-read), not data.  The acknowledging wave's loads have
  // RETURNED (s_waitcnt vmcnt(0) in head_body) before its ack is issued, so no later
  // store can change what they read; the waiter issues its stores only after the
  // poll observed every ack (in-order issue; the stores depend on the loop's exit).
  // What remains is the compiler: the "memory" clobbers (the waitcnt asm on the ack
  // side, this one on the waiter's) stop it from moving memory operations across
  // either point.  No cache maintenance is needed -- nothing the waiter stores is
  // read back by the acknowledged blocks in this launch.
  asm volatile("" ::: "memory");
  __syncthreads();
}

// DP (kind Step1DP, world size > 1): each tile's dW1 and each small wave's values
// are allreduced over xGMI (tagged granules, as the two-launch StepDP tail) between
// the block's gradient and its Adam -- the exchange sits inside the one launch.
// DPP: -1 world size 1 (Step1); else the exchange protocol of Step1DP (0 granule,
// 1 packed, 2 owner) as a template parameter -- each instance carries only its own
// protocol's code (a run-time switch over all three cost the head pass ~0.5 us and
// the tile epilogue ~1.4 us of register pressure, profiles/r3_dp/dp_phases.log).
// NW: the rank class of the packed / owner polls (world size <= NW; see dp_peer_issue).
template <int L1, int L2, int DPP, int NW = 8>
__global__ __launch_bounds__(kThreads) void mlp3_one_kernel(MLP3Args a) {
  constexpr bool DP = DPP >= 0;
  using C = typename One<L1, L2>::C;
  using S = SmallTasks<L1, L2>;
  constexpr int TN1 = L1 / 16, Bp = 32;
  __shared__ __attribute__((aligned(16))) char smem[One<L1, L2>::lds];
  __shared__ int sh_fail;
  __bf16* sH2T = (__bf16*)(smem + One<L1, L2>::oImg);
  __bf16* sDH2T = sH2T + L2 * C::TS;
  __bf16* sDH1T = sDH2T + L2 * C::TS;
  __bf16* sX = (__bf16*)(smem + One<L1, L2>::oTile);
  __bf16* sXn = sX + Bp * kXSS;
  __bf16* sW = sXn + Bp * kXSS;
  AdamScal* sh_o = reinterpret_cast<AdamScal*>(sW + L1 * kXSS);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int blk = blockIdx.x;
  const bool tile = blk >= 1 && blk <= kTiles, small = blk > kTiles;
  const int kt = blk - 1;
  if (a.stamps && blk == 1 && tid == 0) a.stamps[8] = __builtin_amdgcn_s_memrealtime();
  stamp_max(a, 13);  // probe builds: the latest block start (dispatch skew)

  // the state of this step: nobody overwrites it before every block's ack
  const int64_t c0 = ld_state(a.counters, 0), cursor = ld_state(a.counters, 1);
  const int64_t slot = ld_state(a.counters, 3), ob = ld_state(a.counters, 4);
  const int64_t seq = ld_state(a.counters, kSeq);
  const uint32_t dgen = DP ? dp_gen_now(a) : 0u;
  const int B = a.B;

  // ---- tail-role loads that need nothing from this step, issued before the head
  // pass and consumed after it (unconditional, clamped addresses: no wait here) ----
  const int m = w * 16 + r16, pix = kt * 16 + 4 * g;
  const bool mw = tile && w < TN1;  // tile waves owning a 16-neuron column
  const int64_t gidx = mw ? (int64_t)m * kD + pix : 0;
  F4 p4, m4, v4;  // loaded by the head's hook (below)
  SmallRes r;
  r.kind = -1;
  const int task = (blk - 1 - kTiles) * kWaves + w;
  if (small) small_compute<L1, L2, true>(a, true, task, r);  // setup + Adam state prefetch
  // the device learning rate through the SCALAR path: as a vector load, the f64 bias
  // corrections below (thread 0) waited vmcnt(0) for it -- i.e. for every prologue
  // prefetch -- before wave 0 issued a single head-pass load (profiles/r4_dp)
  const float lr_now = a.lr_ptr ? ((const __attribute__((address_space(4))) float*)(a.lr_ptr))[0] : a.lr;
  // wave 0 of a tile: row (lane & 31) of X[t] (parked by the previous step) and the
  // sample index of row (lane & 31) of the NEXT batch (its pixels load after the ack)
  __bf16* XR = reinterpret_cast<__bf16*>(a.xring);
  constexpr int64_t tile_elems = (int64_t)Bp * 16;
  const int xb = lane & 31;
  bf16x8 xc0, xc1;
  RepPre pre;
  pre.active = tile && w == PreWave<L1>::wave;
  pre.raw = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(smem + One<L1, L2>::oRaw);
  pre.kt = tile ? kt : 0;
  pre.xn = make_uint4(0u, 0u, 0u, 0u);
  pre.yn = -1;
  int64_t nc = cursor + 1, nob = ob;
  if (nc >= a.n_batches) { nc = 0; nob ^= 1; }
  // the private prologue loads, exactly kRepHookLoads per wave on every block (clamped
  // addresses where the wave does not need them): the next sample index first (its
  // value is needed right after the ack, so it is waited for before the others)
  const int kt_c = tile ? kt : 0;
  auto hook = [&]() {
    pre.si = a.order[nob * a.order_stride + nc * B + (xb < B ? xb : 0)];
    const __bf16* cur = XR + (slot * kTiles + kt_c) * tile_elems + xb * 16;
    xc0 = ld8(cur);
    xc1 = ld8(cur + 8);
    p4 = *reinterpret_cast<const F4*>(a.params + gidx);
    m4 = *reinterpret_cast<const F4*>(a.exp_avg + gidx);
    v4 = *reinterpret_cast<const F4*>(a.exp_avg_sq + gidx);
  };
  if (tid == 0 && blk > 0)
    adam_scalars(*sh_o, a.advance_step ? c0 + 1 : c0, lr_now, a.beta1, a.beta2, a.eps, a.weight_decay, a.adamw);

  // ---- the serial chain, on this CU (tile wave 0 also issues the next batch's loads) ----
  head_body<32, L1, L2, false, true>(a, smem, &pre, hook);

  // (the block's acknowledgement went out inside head_body, once its loads had landed)
  if (a.stamps && blk == 1 && tid == 0) a.stamps[9] = __builtin_amdgcn_s_memrealtime();
  stamp_max(a, 12);  // probe builds: the latest head-pass end over all blocks

  if (tile) {
    // the next batch's pixels (+ label, tile 0) were issued inside the head pass
    if (w == 0 && lane < 32) {
      *reinterpret_cast<bf16x8*>(sX + xb * kXSS) = xc0;
      *reinterpret_cast<bf16x8*>(sX + xb * kXSS + 8) = xc1;
    }
    __syncthreads();
    if (a.stamps && blk == 1 && tid == 0) a.stamps[7] = __builtin_amdgcn_s_memrealtime();
    bf16x4 w4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (mw) {
      // dW1 tile: D[pixel pix+i][neuron m] = sum_b X[b][pix+i] dH1[b][m]
      const int q = r16 >> 2, pp = r16 & 3;
      const bf16x4 lo = tr_read(sX + (8 * g + q) * kXSS + 4 * pp);
      const bf16x4 hi = tr_read(sX + (8 * g + 4 + q) * kXSS + 4 * pp);
      const bf16x8 afrag = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      acc = mfma16(afrag, ld8(sDH1T + m * C::TS + 8 * g), acc);
    }
    bool adam_done = false, store_mv = true;
    if constexpr (DP) {  // the tile's allreduce, inside the epilogue (protocol: a.dp_proto)
      const uint32_t gen = dgen;
      const int dslot = (int)(gen & 1u);
      int fail = 0;
      if (mw) {
        if constexpr (DPP == 0) {  // round 2: arena-indexed {gen, fp32} granules
#pragma unroll
          for (int i = 0; i < 4; ++i) dp_push_gran(a, dslot, gidx + i, acc[i], gen);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = dp_sum_gran(a, dslot, gidx + i, gen, &fail) * a.grad_scale;
        } else {
          float v[4] = {acc[0], acc[1], acc[2], acc[3]};
          const int unit = blk * kWaves + w;
          if constexpr (DPP == 1) {
            dp_packed_exchange<NW>(a, unit, gen, v, a.grad_scale, &fail);
          } else {
            const AdamScal o = *sh_o;
            store_mv = dp_owner_step<NW>(a, unit, dp_task_owner(a, kt), gen, v, a.grad_scale, &fail,
                                     [&](float (&x)[4]) {
#pragma unroll
                                       for (int i = 0; i < 4; ++i) x[i] = adam1(p4.v[i], x[i], m4.v[i], v4.v[i], o);
                                     });
            store_mv = store_mv || a.dp_loop;  // loopback: this process holds every rank's state
            adam_done = true;
#pragma unroll
            for (int i = 0; i < 4; ++i) p4.v[i] = v[i];
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = v[i];
        }
      }
      dp_end_nosync(a, gen, fail);
    }
    if (mw) {
      if (!adam_done) {
        const AdamScal o = *sh_o;
#pragma unroll
        for (int i = 0; i < 4; ++i) p4.v[i] = adam1(p4.v[i], acc[i], m4.v[i], v4.v[i], o);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) w4[i] = (__bf16)p4.v[i];
      *reinterpret_cast<F4*>(a.params + gidx) = p4;
      if (store_mv) {  // owner protocol: only the task's owner holds its current Adam state
        *reinterpret_cast<F4*>(a.exp_avg + gidx) = m4;
        *reinterpret_cast<F4*>(a.exp_avg_sq + gidx) = v4;
      }
      *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.shadow) + gidx) = w4;
      *reinterpret_cast<bf16x4*>(sW + m * kXSS + 4 * g) = w4;
    }
    if (w == PreWave<L1>::wave && lane >= 32) {
      // X[t+1] row xb -> sXn, parked in xring[slot ^ 1] for the next step (+ its labels, tile 0)
      uint4 xn = pre.xn;
      int yn = (int)pre.yn;
      if constexpr (PreWave<L1>::hidden) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA (this wave's only vector-memory ops in flight)
        const char* raw = smem + One<L1, L2>::oRaw;
        xn = *reinterpret_cast<const uint4*>(raw + 16 * lane);
        yn = (int)*reinterpret_cast<const int64_t*>(raw + 1024 + 8 * xb);
      }
      bf16x8 lo = zero8(), hi = zero8();
      if (xb < B) u8x16_to_bf16(xn, lo, hi);
      *reinterpret_cast<bf16x8*>(sXn + xb * kXSS) = lo;
      *reinterpret_cast<bf16x8*>(sXn + xb * kXSS + 8) = hi;
      __bf16* nx = XR + ((slot ^ 1) * kTiles + kt) * tile_elems + xb * 16;
      *reinterpret_cast<bf16x8*>(nx) = lo;
      *reinterpret_cast<bf16x8*>(nx + 8) = hi;
      if (kt == 0) a.yring[(slot ^ 1) * Bp + xb] = xb < B ? yn : -1;
    }
    __syncthreads();
    if (a.stamps && blk == 1 && tid == 0) a.stamps[14] = __builtin_amdgcn_s_memrealtime();
    stamp_max(a, 15);  // probe builds: the latest tile block past its staging barrier
    if (mw) {
      // next step's layer-1 partial: H1pre[b][m] += sum_{16 px} X'[b][px] W1[m][px]
      constexpr int G = H1Copies<L1>::G;
      unsigned* h1 = reinterpret_cast<unsigned*>(a.h1pre + ((slot ^ 1) * G + kt % G) * (int64_t)Bp * L1);
      const bf16x8 bfrag = (g < 2) ? ld8(sW + (w * 16 + r16) * kXSS + 8 * g) : zero8();
#pragma unroll
      for (int mt = 0; mt < Bp / 16; ++mt) {
        const bf16x8 afrag = (g < 2) ? ld8(sXn + (mt * 16 + r16) * kXSS + 8 * g) : zero8();
        const f32x4 d = mfma16(afrag, bfrag, f32x4{0.f, 0.f, 0.f, 0.f});
        unsigned* dst = h1 + (int64_t)((mt * TN1 + w) * 4) * 64 + lane;
#pragma unroll
        for (int i = 0; i < 4; ++i) atomicAdd(dst + i * 64, f32_to_fixed(d[i]));
      }
    }
    if (a.stamps && blk == 1 && tid == 0) a.stamps[10] = __builtin_amdgcn_s_memrealtime();
    stamp_max(a, 5);  // probe builds: the latest W1-tile block end
  } else if (small) {
    const RepLds L{(const __bf16*)(smem + C::oH1T), sH2T, sDH2T, (const __bf16*)(smem + C::odZT), sDH1T, C::TS};
    small_compute<L1, L2, true>(a, true, task, r, &L);
    bool adam_done = false, store_mv = true;
    if constexpr (DP) {
      const uint32_t gen = dgen;
      const int dslot = (int)(gen & 1u);
      int fail = 0;
      if constexpr (DPP == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r.valid[i]) dp_push_gran(a, dslot, r.gi[i], r.v[i], gen);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r.valid[i]) r.v[i] = dp_sum_gran(a, dslot, r.gi[i], gen, &fail) * a.grad_scale;
      } else if (task < S::NTASK) {  // whole waves (idle lanes exchange zeros)
        float v[4] = {r.v[0], r.v[1], r.v[2], r.v[3]};
        const int unit = blk * kWaves + w;
        if constexpr (DPP == 1) {
          dp_packed_exchange<NW>(a, unit, gen, v, a.grad_scale, &fail);
        } else {
          // Adam in registers before the acknowledgement wait below: the owner
          // publishes the weights as early as possible, stores after the wait
          const AdamScal o = *sh_o;
          store_mv = dp_owner_step<NW>(a, unit, dp_task_owner(a, kTiles + task), gen, v, a.grad_scale, &fail,
                                   [&](float (&x)[4]) {
#pragma unroll
                                     for (int i = 0; i < 4; ++i) x[i] = adam1(r.pv[i], x[i], r.mv[i], r.vv[i], o);
                                   });
          store_mv = store_mv || a.dp_loop;
          adam_done = true;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) r.v[i] = v[i];
      }
      dp_end_nosync(a, gen, fail);
    }
    one_wait_acks(a, seq, &sh_fail);  // every block has read the weights / biases this overwrites
    if (adam_done) small_store<L1, L2>(a, r, store_mv);  // r.v: the new weights
    else small_finalize<L1, L2>(a, true, r, *sh_o);
    stamp_max(a, 6);  // probe builds: the latest small-parameter block end
  } else {
    // block 0: stats, the consumed H1pre slot zeroed (the invariant), then the advanced state
    one_wait_acks(a, seq, &sh_fail);
    uint4* z = reinterpret_cast<uint4*>(a.h1pre + slot * H1Copies<L1>::G * (int64_t)Bp * L1);
    for (int i = tid; i < H1Copies<L1>::G * Bp * L1 / 4; i += kThreads) z[i] = make_uint4(0u, 0u, 0u, 0u);
    if (tid == 0) {
      const float* misc = (const float*)(smem + C::oMisc);
      const int64_t t = c0 + 1;
      int64_t nc = cursor + 1, nob = ob;
      if (nc >= a.n_batches) { nc = 0; nob ^= 1; }
      const int64_t st[kCnt] = {a.advance_step ? t : t - 1, nc, cursor, slot ^ 1, nob};
      for (int k = 0; k < kCnt; ++k) a.counters[k] = a.counters[kCnt + k] = st[k];
      a.counters[kSeq] = seq + 1;
      if (a.stats) {
        float* sr = a.stats + (int)((t - 1) % (a.stats_ring > 0 ? a.stats_ring : 1)) * 4;
        sr[0] = misc[0] * (1.f / (float)B);
        sr[1] = misc[1];
        sr[2] = misc[2];
        sr[3] = (float)t;
      }
      if (a.stamps) a.stamps[4] = __builtin_amdgcn_s_memrealtime();
    }
  }
  stamp_max(a, 11);
}

template <int L1, int L2>
int dispatch3(const MLP3Args& a, int kind, hipStream_t stream) {
  constexpr int kOneGrid = 1 + kTiles + One<L1, L2>::NSMALL;
  if (kind == kMLP3Step1) {
    if (a.B > 32 || !a.hand || kOneGrid > 256) return -5;
    hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, -1>), dim3(kOneGrid), dim3(kThreads), 0, stream, a);
    return 0;
  }
  if (kind == kMLP3Step1DP) {
    // granule exchange only (the flag protocols stay on the two-launch StepDP)
    if (a.B > 32 || !a.hand || kOneGrid > kDpMaxBlocks || a.dp_world < 1 || a.dp_world > kXgmiMaxRanks ||
        !a.dp_gen || !a.dp_err || a.dp_proto < 0 || a.dp_proto > 2)
      return -6;
    // round-2 granules need 2 floats per parameter, the wave-positioned areas their fixed size
    if (a.dp_proto == 0 ? (a.dp_lite != 2 || a.dp_stride < 2 * Off<L1, L2>::NP) : a.dp_stride < comm::kDpUnitAreaFloats)
      return -7;
    const dim3 g(kOneGrid), b(kThreads);
    const int nw = a.dp_world <= 2 ? 2 : (a.dp_world <= 4 ? 4 : 8);
    if (a.dp_proto == 0) hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, 0>), g, b, 0, stream, a);
    else if (a.dp_proto == 1 && nw == 2) hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, 1, 2>), g, b, 0, stream, a);
    else if (a.dp_proto == 1 && nw == 4) hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, 1, 4>), g, b, 0, stream, a);
    else if (a.dp_proto == 1) hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, 1, 8>), g, b, 0, stream, a);
    else if (nw == 2) hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, 2, 2>), g, b, 0, stream, a);
    else if (nw == 4) hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, 2, 4>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((mlp3_one_kernel<L1, L2, 2, 8>), g, b, 0, stream, a);
    return 0;
  }
  constexpr int NT = 64 * (L1 / 16);
  if (kind == kMLP3StepDP && (a.dp_world < 1 || a.dp_world > kXgmiMaxRanks || !a.dp_gen || !a.dp_err ||
                              a.dp_stride < Off<L1, L2>::NP || kTiles + SmallTasks<L1, L2>::NBLK > kDpMaxBlocks))
    return -3;
  if (kind == kMLP3Step || kind == kMLP3Head || kind == kMLP3StepDP) {
    // one workgroup per 32 batch rows (concurrent), then the 49 gather blocks
    const int nchunks = (a.B + kHeadRows - 1) / kHeadRows;
    if (nchunks > 1 && !a.head_part) return -4;
    if (nchunks > 1)
      hipLaunchKernelGGL((mlp3_head_kernel<kHeadRows, L1, L2, true>), dim3(nchunks + kTiles), dim3(kThreads), 0, stream, a);
    else
      hipLaunchKernelGGL((mlp3_head_kernel<kHeadRows, L1, L2, false>), dim3(1 + kTiles), dim3(kThreads), 0, stream, a);
  }
  int mode = -1, grid = kTiles;
  if (kind == kMLP3Step) { mode = kFused; grid += SmallTasks<L1, L2>::NBLK; }
  else if (kind == kMLP3StepDP) { mode = kFusedDP; grid += SmallTasks<L1, L2>::NBLK; }
  else if (kind == kMLP3TailGrad) { mode = kGrad; grid += SmallTasks<L1, L2>::NBLK; }
  else if (kind == kMLP3Prime) mode = kPrime;
  else if (kind == kMLP3TailAdam) {
    mode = kAdam;
    const int64_t nsmall = Off<L1, L2>::NP - Off<L1, L2>::B1;
    int extra = (int)((nsmall + NT - 1) / NT);
    grid += extra < 64 ? extra : 64;
  }
  if (mode >= 0) hipLaunchKernelGGL((mlp3_tail_kernel<L1, L2>), dim3(grid), dim3(NT), 0, stream, a, mode);
  return 0;
}

static_assert(fits3<kHeadRows, 128, 256>(), "v3 head LDS budget");

__global__ void dp_pack_roundtrip_kernel(const float* x, float* y, int64_t n, uint32_t tag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 < n + 1) {
    const float v0 = x[2 * i], v1 = 2 * i + 1 < n ? x[2 * i + 1] : 0.f;
    const u64 w = pk2(v0, v1, tag);
    y[2 * i] = ((uint32_t)w & 3u) == tag ? pk_lo(w) : __builtin_nanf("");
    if (2 * i + 1 < n) y[2 * i + 1] = pk_hi(w);
  }
}

}  // namespace

int dp_pack_roundtrip(const float* x, float* y, int64_t n, int tag, hipStream_t stream) {
  if (n <= 0 || tag < 0 || tag > 3) return -1;
  const int64_t pairs = (n + 1) / 2;
  hipLaunchKernelGGL(dp_pack_roundtrip_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, stream, x, y, n,
                     (uint32_t)tag);
  return 0;
}

int mlp3_act_rows(int L1, int L2) { return L1 + 2 * L2 + 16; }
int mlp3_h1_copies(int L1) { return L1 <= 64 ? H1Copies<64>::G : H1Copies<128>::G; }
int64_t mlp3_hand_words(int, int) { return kHandWords; }

int launch_mlp3(const MLP3Args& a, int kind, hipStream_t stream) {
  if (a.B > kBMax || a.B < 1) return -2;
#define RLA_CASE(a1, a2) if (a.L1 == a1 && a.L2 == a2) return dispatch3<a1, a2>(a, kind, stream);
  RLA_CASE(32, 32) RLA_CASE(32, 64) RLA_CASE(32, 128) RLA_CASE(32, 256)
  RLA_CASE(64, 64) RLA_CASE(64, 128) RLA_CASE(64, 256)
  RLA_CASE(128, 64) RLA_CASE(128, 128) RLA_CASE(128, 256)
#undef RLA_CASE
  return -1;
}

}  // namespace rla
