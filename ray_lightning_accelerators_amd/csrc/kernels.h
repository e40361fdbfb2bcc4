// Host-callable launch API of the HIP kernels (plain pointers + hipStream_t).
// The torch bindings (bindings.cpp) are the only caller; keeping this header
// free of torch types lets the .hip files compile with hipcc alone.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rla {

struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  uint16_t* p_bf16;        // optional bf16 copy-out of the updated params
  int64_t n;
  float lr, beta1, beta2, eps, weight_decay, grad_scale;
  int adamw, maximize;
  const int64_t* step_ptr;  // device step counter (already incremented) or null
  int64_t host_step;        // used when step_ptr is null
  const float* lr_ptr;      // device learning rate (graph-replay friendly) or null
};

struct SGDArgs {
  float* p;
  const float* g;
  float* buf;
  uint16_t* p_bf16;
  int64_t n;
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, maximize;
  const int64_t* step_ptr;
  int64_t host_step;
  const float* lr_ptr;
};

void launch_adam(const AdamArgs& a, hipStream_t stream);
void launch_sgd(const SGDArgs& a, hipStream_t stream);
void launch_multi_copy(const int64_t* table, int64_t nchunks, float scale, int accumulate,
                       hipStream_t stream);
void launch_scale(float* x, int64_t n, float s, hipStream_t stream);
void launch_sumsq(const float* x, int64_t n, float* out, hipStream_t stream);

// ---------------------------------------------------------------------------
// Fused BatchNorm(+ReLU)(+residual add) over NHWC bf16 activations viewed as
// [M, C] rows (csrc/bn_act.hip).  C % 8 == 0 and C <= kBnMaxC.
// ---------------------------------------------------------------------------
constexpr int kBnThreads = 256;

// NHWC bf16 max pooling with a one-byte window argmax (csrc/pool.hip)
// bn_ss (or null): x is a BatchNorm's input, pooled as bf16(relu(x * ss[2] + ss[3])) (the stem's
// BatchNorm + ReLU folded into the pool); nbt_inc as launch_bn_apply's
int launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int OH, int OW,
                       int k, int s, int pad, hipStream_t stream, const float* bn_ss = nullptr,
                       int64_t* nbt_inc = nullptr);
int launch_maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int OH,
                       int OW, int k, int s, int pad, hipStream_t stream);
// global average pool backward over NHWC rows: dx[n][p][c] = dy[n][c] / HW
int launch_gap_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t stream);
// d [N, H, W, C] += g [N, OH, OW, C] at every s-th pixel (NHWC bf16, fp32 add)
int launch_strided_add(uint16_t* d, const uint16_t* g, int N, int H, int W, int C, int OH, int OW, int s,
                       hipStream_t stream);
// a max pool's backward seen from the layer before it (csrc/pool_gather.h)
struct PoolGrad {
  const uint16_t* g;   // gradient of the pooled output [N, OH, OW, C] bf16
  const uint8_t* arg;  // window argmax bytes [N, OH, OW, C]
  int H, W, OH, OW, k, s, pad;
};
constexpr int kBnMaxC = 2048;  // 8 channels per thread x 256 threads per row

struct BnPlan {
  int64_t rows_per_blk;  // rows each block of the partial kernels reduces
  int blocks;
  int group;   // > 1: blocks per group of the in-kernel second reduction level (fp64 rows)
  int groups;  // ceil(blocks / group): rows the finalize reads
};
BnPlan bn_plan(int64_t M, int C);
// second reduction level of the partial kernels (see bn_act.hip BnL2)
struct BnLevel2 {
  double* rows;  // [groups, 2, C] or nullptr (single level)
  int* tickets;  // [groups] zero-initialised, self-resetting
};

// per-block partial sums part[b][0][c], part[b][1][c]:
//   mode 0 (forward):  sum x, sum x^2   (nbt, if given, is incremented by block 0)
//   mode 1 (backward): sum dz, sum dz*x with dz = dy * (y > 0 if relu)
void launch_bn_partial(const uint16_t* x, const uint16_t* y, const uint16_t* dy, int64_t M, int C, int mode,
                       bool relu, const BnPlan& plan, float* part, int64_t* nbt, hipStream_t s,
                       const uint16_t* dy2 = nullptr,   // backward: gradient = dy + dy2
                       const float* ss = nullptr,       // backward ReLU mask from the fwd stats, not y
                       BnLevel2 l2 = BnLevel2{nullptr, nullptr},
                       uint16_t* dout = nullptr,        // backward: also write d = masked dy (+dy2), bf16
                       const PoolGrad* pool = nullptr);  // backward: dy gathered through a max pool (relu, ss)

// forward finalize of `nparts` partial rows: stats[0]=mean [1]=invstd [2]=scale [3]=shift ([4, C]);
// running stats update (momentum < 0: cumulative average over num_batches_tracked)
void launch_bn_finalize(const float* part, int nparts, int C, double count, const float* gamma,
                        const float* beta, float* running_mean, float* running_var, const int64_t* nbt,
                        float momentum, float eps, float* stats, hipStream_t s,
                        int nbt_pending = 0);  // 1: nbt's += 1 is still to come (bn_apply's nbt_inc)
// the same from the fp64 rows of the second reduction level
void launch_bn_finalize64(const double* part, int nparts, int C, double count, const float* gamma,
                          const float* beta, float* running_mean, float* running_var, const int64_t* nbt,
                          float momentum, float eps, float* stats, hipStream_t s);

// backward finalize: coef[0]=dgamma [1]=dbeta [2]=A [3]=B [4]=Cc ([5, C]); dx = A*dz + B*x + Cc
void launch_bn_bwd_finalize(const float* part, int nparts, int C, double count, const float* gamma,
                            const float* mean, const float* invstd, float* coef, hipStream_t s);
void launch_bn_bwd_finalize64(const double* part, int nparts, int C, double count, const float* gamma,
                              const float* mean, const float* invstd, float* coef, hipStream_t s);

// y = act(x*scale + shift (+ res))
void launch_bn_apply(const uint16_t* x, const uint16_t* res, const float* scale, const float* shift, int64_t M,
                     int C, bool relu, uint16_t* y, hipStream_t s,
                     int64_t* nbt_inc = nullptr);  // block 0 adds 1 (statistics came from a conv epilogue)

// dz = dy * (y > 0 if relu); dx = A*dz + B*x + Cc; dres = dz (if dres)
void launch_bn_bwd_apply(const uint16_t* x, const uint16_t* y, const uint16_t* dy, const float* coef, int64_t M,
                         int C, bool relu, uint16_t* dx, uint16_t* dres, hipStream_t s,
                         const uint16_t* dy2 = nullptr,  // gradient = dy + dy2
                         const float* ss = nullptr,      // ReLU mask from the fwd stats [4, C], not y
                         const PoolGrad* pool = nullptr);  // dy gathered through a max pool (relu, ss)

// 1x1 / stride-1 conv forward y[M][N] = x[M][K] . w[N][K]^T with the next BatchNorm's
// partial sums of bf16(y) in the epilogue: part [gx, 2, N] fp32, bn_finalize's layout
// (csrc/conv1x1.hip)
struct Conv1x1Plan {
  int tnw;            // 32-channel blocks per wave (1 or 2)
  int gy;             // channel columns of 64 tnw
  int gx;             // pixel ranges = partial rows (multiple of 8)
  int tiles_per_blk;  // 128-pixel tiles per range
};
bool conv1x1_stats_ok(int64_t M, int K, int N);
// pre_ss ([4, K] BatchNorm stats, K <= 512): x is a deferred BatchNorm + ReLU's input,
// each x fragment becomes bf16(relu(x * scale + shift)) in the kernel (nbt_inc += 1)
bool conv1x1_pre_ok(int64_t M, int K, int N);
Conv1x1Plan conv1x1_stats_plan(int64_t M, int N);
void launch_conv1x1_stats(const uint16_t* x, const uint16_t* w, uint16_t* y, int64_t M, int K, int N,
                          const Conv1x1Plan& p, float* part, hipStream_t s, const float* pre_ss = nullptr,
                          int64_t* nbt_inc = nullptr);
// input gradient of a 1x1 conv (dy1 [M][K] . W, wt = W^T [N][K]) fused with the previous
// BatchNorm's backward partial: d = (da + dy2) * (yb > 0) written to d, part [rows, 2, N]
// = sums of d and d * xb.  part == nullptr: only *rows is set (the partial row count).
bool conv1x1_bn_bwd_ok(int64_t M, int K, int N);
void launch_conv1x1_bn_bwd(const uint16_t* dy1, const uint16_t* wt, uint16_t* d, int64_t M, int K, int N,
                           const uint16_t* dy2, const uint16_t* yb, const uint16_t* xb, float* part, int* rows,
                           hipStream_t s);

// ---------------------------------------------------------------------------
// Fused MNIST-MLP training step (784 -> L1 -> L2 -> 10, ReLU, log_softmax+NLL).
// ---------------------------------------------------------------------------
struct MLPStepArgs {
  // input: either a uint8 dataset gathered through `order` (GPU-resident data,
  // pixels scaled by 1/255 in-kernel) or a dense fp32 batch [B, 784].
  const uint8_t* x_u8;      // [N_data, 784] or null
  const float* x_f32;       // [B, 784] or null
  const int64_t* labels;    // [N_data] (u8 mode) or [B] (f32 mode)
  const int64_t* order;     // [n_batches * B] sample indices for the epoch (u8 mode)
  int64_t* counters;        // [0] optimizer step t, [1] batch cursor (u8 mode)
  int64_t n_batches;        // cursor wraps modulo this (u8 mode)
  int B;                    // full batch size (loss is a mean over B)
  int L1, L2;
  float* params;            // arena: W1[L1,784] b1[L1] W2[L2,L1] b2[L2] W3[10,L2] b3[10]
  float* grads;             // same layout
  float* exp_avg;           // Adam state (same layout) when apply_adam
  float* exp_avg_sq;
  float* stats;             // ring [ring, 4]: loss, correct, count, step
  int stats_ring;
  int accumulate_grad;      // add existing grads (gradient accumulation)
  int apply_adam;           // fuse Adam into the gradient epilogues (world size 1)
  int advance_step;         // increment counters[0] (this call completes an optimizer step)
  float lr, beta1, beta2, eps, weight_decay;
  const float* lr_ptr;
  int adamw;
  int64_t* stamps;          // optional [16] phase timestamps (diagnostics)
  // v2 (two-kernel) step only:
  uint16_t* shadow;         // bf16 weight shadows (row-major copy + W2^T + W3^T), see mlp_shadow_layout
  uint16_t* dh1t;           // scratch [L1, round_up(B, 32)] bf16: dH1^T handed from head to W1 kernel
};

// bf16 shadow layout (elements): [0, np) row-major copy of the fp32 arena,
// [w2t, w2t + L1*L2) W2^T [L1][L2], [w3t, w3t + 16*L2) W3^T [L2][16] (classes
// zero-padded to 16).  The forward/backward read 16-byte bf16 fragments from it.
struct MLPShadowLayout {
  int64_t np, w2t, w3t, total;
};
MLPShadowLayout mlp_shadow_layout(int L1, int L2);

struct MLPAdamArgs {
  float* params;
  const float* grads;
  float* exp_avg;
  float* exp_avg_sq;
  uint16_t* shadow;
  int L1, L2;
  float lr, beta1, beta2, eps, weight_decay, grad_scale;
  int adamw;
  int update;               // 0: only refresh the shadows from params
  const int64_t* step_ptr;  // already-incremented step
  const float* lr_ptr;
};

struct MLPEvalArgs {
  const uint8_t* x_u8;
  const float* x_f32;
  const int64_t* labels;
  const int64_t* index;     // [B] sample indices (u8 mode) or null
  int B, L1, L2;
  const float* params;
  float* logits;            // optional [B, 10] output (log-probabilities)
  float* out;               // [2]: += sum of NLL, += correct count
                            // (partials: [ceil(B/32), 2] per-32-row-chunk sums, overwritten)
  int partials;
};

// v3 (cross-step pipelined layer 1, resident uint8 dataset only); see mlp_step3.hip.
struct MLP3Args {
  const uint8_t* x_u8;      // [N_data, 784]
  const int64_t* labels;    // [N_data]
  const int64_t* order;     // [2][order_stride]: two epochs' sample orders
  int64_t order_stride;     // n_batches * B
  int64_t* counters;        // [10]: (step, next cursor, consumed cursor, ring slot, order buffer) x {current, next};
                            // [10] launch sequence number of the one-launch step (counters of >= 16)
  int64_t n_batches;
  int B, L1, L2;
  float* params;
  float* grads;
  float* exp_avg;
  float* exp_avg_sq;
  uint16_t* shadow;         // bf16 weight shadows (mlp_shadow_layout)
  uint16_t* dh1t;           // [L1][Bp] bf16
  uint16_t* xring;          // [2][49][Bp][16] bf16 X tiles
  int* h1pre;               // [2][copies][Bp * L1] layer-1 pre-activations, 12.20 fixed point (fragment order)
  uint16_t* act;            // [L1 + 2*L2 + 16][Bp] bf16 head -> tail: H1^T, H2^T, dH2^T, dZ^T
  int* yring;               // [2][Bp] int32 staged labels (-1 past B), slot-indexed like xring
  float* stats;
  int stats_ring;
  float* head_part;         // [ceil(B/32)][4] per-head-block (sum NLL, #correct, #rows); B > 32
  int apply_adam;           // head: Adam on the small parameters (world size 1)
  int advance_step;
  float lr, beta1, beta2, eps, weight_decay, grad_scale;
  const float* lr_ptr;
  int adamw;
  int64_t* stamps;
  // fused data-parallel tail (kMLP3StepDP): the comm engine's auxiliary peer
  // region (csrc/comm/communicator.h aux_context)
  char* dp_regions[8];
  uint32_t* dp_gen;         // [128] per-block generations (local device memory)
  int* dp_err;              // host-mapped error word
  int64_t dp_stride;        // floats per (slot, rank) receive area (>= param count)
  int64_t dp_spin;          // poll bound
  int dp_rank, dp_world;
  int dp_lite;              // exchange protocol: 2 tagged granules (default), 1 flags + one fencing wave, 0 flags + all waves
  // one-launch step (kMLP3Step1DP) exchange: 0 arena-indexed {gen, fp32} granules (round 2),
  // 1 "packed" one-shot (wave-positioned, two values per granule), 2 "owner" (reduce-scatter to
  // the task's owner rank, Adam there, all-gather of the fp32 weights)
  int dp_proto;
  // loopback (diagnostic): one process plays all dp_world ranks through its own region
  // (every region pointer is this rank's; the block writes every source slot itself)
  int dp_loop;
  // one-launch step (kMLP3Step1): in-launch hand-off words (mlp_step3.hip) and their poll bound
  unsigned long long* hand;
  int64_t hand_spin;
};
enum MLP3Kind { kMLP3Step = 0, kMLP3Head = 1, kMLP3TailGrad = 2, kMLP3TailAdam = 3, kMLP3Prime = 4,
                kMLP3StepDP = 5, kMLP3Step1 = 6, kMLP3Step1DP = 7 };
int64_t mlp3_hand_words(int L1, int L2);  // int64 words of the one-launch step's hand-off buffer
int launch_mlp3(const MLP3Args& a, int kind, hipStream_t stream);

int mlp3_act_rows(int L1, int L2);
int mlp3_h1_copies(int L1);  // H1pre copies per ring slot (mlp_step3.hip H1Copies)
// the packed DP exchange's wire form of fp32 pairs, encoded and decoded (tests)
int dp_pack_roundtrip(const float* x, float* y, int64_t n, int tag, hipStream_t stream);

// returns 0 on success, -1 if (L1, L2) has no compiled instantiation
int launch_mlp_train_step(const MLPStepArgs& a, hipStream_t stream);
int launch_mlp_eval(const MLPEvalArgs& a, hipStream_t stream);
bool mlp_supported(int L1, int L2);
int launch_mlp_adam(const MLPAdamArgs& a, hipStream_t stream);

}  // namespace rla

namespace rla {
// ---------------------------------------------------------------------------
// Weight gradient of NHWC bf16 convolutions on MFMA (csrc/conv_wgrad.hip):
// dW [Cout][KH][KW][Cin] fp32 = sum over output rows of dy x shifted x.
// Cout % 64 == 0, Cin % 64 == 0.
// ---------------------------------------------------------------------------
struct WgradGeom {
  int N, H, W, Cin;   // x  [N, H, W, Cin]
  int OH, OW, Cout;   // dy [N, OH, OW, Cout]
  int KH, KW, sh, sw, ph, pw;
};
struct WgradPlan {
  int kind;                // 0 generic (any geometry), 1 3x3 / stride 1 / pad 1 halo kernel
  int wa, wb;              // workgroup tile = (64 wa) x (64 wb) channels
  int splits;              // row splits (> 1: fp32 partials + a reduce kernel)
  int64_t rows_per_split;  // kind 1: stages (64 output rows each) per split
};
// splits <= 0: automatic; algo 0: the halo kernel when the geometry allows, 1: generic
WgradPlan wgrad_plan(const WgradGeom& g, int splits, int algo = 0);
// part: splits * Cout * KH * KW * Cin floats when plan.splits > 1 (else unused)
// pre_ss ([4, Cin] BatchNorm stats; generic 1x1 / stride-1 plans only): x is a deferred
// BatchNorm + ReLU's input, staged as bf16(relu(x * scale + shift))
void launch_wgrad(const uint16_t* dy, const uint16_t* x, float* out, float* part, const WgradGeom& g,
                  const WgradPlan& p, hipStream_t stream, const float* pre_ss = nullptr);

// ---------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 NHWC bf16 convolution on MFMA (csrc/conv3x3.hip):
// y [N, H, W, Cout] = conv(x [N, H, W, Cin], w [Cout][3][3][Cin]); also the input
// gradient with the flipped, transposed weight.  Cin % 16 == 0, Cout % 64 == 0.
// ---------------------------------------------------------------------------
struct Conv3x3Geom {
  int N, H, W, Cin, Cout;
  int vrows;  // halo rows of the largest pixel tile (conv3x3_vrows)
  int tm;     // pixels per workgroup tile: 256 or 512 (conv3x3_pick_tm)
  int wpb;    // workgroups per 64-channel output block = contiguous pixel ranges (conv3x3_wpb)
};
int conv3x3_wpb(int N, int H, int W, int Cout);
int conv3x3_pick_tm(int N, int H, int W, int Cout);
int conv3x3_vrows(const Conv3x3Geom& g);
bool conv3x3_ok(const Conv3x3Geom& g);
// flip: input gradient -- x is dy [N, H, W, Cin], w the FORWARD weight [Cin][3][3][Cout]
// (Cin = the forward's output channels), y is dx [N, H, W, Cout]
// part (forward only, or null): BatchNorm partial sums of bf16(y), [g.wpb][2][Cout] fp32
// pre_ss (forward with part only; [4, Cin] BatchNorm stats, Cin <= 512): x is a deferred
// BatchNorm + ReLU's input, staged as bf16(relu(x * scale + shift)); nbt_inc += 1
bool conv3x3_pre_ok(const Conv3x3Geom& g);
bool launch_conv3x3(const uint16_t* x, const uint16_t* w, uint16_t* y, const Conv3x3Geom& g, bool flip,
                    hipStream_t stream, float* part = nullptr, const float* pre_ss = nullptr,
                    int64_t* nbt_inc = nullptr);

// ResNet stem: 7x7 / stride 2 / pad 3 convolution, 3 -> 64 channels, NHWC bf16 (csrc/stem.hip);
// part (or null): BatchNorm partial sums of bf16(y), [stem_grid(g)][2][64] fp32
struct StemGeom {
  int N, H, W, OH, OW;
};
bool stem_ok(const StemGeom& g);
int stem_grid(const StemGeom& g);
bool launch_stem_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, float* part, const StemGeom& g,
                     hipStream_t stream);
// weight gradient: dy [N, OH, OW, 64] bf16 -> dw [64][7][7][3] fp32; part: [stem_grid(g)][64][224] fp32 workspace
bool launch_stem_wgrad(const uint16_t* x, const uint16_t* dy, float* part, float* dw, const StemGeom& g,
                       hipStream_t stream);

}  // namespace rla
