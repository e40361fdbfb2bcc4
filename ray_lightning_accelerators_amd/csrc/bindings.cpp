// torch bindings for the gfx950 kernels (module `ray_lightning_accelerators_amd._C`).
//
// Every entry point validates device / dtype / contiguity / sizes on the host
// before launching: a hand-written kernel must never see a shape it was not
// built for (an out-of-bounds access can reset every GPU of the host).
#include <torch/extension.h>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels.h"
#include "comm/xgmi.h"

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream(const Tensor& t) {
  return at::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.get_device()).stream();
}

void check_dev(const Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

template <class T>
T* ptr_or_null(const optional<Tensor>& t, const char* name, at::ScalarType dt, int64_t min_numel = 0) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_dev(*t, name, dt);
  TORCH_CHECK(t->numel() >= min_numel, name, " has ", t->numel(), " elements, need >= ", min_numel);
  return reinterpret_cast<T*>(t->data_ptr());
}

void adam_step(Tensor p, Tensor g, Tensor m, Tensor v, optional<Tensor> p_bf16, double lr,
               double beta1, double beta2, double eps, double weight_decay, double grad_scale,
               bool adamw, bool maximize, optional<Tensor> step, int64_t host_step,
               optional<Tensor> lr_t) {
  check_dev(p, "param", at::kFloat);
  check_dev(g, "grad", at::kFloat);
  check_dev(m, "exp_avg", at::kFloat);
  check_dev(v, "exp_avg_sq", at::kFloat);
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam arena size mismatch");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  rla::AdamArgs a{};
  a.p = p.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.m = m.data_ptr<float>();
  a.v = v.data_ptr<float>();
  a.p_bf16 = ptr_or_null<uint16_t>(p_bf16, "param_bf16", at::kBFloat16, n);
  a.n = n;
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.weight_decay = (float)weight_decay; a.grad_scale = (float)grad_scale;
  a.adamw = adamw; a.maximize = maximize;
  a.step_ptr = ptr_or_null<const int64_t>(step, "step", at::kLong, 1);
  a.host_step = host_step;
  a.lr_ptr = ptr_or_null<const float>(lr_t, "lr", at::kFloat, 1);
  TORCH_CHECK(a.step_ptr || host_step >= 1, "adam: step must be >= 1");
  rla::launch_adam(a, cur_stream(p));
}

void sgd_step(Tensor p, Tensor g, optional<Tensor> buf, optional<Tensor> p_bf16, double lr,
              double momentum, double dampening, double weight_decay, double grad_scale,
              bool nesterov, bool maximize, optional<Tensor> step, int64_t host_step,
              optional<Tensor> lr_t) {
  check_dev(p, "param", at::kFloat);
  check_dev(g, "grad", at::kFloat);
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n, "sgd arena size mismatch");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  rla::SGDArgs a{};
  a.p = p.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.buf = ptr_or_null<float>(buf, "momentum_buffer", at::kFloat, n);
  TORCH_CHECK(momentum == 0.0 || a.buf != nullptr, "sgd: momentum needs a buffer");
  a.p_bf16 = ptr_or_null<uint16_t>(p_bf16, "param_bf16", at::kBFloat16, n);
  a.n = n;
  a.lr = (float)lr; a.momentum = (float)momentum; a.dampening = (float)dampening;
  a.weight_decay = (float)weight_decay; a.grad_scale = (float)grad_scale;
  a.nesterov = nesterov; a.maximize = maximize;
  a.step_ptr = ptr_or_null<const int64_t>(step, "step", at::kLong, 1);
  a.host_step = host_step;
  a.lr_ptr = ptr_or_null<const float>(lr_t, "lr", at::kFloat, 1);
  rla::launch_sgd(a, cur_stream(p));
}

void multi_copy(Tensor table, double scale, bool accumulate) {
  check_dev(table, "table", at::kLong);
  TORCH_CHECK(table.dim() == 2 && table.size(1) == 4, "table must be [nchunks, 4]");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  rla::launch_multi_copy(table.data_ptr<int64_t>(), table.size(0), (float)scale, accumulate,
                         cur_stream(table));
}

void scale_(Tensor x, double s) {
  check_dev(x, "x", at::kFloat);
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  rla::launch_scale(x.data_ptr<float>(), x.numel(), (float)s, cur_stream(x));
}

Tensor sumsq(Tensor x) {
  check_dev(x, "x", at::kFloat);
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor out = at::empty({1}, x.options());
  rla::launch_sumsq(x.data_ptr<float>(), x.numel(), out.data_ptr<float>(), cur_stream(x));
  return out;
}

int64_t mlp_param_count(int64_t L1, int64_t L2) {
  return L1 * 784 + L1 + L2 * L1 + L2 + 10 * L2 + 10;
}

void mlp_train_step(optional<Tensor> x_u8, optional<Tensor> x_f32, Tensor labels,
                    optional<Tensor> order, optional<Tensor> counters, int64_t n_batches, int64_t B,
                    int64_t L1, int64_t L2, Tensor params, Tensor grads, optional<Tensor> exp_avg,
                    optional<Tensor> exp_avg_sq, optional<Tensor> stats, bool accumulate_grad,
                    bool apply_adam, bool advance_step, double lr, double beta1, double beta2,
                    double eps, double weight_decay, optional<Tensor> lr_t, bool adamw,
                    optional<Tensor> stamps) {
  TORCH_CHECK(rla::mlp_supported((int)L1, (int)L2), "no fused MLP kernel for layer sizes ", L1, "/", L2);
  TORCH_CHECK(B >= 1, "batch size must be >= 1");
  const int64_t np = mlp_param_count(L1, L2);
  check_dev(params, "params", at::kFloat);
  check_dev(grads, "grads", at::kFloat);
  TORCH_CHECK(params.numel() == np && grads.numel() == np, "param arena must hold ", np, " floats");
  check_dev(labels, "labels", at::kLong);
  const at::hip::HIPGuardMasqueradingAsCUDA guard(params.device());
  rla::MLPStepArgs a{};
  a.x_u8 = ptr_or_null<const uint8_t>(x_u8, "x_u8", at::kByte);
  a.x_f32 = ptr_or_null<const float>(x_f32, "x_f32", at::kFloat);
  TORCH_CHECK((a.x_u8 != nullptr) != (a.x_f32 != nullptr), "pass exactly one of x_u8 / x_f32");
  if (a.x_u8) {
    TORCH_CHECK(x_u8->dim() == 2 && x_u8->size(1) == 784, "x_u8 must be [N, 784]");
    TORCH_CHECK(labels.numel() == x_u8->size(0), "labels must match the dataset");
    a.order = ptr_or_null<const int64_t>(order, "order", at::kLong, n_batches * B);
    TORCH_CHECK(a.order != nullptr && n_batches >= 1, "u8 mode needs order[n_batches * B]");
    a.counters = ptr_or_null<int64_t>(counters, "counters", at::kLong, 2);
    TORCH_CHECK(a.counters != nullptr, "u8 mode needs device counters");
    // Indices are range-checked on the host by the caller when `order` is
    // built (see ops.fused_mlp.MLPDataset); the kernel trusts them.
  } else {
    TORCH_CHECK(x_f32->numel() == B * 784, "x_f32 must be [B, 784]");
    TORCH_CHECK(labels.numel() == B, "labels must be [B]");
    a.counters = ptr_or_null<int64_t>(counters, "counters", at::kLong, 2);
  }
  a.labels = labels.data_ptr<int64_t>();
  a.n_batches = n_batches;
  a.B = (int)B; a.L1 = (int)L1; a.L2 = (int)L2;
  a.params = params.data_ptr<float>();
  a.grads = grads.data_ptr<float>();
  a.exp_avg = ptr_or_null<float>(exp_avg, "exp_avg", at::kFloat, np);
  a.exp_avg_sq = ptr_or_null<float>(exp_avg_sq, "exp_avg_sq", at::kFloat, np);
  TORCH_CHECK(!apply_adam || (a.exp_avg && a.exp_avg_sq), "apply_adam needs optimizer state");
  a.stats = ptr_or_null<float>(stats, "stats", at::kFloat, 4);
  a.stats_ring = a.stats ? (int)(stats->numel() / 4) : 0;
  a.accumulate_grad = accumulate_grad;
  a.apply_adam = apply_adam;
  a.advance_step = advance_step;
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.lr_ptr = ptr_or_null<const float>(lr_t, "lr", at::kFloat, 1);
  a.adamw = adamw;
  a.stamps = ptr_or_null<int64_t>(stamps, "stamps", at::kLong, 16);
  TORCH_CHECK(rla::launch_mlp_train_step(a, cur_stream(params)) == 0, "fused MLP launch failed");
}

// v3 pipelined step.  kind: 0 step (head + fused tail), 1 head only (grads),
// 2 tail GRAD, 3 tail ADAM (after the allreduce), 4 PRIME (H1pre of the pending batch).
void mlp3(int64_t kind, Tensor x_u8, Tensor labels, Tensor order, Tensor counters, int64_t n_batches, int64_t B,
          int64_t L1, int64_t L2, Tensor params, Tensor grads, Tensor exp_avg, Tensor exp_avg_sq, Tensor shadow,
          Tensor dh1t, Tensor xring, Tensor h1pre, Tensor act, Tensor yring, optional<Tensor> stats,
          bool advance_step, double lr,
          double beta1, double beta2, double eps, double weight_decay, double grad_scale, optional<Tensor> lr_t,
          bool adamw, optional<Tensor> stamps, std::vector<int64_t> dp_ctx, optional<Tensor> head_part,
          optional<Tensor> hand, int64_t dp_proto, bool dp_loop, int64_t repeat) {
  TORCH_CHECK(kind >= 0 && kind <= 7, "mlp3: bad kind ", kind);
  TORCH_CHECK(repeat >= 1, "mlp3: repeat must be >= 1");
  TORCH_CHECK(rla::mlp_supported((int)L1, (int)L2), "no fused MLP kernel for layer sizes ", L1, "/", L2);
  TORCH_CHECK(B >= 1 && B <= 256, "fused MLP step supports 1 <= batch <= 256");
  const int64_t np = mlp_param_count(L1, L2);
  const int64_t Bp = (B + 31) / 32 * 32;
  const rla::MLPShadowLayout lay = rla::mlp_shadow_layout((int)L1, (int)L2);
  check_dev(params, "params", at::kFloat);
  check_dev(grads, "grads", at::kFloat);
  check_dev(exp_avg, "exp_avg", at::kFloat);
  check_dev(exp_avg_sq, "exp_avg_sq", at::kFloat);
  TORCH_CHECK(params.numel() == np && grads.numel() == np && exp_avg.numel() == np && exp_avg_sq.numel() == np,
              "param / grad / Adam arenas must hold ", np, " floats");
  check_dev(shadow, "shadow", at::kBFloat16);
  TORCH_CHECK(shadow.numel() >= lay.total, "shadow must hold ", lay.total, " bf16");
  check_dev(dh1t, "dh1t", at::kBFloat16);
  TORCH_CHECK(dh1t.numel() >= L1 * Bp, "dh1t must hold L1 * round_up(B, 32)");
  check_dev(xring, "xring", at::kBFloat16);
  TORCH_CHECK(xring.numel() >= 2 * 49 * Bp * 16, "xring must hold 2 * 49 * round_up(B, 32) * 16");
  check_dev(h1pre, "h1pre", at::kInt);
  TORCH_CHECK(h1pre.numel() >= 2 * rla::mlp3_h1_copies((int)L1) * Bp * L1,
              "h1pre must hold 2 * mlp3_h1_copies(L1) * round_up(B, 32) * L1");
  check_dev(act, "act", at::kBFloat16);
  TORCH_CHECK(act.numel() >= rla::mlp3_act_rows((int)L1, (int)L2) * Bp, "act must hold (L1 + 2 L2 + 16) * Bp");
  check_dev(counters, "counters", at::kLong);
  TORCH_CHECK(counters.numel() >= 10, "counters must hold 10 int64 (current + advanced state)");
  check_dev(yring, "yring", at::kInt);
  TORCH_CHECK(yring.numel() >= 2 * Bp, "yring must hold 2 * round_up(B, 32) int32");
  check_dev(x_u8, "x_u8", at::kByte);
  TORCH_CHECK(x_u8.dim() == 2 && x_u8.size(1) == 784, "x_u8 must be [N, 784]");
  check_dev(labels, "labels", at::kLong);
  TORCH_CHECK(labels.numel() == x_u8.size(0), "labels must match the dataset");
  check_dev(order, "order", at::kLong);
  TORCH_CHECK(n_batches >= 1 && order.numel() >= 2 * n_batches * B, "order must be [2, n_batches * B]");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(params.device());
  rla::MLP3Args a{};
  a.x_u8 = x_u8.data_ptr<uint8_t>();
  a.labels = labels.data_ptr<int64_t>();
  a.order = order.data_ptr<int64_t>();
  a.order_stride = order.numel() / 2;
  a.counters = counters.data_ptr<int64_t>();
  a.n_batches = n_batches;
  a.B = (int)B; a.L1 = (int)L1; a.L2 = (int)L2;
  a.params = params.data_ptr<float>();
  a.grads = grads.data_ptr<float>();
  a.exp_avg = exp_avg.data_ptr<float>();
  a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  a.shadow = reinterpret_cast<uint16_t*>(shadow.data_ptr());
  a.dh1t = reinterpret_cast<uint16_t*>(dh1t.data_ptr());
  a.xring = reinterpret_cast<uint16_t*>(xring.data_ptr());
  a.h1pre = h1pre.data_ptr<int>();
  a.act = reinterpret_cast<uint16_t*>(act.data_ptr());
  a.yring = yring.data_ptr<int>();
  a.stats = ptr_or_null<float>(stats, "stats", at::kFloat, 4);
  a.stats_ring = a.stats ? (int)(stats->numel() / 4) : 0;
  a.head_part = ptr_or_null<float>(head_part, "head_part", at::kFloat, (Bp / 32) * 4);
  TORCH_CHECK(B <= 32 || a.head_part != nullptr, "mlp3: batches above 32 rows need head_part [ceil(B/32), 4]");
  if (kind == rla::kMLP3Step1 || kind == rla::kMLP3Step1DP) {
    TORCH_CHECK(B <= 32, "the one-launch step handles batches of up to 32 rows");
    TORCH_CHECK(counters.numel() >= 16, "the one-launch step needs counters of >= 16 int64 (launch sequence)");
    a.hand = reinterpret_cast<unsigned long long*>(
        ptr_or_null<int64_t>(hand, "hand", at::kLong, rla::mlp3_hand_words((int)L1, (int)L2)));
    TORCH_CHECK(a.hand != nullptr, "the one-launch step needs the hand-off buffer `hand`");
    a.hand_spin = 1 << 20;
  }
  a.apply_adam = kind == rla::kMLP3Step;
  a.advance_step = advance_step;
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.grad_scale = (float)grad_scale;
  a.lr_ptr = ptr_or_null<const float>(lr_t, "lr", at::kFloat, 1);
  a.adamw = adamw;
  a.stamps = ptr_or_null<int64_t>(stamps, "stamps", at::kLong, 16);
  if (kind == rla::kMLP3StepDP || kind == rla::kMLP3Step1DP) {
    // [world, rank, stride, spin, gen_ptr, err_ptr, region_ptr x world] from the comm engine
    TORCH_CHECK(dp_ctx.size() >= 6 && dp_ctx[0] >= 1 && dp_ctx[0] <= 8 && (int64_t)dp_ctx.size() == 6 + dp_ctx[0],
                "mlp3 StepDP needs the comm engine's aux_context()");
    a.dp_world = (int)dp_ctx[0];
    a.dp_rank = (int)dp_ctx[1];
    TORCH_CHECK(a.dp_rank >= 0 && a.dp_rank < a.dp_world, "bad dp rank");
    a.dp_stride = dp_ctx[2];
    TORCH_CHECK(a.dp_stride >= np, "aux receive area smaller than the parameter arena");
    a.dp_spin = dp_ctx[3];
    a.dp_gen = reinterpret_cast<uint32_t*>(dp_ctx[4]);
    a.dp_err = reinterpret_cast<int*>(dp_ctx[5]);
    for (int r = 0; r < a.dp_world; ++r) a.dp_regions[r] = reinterpret_cast<char*>(dp_ctx[6 + r]);
    // exchange protocol: "granule" (default: tagged 8-byte words, no fences; needs a
    // receive area of 2 floats per parameter), "wave" (flags, one wave fences),
    // "all" (flags, every wave fences)
    // one-launch step (dp_proto): 0 "granule" (round 2, arena-indexed), 1 "packed"
    // one-shot, 2 "owner" (reduce-scatter / owner Adam / all-gather); -1: RLA_DP_PROTO
    const char* proto = std::getenv("RLA_DP_PROTO");
    const std::string pr = proto ? proto : "";
    a.dp_lite = pr == "all" ? 0 : (pr == "wave" ? 1 : 2);
    if (a.dp_lite == 2 && a.dp_stride < 2 * np) a.dp_lite = 1;  // area too small for granules
    if (dp_proto < 0) dp_proto = pr == "granule" ? 0 : (pr == "owner" ? 2 : 1);
    TORCH_CHECK(dp_proto >= 0 && dp_proto <= 2, "dp_proto: 0 granule, 1 packed, 2 owner");
    a.dp_proto = (int)dp_proto;
    a.dp_loop = dp_loop ? 1 : 0;
    if (kind == rla::kMLP3Step1DP) {
      TORCH_CHECK(a.dp_proto != 0 || (a.dp_lite == 2 && a.dp_stride >= 2 * np),
                  "the one-launch step's granule protocol needs a receive area of 2 floats per parameter");
      TORCH_CHECK(a.dp_proto == 0 || a.dp_stride >= rla::comm::kDpUnitAreaFloats,
                  "the packed / owner protocols need a receive area of ", rla::comm::kDpUnitAreaFloats,
                  " floats (mlp3_dp_area_floats())");
    }
    TORCH_CHECK(!dp_loop || kind == rla::kMLP3Step1DP, "loopback is a one-launch-step diagnostic");
  }
  // repeat: the same launch back to back (every step's state lives on the device:
  // counters, rings, generations), issued from this C++ loop -- one host call for a
  // window of steps, a few us of launch work each against ~8 us of GPU time
  const hipStream_t st = cur_stream(params);
  for (int64_t i = 0; i < repeat; ++i)
    TORCH_CHECK(rla::launch_mlp3(a, (int)kind, st) == 0, "fused MLP v3 launch failed");
}

void mlp_adam(Tensor params, Tensor grads, Tensor exp_avg, Tensor exp_avg_sq, Tensor shadow, int64_t L1,
              int64_t L2, double lr, double beta1, double beta2, double eps, double weight_decay,
              double grad_scale, bool adamw, bool update, optional<Tensor> step, optional<Tensor> lr_t) {
  TORCH_CHECK(rla::mlp_supported((int)L1, (int)L2), "no fused MLP kernel for layer sizes ", L1, "/", L2);
  const int64_t np = mlp_param_count(L1, L2);
  const rla::MLPShadowLayout lay = rla::mlp_shadow_layout((int)L1, (int)L2);
  check_dev(params, "params", at::kFloat);
  TORCH_CHECK(params.numel() == np, "param arena size mismatch");
  check_dev(shadow, "shadow", at::kBFloat16);
  TORCH_CHECK(shadow.numel() >= lay.total, "shadow too small");
  rla::MLPAdamArgs a{};
  if (update) {
    check_dev(grads, "grads", at::kFloat);
    check_dev(exp_avg, "exp_avg", at::kFloat);
    check_dev(exp_avg_sq, "exp_avg_sq", at::kFloat);
    TORCH_CHECK(grads.numel() == np && exp_avg.numel() == np && exp_avg_sq.numel() == np, "arena size mismatch");
    a.grads = grads.data_ptr<float>();
    a.exp_avg = exp_avg.data_ptr<float>();
    a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
    a.step_ptr = ptr_or_null<const int64_t>(step, "step", at::kLong, 1);
    TORCH_CHECK(a.step_ptr != nullptr, "mlp_adam(update=True) needs the device step counter");
  }
  const at::hip::HIPGuardMasqueradingAsCUDA guard(params.device());
  a.params = params.data_ptr<float>();
  a.shadow = reinterpret_cast<uint16_t*>(shadow.data_ptr());
  a.L1 = (int)L1; a.L2 = (int)L2;
  a.lr = (float)lr; a.beta1 = (float)beta1; a.beta2 = (float)beta2; a.eps = (float)eps;
  a.weight_decay = (float)weight_decay; a.grad_scale = (float)grad_scale;
  a.adamw = adamw; a.update = update;
  a.lr_ptr = ptr_or_null<const float>(lr_t, "lr", at::kFloat, 1);
  TORCH_CHECK(rla::launch_mlp_adam(a, cur_stream(params)) == 0, "mlp_adam launch failed");
}

void mlp_eval(optional<Tensor> x_u8, optional<Tensor> x_f32, Tensor labels, optional<Tensor> index,
              int64_t B, int64_t L1, int64_t L2, Tensor params, optional<Tensor> logits, Tensor out) {
  TORCH_CHECK(rla::mlp_supported((int)L1, (int)L2), "no fused MLP kernel for layer sizes ", L1, "/", L2);
  check_dev(params, "params", at::kFloat);
  TORCH_CHECK(params.numel() == mlp_param_count(L1, L2), "param arena size mismatch");
  check_dev(labels, "labels", at::kLong);
  check_dev(out, "out", at::kFloat);
  TORCH_CHECK(out.is_contiguous(), "out must be contiguous");
  // out [2] accumulates; out [ceil(B/32), 2] receives per-32-row-chunk partial sums
  const bool partials = out.dim() == 2;
  TORCH_CHECK(partials ? (out.size(0) == (B + 31) / 32 && out.size(1) == 2) : out.numel() >= 2,
              "out must be [2] or [ceil(B/32), 2]");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(params.device());
  rla::MLPEvalArgs a{};
  a.x_u8 = ptr_or_null<const uint8_t>(x_u8, "x_u8", at::kByte);
  a.x_f32 = ptr_or_null<const float>(x_f32, "x_f32", at::kFloat);
  TORCH_CHECK((a.x_u8 != nullptr) != (a.x_f32 != nullptr), "pass exactly one of x_u8 / x_f32");
  if (a.x_u8) {
    TORCH_CHECK(x_u8->dim() == 2 && x_u8->size(1) == 784, "x_u8 must be [N, 784]");
    a.index = ptr_or_null<const int64_t>(index, "index", at::kLong, B);
    TORCH_CHECK(a.index != nullptr, "u8 mode needs index[B]");
  } else {
    TORCH_CHECK(x_f32->numel() == B * 784, "x_f32 must be [B, 784]");
    TORCH_CHECK(labels.numel() == B, "labels must be [B]");
  }
  a.labels = labels.data_ptr<int64_t>();
  a.B = (int)B; a.L1 = (int)L1; a.L2 = (int)L2;
  a.params = params.data_ptr<float>();
  a.logits = ptr_or_null<float>(logits, "logits", at::kFloat, B * 10);
  a.out = out.data_ptr<float>();
  a.partials = partials ? 1 : 0;
  TORCH_CHECK(rla::launch_mlp_eval(a, cur_stream(params)) == 0, "fused MLP eval launch failed");
}

// ---- fused BatchNorm(+ReLU)(+residual add) over NHWC bf16 activations --------------
// Tensors are passed as contiguous [..., C] views (channels_last NCHW permuted to
// NHWC): every shape / alignment assumption of csrc/bn_act.hip is checked here.
int64_t bn_rows(const Tensor& x, const char* name, int64_t C) {
  check_dev(x, name, at::kBFloat16);
  TORCH_CHECK(C > 0 && C % 8 == 0 && C <= rla::kBnMaxC, "fused BN: C must be a multiple of 8 and <= ",
              rla::kBnMaxC, ", got ", C);
  TORCH_CHECK(x.dim() >= 1 && x.size(-1) == C, name, " must have C=", C, " as its innermost dimension");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
  return x.numel() / C;
}

void bn_same(const Tensor& a, const Tensor& b, const char* name, int64_t C) {
  TORCH_CHECK(bn_rows(b, name, C) * C == a.numel(), name, " size mismatch");
}

const float* f32_vec(const optional<Tensor>& t, const char* name, int64_t C) {
  return ptr_or_null<const float>(t, name, at::kFloat, C);
}

// optional dy2 (backward only): a second incoming gradient summed with dy in-kernel
const uint16_t* bn_dy2(const Tensor& x, const optional<Tensor>& dy2, int64_t C) {
  if (!dy2.has_value() || !dy2->defined()) return nullptr;
  bn_same(x, *dy2, "dy2", C);
  return reinterpret_cast<const uint16_t*>(dy2->data_ptr());
}

// optional forward statistics [4, C] (mean, invstd, scale, shift): the backward's
// ReLU mask is recomputed from x instead of read from the saved output y
const float* bn_ss(const optional<Tensor>& ss, int64_t C) {
  if (!ss.has_value() || !ss->defined()) return nullptr;
  check_dev(*ss, "stats", at::kFloat);
  TORCH_CHECK(ss->dim() == 2 && ss->size(0) == 4 && ss->size(1) == C && ss->is_contiguous(),
              "stats must be a contiguous [4, C] fp32 tensor");
  return ss->data_ptr<float>();
}

// Ticket counters of the BN partial kernels' second reduction level: one zeroed
// buffer per device, allocated outside any stream capture (hipMalloc is not
// capturable; a capture that finds none yet runs the single-level partials) and
// reset in-kernel by each group's last block.  Launches on one stream never
// overlap, so every call can reuse the same tickets.
int* bn_tickets(int device, hipStream_t stream) {
  static int* bufs[64] = {};
  if (device < 0 || device >= 64) return nullptr;
  if (bufs[device]) return bufs[device];
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  int* p = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&p), 4096 * sizeof(int)) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, 4096 * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return nullptr;
  bufs[device] = p;
  return p;
}

// the stem's pooled BatchNorm (ops/bn.py `pool`): dy is the POOLED output's gradient
// [N, OH, OW, C] and arg its window argmax; geometry (H, W, k, s, pad) of the pool
static bool pool_grad(const Tensor& x, const optional<Tensor>& pool_arg, const Tensor& dy,
                      const std::vector<int64_t>& geo, int64_t C, rla::PoolGrad* pg) {
  if (!(pool_arg.has_value() && pool_arg->defined())) return false;
  TORCH_CHECK(geo.size() == 5, "pool geometry (H, W, k, s, pad)");
  const int64_t H = geo[0], W = geo[1], k = geo[2], s = geo[3], pad = geo[4];
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && pad >= 0 && 2 * pad <= k, "pool: bad geometry");
  const int64_t OH = (H + 2 * pad - k) / s + 1, OW = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(x.numel() % (H * W * C) == 0, "pool: x is not [N, H, W, C]");
  const int64_t N = x.numel() / (H * W * C);
  check_dev(dy, "dy", at::kBFloat16);
  TORCH_CHECK(dy.is_contiguous() && dy.numel() == N * OH * OW * C, "pool: dy must be the pooled [N, OH, OW, C]");
  TORCH_CHECK(pool_arg->is_cuda() && pool_arg->scalar_type() == at::kByte && pool_arg->is_contiguous() &&
                  pool_arg->numel() == dy.numel(),
              "pool: arg must be the forward's argmax bytes");
  *pg = rla::PoolGrad{reinterpret_cast<const uint16_t*>(dy.data_ptr()), pool_arg->data_ptr<uint8_t>(), (int)H,
                      (int)W, (int)OH, (int)OW, (int)k, (int)s, (int)pad};
  return true;
}

Tensor bn_partial(Tensor x, optional<Tensor> y, optional<Tensor> dy, int64_t C, int64_t mode, bool relu,
                  optional<Tensor> nbt, optional<Tensor> dy2, optional<Tensor> ss, optional<Tensor> dout,
                  optional<Tensor> pool_arg, std::vector<int64_t> pool_geo) {
  rla::PoolGrad pg{};
  const bool pooled = mode == 1 && dy.has_value() && pool_grad(x, pool_arg, *dy, pool_geo, C, &pg);
  TORCH_CHECK(!pooled || (relu && ss.has_value() && ss->defined() && !(dout.has_value() && dout->defined()) &&
                          !(dy2.has_value() && dy2->defined())),
              "pooled BN backward: ReLU with the forward stats only");
  const int64_t M = bn_rows(x, "x", C);
  TORCH_CHECK(M > 0, "fused BN: empty input");
  TORCH_CHECK(mode == 0 || mode == 1, "fused BN: mode 0 (forward) or 1 (backward)");
  const uint16_t* yp = nullptr;
  const uint16_t* dyp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(dy.has_value(), "backward partial needs dy");
    if (!pooled) bn_same(x, *dy, "dy", C);
    dyp = reinterpret_cast<const uint16_t*>(dy->data_ptr());
    if (relu && !(ss.has_value() && ss->defined())) {
      TORCH_CHECK(y.has_value(), "ReLU backward needs the saved output y (or the forward stats)");
      bn_same(x, *y, "y", C);
      yp = reinterpret_cast<const uint16_t*>(y->data_ptr());
    }
  }
  uint16_t* doutp = nullptr;
  if (dout.has_value() && dout->defined()) {
    TORCH_CHECK(mode == 1, "dout: backward partial only");
    TORCH_CHECK(!(ss.has_value() && ss->defined()), "dout: y-masked (residual) layers only");
    bn_same(x, *dout, "dout", C);
    doutp = reinterpret_cast<uint16_t*>(dout->data_ptr());
  }
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const rla::BnPlan plan = rla::bn_plan(M, (int)C);
  Tensor part = at::empty({plan.blocks, 2, C}, x.options().dtype(at::kFloat));
  int64_t* nbtp = mode == 0 ? ptr_or_null<int64_t>(nbt, "num_batches_tracked", at::kLong, 1) : nullptr;
  // second reduction level in the partial kernel: the finalize reads `groups` fp64
  // rows (returned instead of the per-block fp32 partials)
  rla::BnLevel2 lv{nullptr, nullptr};
  Tensor rows;
  int* tickets = plan.group > 1 ? bn_tickets(x.device().index(), cur_stream(x)) : nullptr;
  if (tickets) {
    rows = at::empty({plan.groups, 2, C}, x.options().dtype(at::kDouble));
    lv = rla::BnLevel2{rows.data_ptr<double>(), tickets};
  }
  rla::launch_bn_partial(reinterpret_cast<const uint16_t*>(x.data_ptr()), yp, dyp, M, (int)C, (int)mode, relu,
                         plan, part.data_ptr<float>(), nbtp, cur_stream(x), mode == 1 ? bn_dy2(x, dy2, C) : nullptr,
                         mode == 1 && relu ? bn_ss(ss, C) : nullptr, lv, doutp, pooled ? &pg : nullptr);
  return tickets ? rows : part;
}

Tensor bn_finalize(Tensor part, double count, optional<Tensor> weight, optional<Tensor> bias,
                   optional<Tensor> running_mean, optional<Tensor> running_var, optional<Tensor> nbt,
                   double momentum, double eps, bool nbt_pending) {
  const bool l2 = part.scalar_type() == at::kDouble;  // second-level rows of bn_partial
  TORCH_CHECK(!(l2 && nbt_pending), "nbt_pending: conv-epilogue partials are fp32 rows");
  check_dev(part, "partials", l2 ? at::kDouble : at::kFloat);
  TORCH_CHECK(part.dim() == 3 && part.size(1) == 2, "partials must be [blocks, 2, C]");
  const int64_t C = part.size(2);
  TORCH_CHECK(count > 0, "fused BN: count must be > 0");
  float* rm = ptr_or_null<float>(running_mean, "running_mean", at::kFloat, C);
  float* rv = ptr_or_null<float>(running_var, "running_var", at::kFloat, C);
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean / running_var go together");
  const int64_t* nbtp = ptr_or_null<const int64_t>(nbt, "num_batches_tracked", at::kLong, 1);
  TORCH_CHECK(momentum >= 0 || nbtp, "cumulative averaging (momentum=None) needs num_batches_tracked");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(part.device());
  Tensor stats = at::empty({4, C}, part.options().dtype(at::kFloat));
  if (l2)
    rla::launch_bn_finalize64(part.data_ptr<double>(), (int)part.size(0), (int)C, count, f32_vec(weight, "weight", C),
                              f32_vec(bias, "bias", C), rm, rv, nbtp, (float)momentum, (float)eps,
                              stats.data_ptr<float>(), cur_stream(part));
  else
    rla::launch_bn_finalize(part.data_ptr<float>(), (int)part.size(0), (int)C, count, f32_vec(weight, "weight", C),
                            f32_vec(bias, "bias", C), rm, rv, nbtp, (float)momentum, (float)eps,
                            stats.data_ptr<float>(), cur_stream(part), nbt_pending ? 1 : 0);
  return stats;
}

Tensor bn_bwd_finalize(Tensor part, double count, optional<Tensor> weight, Tensor mean, Tensor invstd) {
  const bool l2 = part.scalar_type() == at::kDouble;
  check_dev(part, "partials", l2 ? at::kDouble : at::kFloat);
  TORCH_CHECK(part.dim() == 3 && part.size(1) == 2, "partials must be [blocks, 2, C]");
  const int64_t C = part.size(2);
  check_dev(mean, "mean", at::kFloat);
  check_dev(invstd, "invstd", at::kFloat);
  TORCH_CHECK(mean.numel() == C && invstd.numel() == C, "mean / invstd must have C elements");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(part.device());
  Tensor coef = at::empty({5, C}, part.options().dtype(at::kFloat));
  if (l2)
    rla::launch_bn_bwd_finalize64(part.data_ptr<double>(), (int)part.size(0), (int)C, count,
                                  f32_vec(weight, "weight", C), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                  coef.data_ptr<float>(), cur_stream(part));
  else
    rla::launch_bn_bwd_finalize(part.data_ptr<float>(), (int)part.size(0), (int)C, count,
                                f32_vec(weight, "weight", C), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                                coef.data_ptr<float>(), cur_stream(part));
  return coef;
}

// x: [N, H, W, C] bf16 (NHWC view of a channels_last tensor); returns (y, argmax bytes)
std::vector<Tensor> maxpool_fwd(Tensor x, int64_t k, int64_t s, int64_t pad, c10::optional<Tensor> bn_ss,
                                c10::optional<Tensor> nbt_inc) {
  check_dev(x, "x", at::kBFloat16);
  const float* ss = nullptr;
  int64_t* nbt = nullptr;
  if (bn_ss.has_value() && bn_ss->defined()) {
    check_dev(*bn_ss, "bn_ss", at::kFloat);
    TORCH_CHECK(bn_ss->is_contiguous() && bn_ss->numel() == 4 * x.size(3), "maxpool: bn_ss must be [4, C]");
    ss = bn_ss->data_ptr<float>();
  }
  if (nbt_inc.has_value() && nbt_inc->defined()) {
    TORCH_CHECK(nbt_inc->is_cuda() && nbt_inc->scalar_type() == at::kLong, "maxpool: nbt_inc int64 on the GPU");
    nbt = nbt_inc->data_ptr<int64_t>();
  }
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "maxpool: x must be a contiguous NHWC [N, H, W, C] view");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && k >= 1 && s >= 1 && pad >= 0 && 2 * pad <= k, "maxpool: unsupported geometry");
  const int64_t OH = (H + 2 * pad - k) / s + 1, OW = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "maxpool: empty output");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty({N, OH, OW, C}, x.options());
  Tensor arg = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  TORCH_CHECK(rla::launch_maxpool_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                      reinterpret_cast<uint16_t*>(y.data_ptr()), arg.data_ptr<uint8_t>(), (int)N, (int)H,
                                      (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)pad, cur_stream(x), ss,
                                      nbt) == 0,
              "maxpool forward launch failed");
  return {y, arg};
}

// dy [N, C] bf16 -> dx [N, HW, C] bf16 (NHWC rows of a channels_last tensor)
Tensor gap_bwd(Tensor dy, int64_t HW) {
  check_dev(dy, "dy", at::kBFloat16);
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous() && dy.size(1) % 8 == 0 && HW > 0, "gap_bwd: dy [N, C], C % 8 == 0");
  const int64_t N = dy.size(0), C = dy.size(1);
  const at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx = at::empty({N, HW, C}, dy.options());
  TORCH_CHECK(rla::launch_gap_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()),
                                  reinterpret_cast<uint16_t*>(dx.data_ptr()), (int)N, (int)HW, (int)C,
                                  cur_stream(dy)) == 0,
              "gap backward launch failed");
  return dx;
}

// d [N, C, H, W] channels_last bf16 (in place) += g [N*OH*OW, C] bf16 at every s-th pixel
void strided_add_(Tensor d, Tensor g, int64_t s) {
  TORCH_CHECK(d.is_cuda() && d.scalar_type() == at::kBFloat16, "strided_add_: d must be a bf16 GPU tensor");
  check_dev(g, "g", at::kBFloat16);
  TORCH_CHECK(d.dim() == 4 && d.is_contiguous(at::MemoryFormat::ChannelsLast), "strided_add_: d channels_last [N, C, H, W]");
  const int64_t N = d.size(0), C = d.size(1), H = d.size(2), W = d.size(3);
  TORCH_CHECK(s >= 1 && C % 8 == 0, "strided_add_: C % 8 == 0, s >= 1");
  const int64_t OH = (H - 1) / s + 1, OW = (W - 1) / s + 1;
  TORCH_CHECK(g.is_contiguous() && g.numel() == N * OH * OW * C && g.size(-1) == C, "strided_add_: g [N*OH*OW, C]");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(d.device());
  TORCH_CHECK(rla::launch_strided_add(reinterpret_cast<uint16_t*>(d.data_ptr()),
                                      reinterpret_cast<const uint16_t*>(g.data_ptr()), (int)N, (int)H, (int)W, (int)C,
                                      (int)OH, (int)OW, (int)s, cur_stream(d)) == 0,
              "strided add launch failed");
}

Tensor maxpool_bwd(Tensor dy, Tensor arg, int64_t H, int64_t W, int64_t k, int64_t s, int64_t pad) {
  check_dev(dy, "dy", at::kBFloat16);
  check_dev(arg, "arg", at::kByte);
  TORCH_CHECK(dy.dim() == 4 && dy.is_contiguous() && arg.sizes() == dy.sizes(), "maxpool backward: bad shapes");
  const int64_t N = dy.size(0), OH = dy.size(1), OW = dy.size(2), C = dy.size(3);
  TORCH_CHECK(C % 8 == 0 && OH == (H + 2 * pad - k) / s + 1 && OW == (W + 2 * pad - k) / s + 1,
              "maxpool backward: geometry does not match the forward");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  Tensor dx = at::empty({N, H, W, C}, dy.options());
  TORCH_CHECK(rla::launch_maxpool_bwd(reinterpret_cast<const uint16_t*>(dy.data_ptr()), arg.data_ptr<uint8_t>(),
                                      reinterpret_cast<uint16_t*>(dx.data_ptr()), (int)N, (int)H, (int)W, (int)C,
                                      (int)OH, (int)OW, (int)k, (int)s, (int)pad, cur_stream(dy)) == 0,
              "maxpool backward launch failed");
  return dx;
}

void bn_apply(Tensor x, Tensor scale, Tensor shift, optional<Tensor> res, bool relu, Tensor y,
              optional<Tensor> nbt_inc) {
  const int64_t C = scale.numel();
  const int64_t M = bn_rows(x, "x", C);
  bn_same(x, y, "y", C);
  check_dev(scale, "scale", at::kFloat);
  check_dev(shift, "shift", at::kFloat);
  TORCH_CHECK(shift.numel() == C, "shift must have C elements");
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    bn_same(x, *res, "residual", C);
    rp = reinterpret_cast<const uint16_t*>(res->data_ptr());
  }
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  rla::launch_bn_apply(reinterpret_cast<const uint16_t*>(x.data_ptr()), rp, scale.data_ptr<float>(),
                       shift.data_ptr<float>(), M, (int)C, relu, reinterpret_cast<uint16_t*>(y.data_ptr()),
                       cur_stream(x), ptr_or_null<int64_t>(nbt_inc, "num_batches_tracked", at::kLong, 1));
}

// conv1x1 input gradient + the previous BatchNorm's backward partial (csrc/conv1x1.hip
// BWD): dy1 [M, K], wt [N, K] (the weight transposed), dy2 / yb / xb [M, N]; returns
// (d [M, N] bf16, part [rows, 2, N] fp32 for bn_bwd_finalize)
std::vector<Tensor> conv1x1_bn_bwd(Tensor dy1, Tensor wt, Tensor dy2, Tensor yb, Tensor xb) {
  for (const Tensor* t : {&dy1, &wt, &dy2, &yb, &xb}) {
    check_dev(*t, "conv1x1_bn_bwd operand", at::kBFloat16);
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous() && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "conv1x1_bn_bwd: contiguous 16-byte aligned 2-D operands");
  }
  const int64_t M = dy1.size(0), K = dy1.size(1), N = wt.size(0);
  TORCH_CHECK(wt.size(1) == K, "conv1x1_bn_bwd: wt must be [N, K]");
  for (const Tensor* t : {&dy2, &yb, &xb})
    TORCH_CHECK(t->size(0) == M && t->size(1) == N, "conv1x1_bn_bwd: dy2 / yb / xb must be [M, N]");
  TORCH_CHECK(rla::conv1x1_bn_bwd_ok(M, (int)K, (int)N), "conv1x1_bn_bwd: unsupported shape (K <= 128)");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(dy1.device());
  int rows = 0;
  rla::launch_conv1x1_bn_bwd(nullptr, nullptr, nullptr, M, (int)K, (int)N, nullptr, nullptr, nullptr, nullptr, &rows,
                             cur_stream(dy1));
  Tensor d = at::empty({M, N}, dy1.options());
  Tensor part = at::empty({rows, 2, N}, dy1.options().dtype(at::kFloat));
  auto u = [](const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); };
  rla::launch_conv1x1_bn_bwd(u(dy1), u(wt), reinterpret_cast<uint16_t*>(d.data_ptr()), M, (int)K, (int)N, u(dy2),
                             u(yb), u(xb), part.data_ptr<float>(), &rows, cur_stream(dy1));
  return {d, part};
}

// 1x1 conv forward with BatchNorm partial sums: x [M, K] (NHWC rows), w [N, K], both
// bf16 contiguous; returns (y [M, N] bf16, part [gx, 2, N] fp32 for bn_finalize)
std::vector<Tensor> conv1x1_stats(Tensor x, Tensor w, optional<Tensor> pre_ss, optional<Tensor> nbt_inc) {
  check_dev(x, "x", at::kBFloat16);
  check_dev(w, "w", at::kBFloat16);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.is_contiguous() && w.is_contiguous(),
              "conv1x1_stats: x [M, K] and w [N, K] must be contiguous 2-D");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "conv1x1_stats: w must be [N, K]");
  TORCH_CHECK(rla::conv1x1_stats_ok(M, (int)K, (int)N), "conv1x1_stats: unsupported shape (K % 32, N % 64)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "conv1x1_stats: 16-byte aligned operands");
  const float* pre = nullptr;
  int64_t* nbt = nullptr;
  if (pre_ss.has_value() && pre_ss->defined()) {
    // a deferred BatchNorm + ReLU on x: bn_finalize's [4, K] stats (rows 2 / 3 = scale / shift)
    check_dev(*pre_ss, "pre_ss", at::kFloat);
    TORCH_CHECK(pre_ss->is_contiguous() && pre_ss->dim() == 2 && pre_ss->size(0) == 4 && pre_ss->size(1) == K,
                "conv1x1_stats: pre_ss must be [4, K] contiguous fp32");
    TORCH_CHECK(rla::conv1x1_pre_ok(M, (int)K, (int)N), "conv1x1_stats: pre_ss needs K <= 512");
    pre = pre_ss->data_ptr<float>();
    if (nbt_inc.has_value() && nbt_inc->defined()) {
      check_dev(*nbt_inc, "nbt_inc", at::kLong);
      nbt = nbt_inc->data_ptr<int64_t>();
    }
  }
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const rla::Conv1x1Plan p = rla::conv1x1_stats_plan(M, (int)N);
  Tensor y = at::empty({M, N}, x.options());
  Tensor part = at::empty({p.gx, 2, N}, x.options().dtype(at::kFloat));
  rla::launch_conv1x1_stats(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                            reinterpret_cast<const uint16_t*>(w.data_ptr()), reinterpret_cast<uint16_t*>(y.data_ptr()),
                            M, (int)K, (int)N, p, part.data_ptr<float>(), cur_stream(x), pre, nbt);
  return {y, part};
}

void bn_bwd_apply(Tensor x, optional<Tensor> y, Tensor dy, Tensor coef, bool relu, Tensor dx,
                  optional<Tensor> dres, optional<Tensor> dy2, optional<Tensor> ss, optional<Tensor> pool_arg,
                  std::vector<int64_t> pool_geo) {
  check_dev(coef, "coef", at::kFloat);
  TORCH_CHECK(coef.dim() == 2 && coef.size(0) == 5, "coef must be [5, C]");
  const int64_t C = coef.size(1);
  const int64_t M = bn_rows(x, "x", C);
  rla::PoolGrad pg{};
  const bool pooled = pool_grad(x, pool_arg, dy, pool_geo, C, &pg);
  TORCH_CHECK(!pooled || (relu && ss.has_value() && ss->defined() && !(dres.has_value() && dres->defined()) &&
                          !(dy2.has_value() && dy2->defined())),
              "pooled BN backward: ReLU with the forward stats only");
  if (!pooled) bn_same(x, dy, "dy", C);
  bn_same(x, dx, "dx", C);
  const uint16_t* yp = nullptr;
  const float* ssp = relu ? bn_ss(ss, C) : nullptr;
  if (relu && !ssp) {
    TORCH_CHECK(y.has_value(), "ReLU backward needs the saved output y (or the forward stats)");
    bn_same(x, *y, "y", C);
    yp = reinterpret_cast<const uint16_t*>(y->data_ptr());
  }
  uint16_t* drp = nullptr;
  if (dres.has_value() && dres->defined()) {
    bn_same(x, *dres, "dres", C);
    drp = reinterpret_cast<uint16_t*>(dres->data_ptr());
  }
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  rla::launch_bn_bwd_apply(reinterpret_cast<const uint16_t*>(x.data_ptr()), yp,
                           reinterpret_cast<const uint16_t*>(dy.data_ptr()), coef.data_ptr<float>(), M, (int)C,
                           relu, reinterpret_cast<uint16_t*>(dx.data_ptr()), drp, cur_stream(x), bn_dy2(x, dy2, C),
                           ssp, pooled ? &pg : nullptr);
}

// dW of an NHWC bf16 convolution (csrc/conv_wgrad.hip): dy [N, OH, OW, Cout] and
// x [N, H, W, Cin] as contiguous NHWC memory; returns fp32 [Cout, KH, KW, Cin]
// (the channels_last weight's memory order).
Tensor conv_wgrad(Tensor dy, Tensor x, int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t OH, int64_t OW,
                  int64_t Cout, int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                  int64_t splits, int64_t algo, optional<Tensor> pre_ss) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda(), "conv_wgrad: GPU tensors");
  TORCH_CHECK(algo == 0 || algo == 1, "conv_wgrad: algo 0 (auto) or 1 (generic)");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "conv_wgrad: bf16 inputs");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous(), "conv_wgrad: contiguous NHWC memory");
  TORCH_CHECK(Cout % 64 == 0 && Cin % 64 == 0 && Cout > 0 && Cin > 0, "conv_wgrad: channels must be multiples of 64");
  TORCH_CHECK(N > 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && KH > 0 && KW > 0 && sh > 0 && sw > 0 && ph >= 0 &&
                  pw >= 0, "conv_wgrad: bad geometry");
  TORCH_CHECK((H + 2 * ph - KH) / sh + 1 == OH && (W + 2 * pw - KW) / sw + 1 == OW, "conv_wgrad: output size mismatch");
  TORCH_CHECK(dy.numel() == N * OH * OW * Cout, "conv_wgrad: dy has ", dy.numel(), " elements");
  TORCH_CHECK(x.numel() == N * H * W * Cin, "conv_wgrad: x has ", x.numel(), " elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "conv_wgrad: 16-byte aligned inputs");
  TORCH_CHECK(N * std::max(OH * OW, H * W) < (int64_t(1) << 31) / 4, "conv_wgrad: too many rows");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  rla::WgradGeom g{(int)N, (int)H, (int)W, (int)Cin, (int)OH, (int)OW, (int)Cout, (int)KH, (int)KW,
                   (int)sh, (int)sw, (int)ph, (int)pw};
  const rla::WgradPlan plan = rla::wgrad_plan(g, (int)splits, (int)algo);
  const float* pre = nullptr;
  if (pre_ss.has_value() && pre_ss->defined()) {
    // x is a deferred BatchNorm + ReLU's input: the generic kernel stages the activation
    check_dev(*pre_ss, "pre_ss", at::kFloat);
    TORCH_CHECK(pre_ss->is_contiguous() && pre_ss->dim() == 2 && pre_ss->size(0) == 4 && pre_ss->size(1) == Cin,
                "conv_wgrad: pre_ss must be [4, Cin] contiguous fp32");
    TORCH_CHECK(Cin <= 4096, "conv_wgrad: pre_ss with Cin <= 4096");
    pre = pre_ss->data_ptr<float>();
  }
  Tensor out = at::empty({Cout, KH, KW, Cin}, x.options().dtype(at::kFloat));
  Tensor part;
  if (plan.splits > 1) part = at::empty({(int64_t)plan.splits * Cout * KH * KW * Cin}, out.options());
  rla::launch_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                    out.data_ptr<float>(), plan.splits > 1 ? part.data_ptr<float>() : nullptr, g, plan, cur_stream(x),
                    pre);
  return out;
}

std::vector<int64_t> conv_wgrad_plan(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t OH, int64_t OW,
                                     int64_t Cout, int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t ph,
                                     int64_t pw, int64_t splits, int64_t algo) {
  rla::WgradGeom g{(int)N, (int)H, (int)W, (int)Cin, (int)OH, (int)OW, (int)Cout, (int)KH, (int)KW,
                   (int)sh, (int)sw, (int)ph, (int)pw};
  const rla::WgradPlan p = rla::wgrad_plan(g, (int)splits, (int)algo);
  return {p.kind, p.wa, p.wb, p.splits, p.rows_per_split};
}

// 3x3 / stride 1 / pad 1 NHWC bf16 convolution (csrc/conv3x3.hip): x [N, H, W, Cin]
// and w [Cout, 3, 3, Cin] as contiguous memory; returns y as contiguous [N, H, W, Cout].
// flip: the input gradient -- x = dy, w = the forward weight [Cin][3][3][Cout]
// stats: also the next BatchNorm's partial sums of bf16(y) -> {y, part [rows, 2, Cout]}
std::vector<Tensor> conv3x3_impl(Tensor x, Tensor w, int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                 bool flip, bool stats, optional<Tensor> pre_ss = {},
                                 optional<Tensor> nbt_inc = {}) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda(), "conv3x3: GPU tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "conv3x3: bf16 inputs");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "conv3x3: contiguous NHWC / [Cout,3,3,Cin] memory");
  TORCH_CHECK(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0, "conv3x3: bad geometry");
  TORCH_CHECK(x.numel() == N * H * W * Cin, "conv3x3: x has ", x.numel(), " elements");
  TORCH_CHECK(w.numel() == Cout * 9 * Cin, "conv3x3: w has ", w.numel(), " elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "conv3x3: 16-byte aligned inputs");
  TORCH_CHECK(N * (H + 2) * (W + 2) < (int64_t(1) << 30), "conv3x3: too many pixels");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  rla::Conv3x3Geom g{(int)N, (int)H, (int)W, (int)Cin, (int)Cout, 0,
                     rla::conv3x3_pick_tm((int)N, (int)H, (int)W, (int)Cout),
                     rla::conv3x3_wpb((int)N, (int)H, (int)W, (int)Cout)};
  static std::map<std::tuple<int64_t, int64_t, int64_t, int, int>, int> vrows_cache;
  static std::mutex mu;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_tuple(N, H, W, g.tm, g.wpb);
    auto it = vrows_cache.find(key);
    if (it == vrows_cache.end()) it = vrows_cache.emplace(key, rla::conv3x3_vrows(g)).first;
    g.vrows = it->second;
  }
  TORCH_CHECK(rla::conv3x3_ok(g), "conv3x3: unsupported shape (Cin % 16, Cout % 64, halo tile size)");
  TORCH_CHECK(!(flip && stats), "conv3x3: statistics are a forward epilogue");
  const float* pre = nullptr;
  int64_t* nbt = nullptr;
  if (pre_ss.has_value() && pre_ss->defined()) {
    // a deferred BatchNorm + ReLU on x (the statistics forward only)
    check_dev(*pre_ss, "pre_ss", at::kFloat);
    TORCH_CHECK(stats && pre_ss->is_contiguous() && pre_ss->dim() == 2 && pre_ss->size(0) == 4 &&
                    pre_ss->size(1) == Cin && rla::conv3x3_pre_ok(g),
                "conv3x3: pre_ss must be [4, Cin] fp32 (Cin <= 512) on the statistics forward");
    pre = pre_ss->data_ptr<float>();
    if (nbt_inc.has_value() && nbt_inc->defined()) {
      check_dev(*nbt_inc, "nbt_inc", at::kLong);
      nbt = nbt_inc->data_ptr<int64_t>();
    }
  }
  Tensor y = at::empty({N, H, W, Cout}, x.options());
  Tensor part;
  if (stats) part = at::empty({g.wpb, 2, Cout}, x.options().dtype(at::kFloat));
  TORCH_CHECK(rla::launch_conv3x3(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                  reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                  reinterpret_cast<uint16_t*>(y.data_ptr()), g, flip, cur_stream(x),
                                  stats ? part.data_ptr<float>() : nullptr, pre, nbt),
              "conv3x3: launch refused");
  if (stats) return {y, part};
  return {y};
}

Tensor conv3x3(Tensor x, Tensor w, int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout, bool flip) {
  return conv3x3_impl(x, w, N, H, W, Cin, Cout, flip, false)[0];
}

std::vector<Tensor> conv3x3_stats(Tensor x, Tensor w, int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout,
                                  optional<Tensor> pre_ss, optional<Tensor> nbt_inc) {
  return conv3x3_impl(x, w, N, H, W, Cin, Cout, false, true, pre_ss, nbt_inc);
}

// ResNet stem forward: x [N, H, W, 3] NHWC bf16, w [64, 7, 7, 3] bf16 -> {y [N, OH, OW, 64]} or, with
// stats, {y, part [rows, 2, 64]} (the next BatchNorm's partial sums of bf16(y))
std::vector<Tensor> stem_fwd(Tensor x, Tensor w, bool stats) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda(), "stem: GPU tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "stem: bf16 inputs");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 3 && x.is_contiguous(), "stem: x must be contiguous [N, H, W, 3]");
  TORCH_CHECK(w.numel() == 64 * 147 && w.is_contiguous(), "stem: w must be contiguous [64, 7, 7, 3]");
  const rla::StemGeom g{(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)((x.size(1) - 1) / 2 + 1),
                        (int)((x.size(2) - 1) / 2 + 1)};
  TORCH_CHECK(rla::stem_ok(g), "stem: unsupported shape (W even, W <= 256)");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = at::empty({g.N, g.OH, g.OW, 64}, x.options());
  Tensor part;
  if (stats) part = at::empty({rla::stem_grid(g), 2, 64}, x.options().dtype(at::kFloat));
  TORCH_CHECK(rla::launch_stem_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                   reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                   reinterpret_cast<uint16_t*>(y.data_ptr()), stats ? part.data_ptr<float>() : nullptr,
                                   g, cur_stream(x)),
              "stem: launch refused");
  if (stats) return {y, part};
  return {y};
}

// ResNet stem weight gradient: x [N, H, W, 3], dy [N, OH, OW, 64] (NHWC bf16) -> fp32 [64, 7, 7, 3]
Tensor stem_wgrad(Tensor x, Tensor dy) {
  TORCH_CHECK(x.is_cuda() && dy.is_cuda(), "stem_wgrad: GPU tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16, "stem_wgrad: bf16 inputs");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 3 && x.is_contiguous(), "stem_wgrad: x must be contiguous [N, H, W, 3]");
  const rla::StemGeom g{(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)((x.size(1) - 1) / 2 + 1),
                        (int)((x.size(2) - 1) / 2 + 1)};
  TORCH_CHECK(rla::stem_ok(g), "stem_wgrad: unsupported shape");
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == g.N && dy.size(1) == g.OH && dy.size(2) == g.OW && dy.size(3) == 64 &&
                  dy.is_contiguous(),
              "stem_wgrad: dy must be contiguous [N, OH, OW, 64]");
  const at::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor part = at::empty({rla::stem_grid(g), 64, 224}, x.options().dtype(at::kFloat));
  Tensor dw = at::empty({64, 7, 7, 3}, x.options().dtype(at::kFloat));
  TORCH_CHECK(rla::launch_stem_wgrad(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                     reinterpret_cast<const uint16_t*>(dy.data_ptr()), part.data_ptr<float>(),
                                     dw.data_ptr<float>(), g, cur_stream(x)),
              "stem_wgrad: launch refused");
  return dw;
}

bool stem_supported(int64_t N, int64_t H, int64_t W) {
  const rla::StemGeom g{(int)N, (int)H, (int)W, (int)((H - 1) / 2 + 1), (int)((W - 1) / 2 + 1)};
  return rla::stem_ok(g);
}

bool conv3x3_supported(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout) {
  if (N <= 0 || H <= 0 || W <= 0 || Cout <= 0 || N * (H + 2) * (W + 2) >= (int64_t(1) << 30)) return false;
  rla::Conv3x3Geom g{(int)N, (int)H, (int)W, (int)Cin, (int)Cout, 0,
                     rla::conv3x3_pick_tm((int)N, (int)H, (int)W, (int)Cout),
                     rla::conv3x3_wpb((int)N, (int)H, (int)W, (int)Cout)};
  g.vrows = rla::conv3x3_vrows(g);
  return rla::conv3x3_ok(g);
}

Tensor dp_pack_roundtrip(Tensor x, int64_t tag) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "x: contiguous fp32 on the GPU");
  Tensor y = at::empty_like(x);
  TORCH_CHECK(rla::dp_pack_roundtrip(x.data_ptr<float>(), y.data_ptr<float>(), x.numel(), (int)tag, cur_stream(x)) == 0,
              "dp_pack_roundtrip: bad arguments");
  return y;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels of ray_lightning_accelerators_amd";
  m.def("adam_step", &adam_step, "fused Adam over a flat fp32 arena");
  m.def("sgd_step", &sgd_step, "fused SGD (momentum/nesterov/wd) over a flat fp32 arena");
  m.def("multi_copy", &multi_copy, "multi-tensor copy/scale/cast via a chunk table");
  m.def("scale_", &scale_, "in-place scale of an fp32 arena");
  m.def("sumsq", &sumsq, "sum of squares of an fp32 arena");
  m.def("mlp_train_step", &mlp_train_step, "fused MNIST-MLP forward+backward(+Adam) step",
        py::arg("x_u8"), py::arg("x_f32"), py::arg("labels"), py::arg("order"), py::arg("counters"),
        py::arg("n_batches"), py::arg("B"), py::arg("L1"), py::arg("L2"), py::arg("params"),
        py::arg("grads"), py::arg("exp_avg"), py::arg("exp_avg_sq"), py::arg("stats"),
        py::arg("accumulate_grad"), py::arg("apply_adam"), py::arg("advance_step"), py::arg("lr"),
        py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"), py::arg("lr_t"),
        py::arg("adamw"), py::arg("stamps") = py::none());
  m.def("mlp_eval", &mlp_eval, "fused MNIST-MLP forward + NLL/accuracy");
  m.def("mlp3", &mlp3, "fused MNIST-MLP step v3 (pipelined layer 1): kind 0 step, 1 head, 2 tail-grad, "
        "3 tail-adam, 4 prime, 5 step with the in-kernel xGMI exchange, 6 one-launch step (B <= 32)");
  m.def("dp_pack_roundtrip", &dp_pack_roundtrip, "packed DP exchange wire form of fp32 pairs, encoded + decoded");
  m.def("mlp3_hand_words", [](int64_t l1, int64_t l2) { return rla::mlp3_hand_words((int)l1, (int)l2); });
  m.def("mlp3_h1_copies", [](int64_t l1) { return rla::mlp3_h1_copies((int)l1); },
        "H1pre copies per ring slot of the v3 step (the layer-1 partials' atomic fan-in is split over them)");
  m.def("mlp3_dp_area_floats", []() { return rla::comm::kDpUnitAreaFloats; },
        "aux receive-area stride (floats) of the one-launch step's packed / owner protocols");
  m.def("mlp_adam", &mlp_adam, "MLP arena Adam + bf16 shadow refresh (update=False: refresh only)");
  m.def("mlp_shadow_size", [](int64_t l1, int64_t l2) { return rla::mlp_shadow_layout((int)l1, (int)l2).total; });
  m.def("mlp_supported", [](int64_t a, int64_t b) { return rla::mlp_supported((int)a, (int)b); });
  m.def("mlp_param_count", &mlp_param_count);
  m.def("bn_partial", &bn_partial, "fused BN: per-block partial sums (mode 0 fwd stats, 1 bwd dz/dz*x)",
        py::arg("x"), py::arg("y"), py::arg("dy"), py::arg("C"), py::arg("mode"), py::arg("relu"), py::arg("nbt"),
        py::arg("dy2") = py::none(), py::arg("ss") = py::none(), py::arg("dout") = py::none(),
        py::arg("pool_arg") = py::none(), py::arg("pool_geo") = std::vector<int64_t>{});
  m.def("bn_finalize", &bn_finalize, "fused BN: mean/invstd/scale/shift + running stats from partials",
        py::arg("part"), py::arg("count"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("nbt"), py::arg("momentum"), py::arg("eps"), py::arg("nbt_pending") = false);
  m.def("bn_bwd_finalize", &bn_bwd_finalize, "fused BN backward: dgamma/dbeta + dx coefficients");
  m.def("bn_apply", &bn_apply, "fused BN apply: y = act(x*scale + shift (+res))", py::arg("x"), py::arg("scale"),
        py::arg("shift"), py::arg("res"), py::arg("relu"), py::arg("y"), py::arg("nbt_inc") = py::none());
  m.def("conv1x1_stats", &conv1x1_stats, "1x1 conv forward on MFMA + BatchNorm partial sums of its output",
        py::arg("x"), py::arg("w"), py::arg("pre_ss") = py::none(), py::arg("nbt_inc") = py::none());
  m.def("conv1x1_pre_ok", [](int64_t M, int64_t K, int64_t N) { return rla::conv1x1_pre_ok(M, (int)K, (int)N); });
  m.def("conv1x1_bn_bwd", &conv1x1_bn_bwd,
        "1x1 conv input gradient fused with the previous BatchNorm's backward partial -> (d, part)");
  m.def("conv1x1_bn_bwd_ok", [](int64_t M, int64_t K, int64_t N) { return rla::conv1x1_bn_bwd_ok(M, (int)K, (int)N); });
  m.def("conv1x1_stats_ok", [](int64_t M, int64_t K, int64_t N) { return rla::conv1x1_stats_ok(M, (int)K, (int)N); });
  m.def("maxpool_fwd", &maxpool_fwd,
        "NHWC bf16 max pool -> (y, one-byte window argmax); bn_ss: pool bf16(relu(x * scale + shift)) instead",
        py::arg("x"), py::arg("k"), py::arg("s"), py::arg("pad"), py::arg("bn_ss") = py::none(),
        py::arg("nbt_inc") = py::none());
  m.def("strided_add_", &strided_add_, "d[:, :, ::s, ::s] += g in place over NHWC bf16 rows (fp32 add)");
  m.def("gap_bwd", &gap_bwd, "global average pool backward over NHWC rows (16-byte stores)");
  m.def("maxpool_bwd", &maxpool_bwd, "NHWC bf16 max pool backward (gather through the argmax bytes)");
  m.def("bn_bwd_apply", &bn_bwd_apply, "fused BN backward apply: dx (+ dres = relu-masked dy)", py::arg("x"),
        py::arg("y"), py::arg("dy"), py::arg("coef"), py::arg("relu"), py::arg("dx"), py::arg("dres"),
        py::arg("dy2") = py::none(), py::arg("ss") = py::none(), py::arg("pool_arg") = py::none(),
        py::arg("pool_geo") = std::vector<int64_t>{});
  m.def("conv_wgrad", &conv_wgrad, "NHWC bf16 conv weight gradient on MFMA -> fp32 [Cout, KH, KW, Cin]",
        py::arg("dy"), py::arg("x"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("OH"),
        py::arg("OW"), py::arg("Cout"), py::arg("KH"), py::arg("KW"), py::arg("sh"), py::arg("sw"), py::arg("ph"),
        py::arg("pw"), py::arg("splits") = 0, py::arg("algo") = 0, py::arg("pre_ss") = py::none());
  m.def("conv_wgrad_plan", &conv_wgrad_plan, "the wgrad kernel's (kind, wa, wb, splits, rows_per_split)",
        py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("OH"), py::arg("OW"), py::arg("Cout"),
        py::arg("KH"), py::arg("KW"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("splits") = 0, py::arg("algo") = 0);
  m.def("conv3x3", &conv3x3, "3x3 / stride 1 / pad 1 NHWC bf16 convolution on MFMA -> [N, H, W, Cout]",
        py::arg("x"), py::arg("w"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"),
        py::arg("flip") = false);
  m.def("conv3x3_stats", &conv3x3_stats,
        "3x3 / stride 1 / pad 1 forward + BatchNorm partial sums of its bf16 output -> (y, part [rows, 2, Cout])",
        py::arg("x"), py::arg("w"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"),
        py::arg("pre_ss") = py::none(), py::arg("nbt_inc") = py::none());
  m.def("conv3x3_supported", &conv3x3_supported, "shapes the 3x3 MFMA convolution covers");
  m.def("stem_fwd", &stem_fwd, "ResNet stem 7x7/s2 conv (3 -> 64) on MFMA [+ BatchNorm partial sums]");
  m.def("stem_supported", &stem_supported, "input shapes the stem kernel covers");
  m.def("stem_wgrad", &stem_wgrad, "ResNet stem weight gradient on MFMA -> fp32 [64, 7, 7, 3] (channels_last order)");
  m.attr("ARCH") = "gfx950";
}
