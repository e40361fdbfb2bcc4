// Parameter-arena pieces shared by the fused MNIST-MLP step (mlp_step3.hip):
// the bf16 weight-shadow layout and the multi-workgroup Adam over the whole
// arena (+ shadow refresh), used after a host-side gradient allreduce, after a
// parameter load (update = 0: shadow refresh only) and by the fp32 fallback.
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

template <int L1, int L2>
int dispatch_adam(const MLPAdamArgs& a, hipStream_t stream) {
  const int64_t np = Off<L1, L2>::NP;
  int blocks = (int)((np + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL((mlp_adam_kernel<L1, L2>), dim3(blocks), dim3(256), 0, stream, a);
  return 0;
}

#define RLA_MLP_SHAPES(X) \
  X(32, 32) X(32, 64) X(32, 128) X(32, 256) \
  X(64, 64) X(64, 128) X(64, 256) \
  X(128, 128) X(128, 256) X(128, 64)

}  // namespace

int launch_mlp_adam(const MLPAdamArgs& a, hipStream_t stream) {
#define RLA_CASE(a1, a2) if (a.L1 == a1 && a.L2 == a2) return dispatch_adam<a1, a2>(a, stream);
  RLA_MLP_SHAPES(RLA_CASE)
#undef RLA_CASE
  return -1;
}

}  // namespace rla
