// Flat-arena optimizer and gradient-bucket kernels for gfx950.
//
// Parameters, gradients and optimizer state of a whole model live in a few
// contiguous fp32 arenas (see parallel/arena.py), so one optimizer step is ONE
// launch over the arena instead of a multi-tensor-apply over hundreds of
// tensors.  The same arena slices are the DDP gradient buckets, so the only
// per-step bucket work left is the averaging scale (fused into the optimizer
// via `grad_scale`) and optional bf16 compression (`multi_copy` below).
//
// Reference parity: these replace the upstream torch.optim.Adam / SGD steps
// used by the reference workloads (tests/utils.py:74 of
// the reference uses SGD, the Ray Tune MNIST example uses Adam) and the DDP
// reducer's flatten/unflatten copies.
#include "common.h"
#include "kernels.h"
#include <math.h>

namespace rla {

constexpr int kOptThreads = 256;

__device__ __forceinline__ void adam_scalars(const AdamArgs& a, float* s_lr, float* s_step_size,
                                             float* s_bc2_sqrt) {
  if (threadIdx.x == 0) {
    const int64_t t = a.step_ptr ? a.step_ptr[0] : a.host_step;
    const float lr = a.lr_ptr ? a.lr_ptr[0] : a.lr;
    const double bc1 = 1.0 - pow((double)a.beta1, (double)t);
    const double bc2 = 1.0 - pow((double)a.beta2, (double)t);
    *s_lr = lr;
    *s_step_size = (float)((double)lr / bc1);
    *s_bc2_sqrt = (float)sqrt(bc2);
  }
  __syncthreads();
}

__device__ __forceinline__ float adam_elem(float p, float g, float& m, float& v, float lr,
                                           float step_size, float bc2_sqrt, const AdamArgs& a) {
  if (a.maximize) g = -g;
  if (a.weight_decay != 0.f) {
    if (a.adamw) p = p * (1.f - lr * a.weight_decay);
    else g = g + a.weight_decay * p;
  }
  // exp_avg.lerp_(grad, 1 - beta1)  (weight < 0.5 branch of ATen's lerp)
  m = m + (1.f - a.beta1) * (g - m);
  v = v * a.beta2 + (1.f - a.beta2) * (g * g);
  const float denom = sqrtf(v) / bc2_sqrt + a.eps;
  return p + (-step_size) * (m / denom);
}

__global__ __launch_bounds__(kOptThreads) void adam_kernel(AdamArgs a) {
  __shared__ float s_lr, s_step_size, s_bc2_sqrt;
  adam_scalars(a, &s_lr, &s_step_size, &s_bc2_sqrt);
  const float lr = s_lr, step_size = s_step_size, bc2_sqrt = s_bc2_sqrt;
  const int64_t n4 = a.n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  F4* p4 = reinterpret_cast<F4*>(a.p);
  const F4* g4 = reinterpret_cast<const F4*>(a.g);
  F4* m4 = reinterpret_cast<F4*>(a.m);
  F4* v4 = reinterpret_cast<F4*>(a.v);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    F4 p = p4[i], m = m4[i], v = v4[i];
    const F4 g = g4[i];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      p.v[k] = adam_elem(p.v[k], g.v[k] * a.grad_scale, m.v[k], v.v[k], lr, step_size, bc2_sqrt, a);
    p4[i] = p; m4[i] = m; v4[i] = v;
    if (a.p_bf16) {
      uint2 packed;
      packed.x = (uint32_t)f2bf_bits(p.v[0]) | ((uint32_t)f2bf_bits(p.v[1]) << 16);
      packed.y = (uint32_t)f2bf_bits(p.v[2]) | ((uint32_t)f2bf_bits(p.v[3]) << 16);
      reinterpret_cast<uint2*>(a.p_bf16)[i] = packed;
    }
  }
  // scalar tail (n % 4 elements), handled by block 0
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < a.n; i += blockDim.x) {
      float m = a.m[i], v = a.v[i];
      const float p = adam_elem(a.p[i], a.g[i] * a.grad_scale, m, v, lr, step_size, bc2_sqrt, a);
      a.p[i] = p; a.m[i] = m; a.v[i] = v;
      if (a.p_bf16) a.p_bf16[i] = f2bf_bits(p);
    }
  }
}

__device__ __forceinline__ float sgd_elem(float p, float g, float& buf, bool first, float lr,
                                          const SGDArgs& a) {
  if (a.maximize) g = -g;
  if (a.weight_decay != 0.f) g = g + a.weight_decay * p;
  if (a.momentum != 0.f) {
    if (first) buf = g;
    else buf = buf * a.momentum + (1.f - a.dampening) * g;
    g = a.nesterov ? g + a.momentum * buf : buf;
  }
  return p + (-lr) * g;
}

__global__ __launch_bounds__(kOptThreads) void sgd_kernel(SGDArgs a) {
  __shared__ float s_lr;
  __shared__ int s_first;
  if (threadIdx.x == 0) {
    const int64_t t = a.step_ptr ? a.step_ptr[0] : a.host_step;
    s_lr = a.lr_ptr ? a.lr_ptr[0] : a.lr;
    s_first = (t <= 1) ? 1 : 0;
  }
  __syncthreads();
  const float lr = s_lr;
  const bool first = s_first != 0;
  const int64_t n4 = a.n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  F4* p4 = reinterpret_cast<F4*>(a.p);
  const F4* g4 = reinterpret_cast<const F4*>(a.g);
  F4* b4 = reinterpret_cast<F4*>(a.buf);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    F4 p = p4[i];
    const F4 g = g4[i];
    F4 b = (a.momentum != 0.f) ? b4[i] : F4{{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int k = 0; k < 4; ++k) p.v[k] = sgd_elem(p.v[k], g.v[k] * a.grad_scale, b.v[k], first, lr, a);
    p4[i] = p;
    if (a.momentum != 0.f) b4[i] = b;
    if (a.p_bf16) {
      uint2 packed;
      packed.x = (uint32_t)f2bf_bits(p.v[0]) | ((uint32_t)f2bf_bits(p.v[1]) << 16);
      packed.y = (uint32_t)f2bf_bits(p.v[2]) | ((uint32_t)f2bf_bits(p.v[3]) << 16);
      reinterpret_cast<uint2*>(a.p_bf16)[i] = packed;
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < a.n; i += blockDim.x) {
      float b = (a.momentum != 0.f) ? a.buf[i] : 0.f;
      const float p = sgd_elem(a.p[i], a.g[i] * a.grad_scale, b, first, lr, a);
      a.p[i] = p;
      if (a.momentum != 0.f) a.buf[i] = b;
      if (a.p_bf16) a.p_bf16[i] = f2bf_bits(p);
    }
  }
}

static int opt_grid(int64_t n) {
  int64_t blocks = ((n >> 2) + kOptThreads - 1) / kOptThreads;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;  // grid-stride beyond 8 blocks/CU x 256 CUs
  return (int)blocks;
}

void launch_adam(const AdamArgs& a, hipStream_t stream) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(adam_kernel, dim3(opt_grid(a.n)), dim3(kOptThreads), 0, stream, a);
}

void launch_sgd(const SGDArgs& a, hipStream_t stream) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(sgd_kernel, dim3(opt_grid(a.n)), dim3(kOptThreads), 0, stream, a);
}

// ---------------------------------------------------------------------------
// Multi-tensor copy / scale / cast (bucket flatten, unflatten, bf16 compress).
//
// `table` holds one 4 x int64 row per chunk: {src_addr, dst_addr, numel, dtypes}
// where dtypes = src_dtype | (dst_dtype << 8), dtype 0 = fp32, 1 = bf16.
// Each workgroup owns one chunk (<= kChunkElems elements), so the grid is the
// chunk count and no tensor-boundary search happens on the device.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float ld_elem(const void* base, int64_t i, int dt) {
  return dt == 0 ? reinterpret_cast<const float*>(base)[i]
                 : bfbits2f(reinterpret_cast<const uint16_t*>(base)[i]);
}
__device__ __forceinline__ void st_elem(void* base, int64_t i, int dt, float v) {
  if (dt == 0) reinterpret_cast<float*>(base)[i] = v;
  else reinterpret_cast<uint16_t*>(base)[i] = f2bf_bits(v);
}

__global__ __launch_bounds__(kOptThreads) void multi_copy_kernel(const int64_t* __restrict__ table,
                                                                 float scale, int accumulate) {
  const int64_t* row = table + (int64_t)blockIdx.x * 4;
  const void* src = reinterpret_cast<const void*>(row[0]);
  void* dst = reinterpret_cast<void*>(row[1]);
  const int64_t n = row[2];
  const int sdt = (int)(row[3] & 0xff), ddt = (int)((row[3] >> 8) & 0xff);
  const bool aligned = ((row[0] | row[1]) & 15) == 0;
  if (sdt == 0 && ddt == 0 && aligned) {
    const int64_t n4 = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
      float4 v = s4[i];
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      if (accumulate) {
        const float4 o = d4[i];
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
      }
      d4[i] = v;
    }
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float v = reinterpret_cast<const float*>(src)[i] * scale;
      if (accumulate) v += reinterpret_cast<float*>(dst)[i];
      reinterpret_cast<float*>(dst)[i] = v;
    }
    return;
  }
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    float v = ld_elem(src, i, sdt) * scale;
    if (accumulate) v += ld_elem(dst, i, ddt);
    st_elem(dst, i, ddt, v);
  }
}

void launch_multi_copy(const int64_t* table, int64_t nchunks, float scale, int accumulate,
                       hipStream_t stream) {
  if (nchunks <= 0) return;
  hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)nchunks), dim3(kOptThreads), 0, stream,
                     table, scale, accumulate);
}

// ---------------------------------------------------------------------------
// Arena-wide helpers: in-place scale (DDP averaging when not fused into the
// optimizer) and sum of squares (gradient clipping / grad-norm logging).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kOptThreads) void scale_kernel(float* x, int64_t n, float s) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float4* x4 = reinterpret_cast<float4*>(x);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = x4[i];
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    x4[i] = v;
  }
  if (blockIdx.x == 0)
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) x[i] *= s;
}

__global__ __launch_bounds__(kOptThreads) void sumsq_kernel(const float* x, int64_t n, float* out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float acc = 0.f;
  const int64_t n4 = n >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = x4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) acc += x[i] * x[i];
  // wave64 reduction
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  __shared__ float part[kOptThreads / kWave];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < kOptThreads / kWave; ++i) s += part[i];
    atomicAdd(out, s);
  }
}

void launch_scale(float* x, int64_t n, float s, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scale_kernel, dim3(opt_grid(n)), dim3(kOptThreads), 0, stream, x, n, s);
}

void launch_sumsq(const float* x, int64_t n, float* out, hipStream_t stream) {
  (void)hipMemsetAsync(out, 0, sizeof(float), stream);
  if (n <= 0) return;
  hipLaunchKernelGGL(sumsq_kernel, dim3(opt_grid(n)), dim3(kOptThreads), 0, stream, x, n, out);
}

}  // namespace rla
