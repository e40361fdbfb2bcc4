// Price of the one-launch MNIST step's step boundary: a kernel
// boundary between K graph-replayed launches vs an in-kernel grid barrier of ONE
// persistent launch that loops over the K steps.  Same geometry as
// mlp3_one_kernel<32, 64> (60 workgroups x 512 threads, one per CU), same kind of
// hand-off the step needs across its boundary: every block publishes 256 B
// (the weights / H1pre it produced) and, after the boundary, reads every other
// block's 256 B.  Body: `work_ns` of s_sleep-paced idling per step (the step's
// ~6.5 us of block work), so only the boundary differs between the arms.
//
//   arm "launch":  K launches of step_kernel in one hipGraph (plain stores; the
//                  kernel boundary provides visibility)
//   arm "persist": one launch of persist_kernel, K iterations; barrier = every
//                  block's wave 0 stores its record write-through (sc1), waits its
//                  vmcnt, one lane adds to an arrival counter (agent scope); lane 0
//                  polls the counter with sc1 loads until all blocks of this step
//                  arrived; the records are then read with sc1 loads (no acquire
//                  fence: the guide's write-through + sc1 hand-off form)
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/step_barrier_probe scripts/probes/step_barrier_probe.hip
// Run:   build/step_barrier_probe [K] [work_ns]   (prints one JSON line per arm)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

constexpr int kBlocks = 60, kThreads = 512, kRec = 64;  // 64 floats = 256 B per block

__device__ __forceinline__ void idle_ns(int ns) {
  if (ns <= 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  const uint64_t ticks = (uint64_t)ns / 10;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one step: read every block's record of the previous step, idle, publish ours
__global__ __launch_bounds__(kThreads) void step_kernel(float* rec, int work_ns, float* sink) {
  const int tid = threadIdx.x, b = blockIdx.x;
  float acc = 0.f;
  if (tid < kRec)
    for (int j = 0; j < kBlocks; ++j) acc += rec[j * kRec + tid];
  idle_ns(work_ns);
  __syncthreads();
  if (tid < kRec) rec[b * kRec + tid] = acc * 1e-3f + (float)b;
  if (acc == -1.f) sink[0] = acc;
}

__global__ __launch_bounds__(kThreads) void persist_kernel(float* rec, unsigned* arrive, int K, int work_ns,
                                                           float* sink, int* err) {
  const int tid = threadIdx.x, b = blockIdx.x;
  __shared__ int sh_fail;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) {
    if (tid < kRec)
      for (int j = 0; j < kBlocks; ++j) acc += ld_sc1(rec + (size_t)(k & 1) * kBlocks * kRec + j * kRec + tid);
    idle_ns(work_ns);
    // publish into the other half (step k + 1 reads it; step k's readers still read this half)
    if (tid < kRec) st_sc1(rec + (size_t)((k + 1) & 1) * kBlocks * kRec + b * kRec + tid, acc * 1e-3f + (float)b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      sh_fail = 0;
      __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(k + 1) * kBlocks;
      int64_t spins = 0;
      while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (++spins > (1 << 24)) {  // bounded: every block leaves even if one never arrives
          sh_fail = 1;
          atomicExch(err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    asm volatile("" ::: "memory");
    __syncthreads();
    if (sh_fail) break;
  }
  if (acc == -1.f) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 2000;
  const int work_ns = argc > 2 ? atoi(argv[2]) : 6500;
  float *rec, *sink;
  unsigned* arrive;
  int* err;
  CHECK(hipMalloc(&rec, 2 * kBlocks * kRec * sizeof(float)));
  CHECK(hipMalloc(&sink, sizeof(float)));
  CHECK(hipMalloc(&arrive, sizeof(unsigned)));
  CHECK(hipMalloc(&err, sizeof(int)));
  CHECK(hipMemset(rec, 0, 2 * kBlocks * kRec * sizeof(float)));
  CHECK(hipMemset(err, 0, sizeof(int)));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));

  // arm "launch": G launches per graph, K / G replays
  const int G = K < 20 ? K : 20;
  hipGraph_t graph;
  hipGraphExec_t exec;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < G; ++i) hipLaunchKernelGGL(step_kernel, dim3(kBlocks), dim3(kThreads), 0, s, rec, work_ns, sink);
  CHECK(hipStreamEndCapture(s, &graph));
  CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  for (int w = 0; w < 5; ++w) CHECK(hipGraphLaunch(exec, s));
  CHECK(hipStreamSynchronize(s));
  float best_l = 1e30f, best_p = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < K / G; ++i) CHECK(hipGraphLaunch(exec, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best_l) best_l = ms;
    // arm "persist": one launch of K steps
    CHECK(hipMemsetAsync(arrive, 0, sizeof(unsigned), s));
    CHECK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(persist_kernel, dim3(kBlocks), dim3(kThreads), 0, s, rec, arrive, K, work_ns, sink, err);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best_p) best_p = ms;
  }
  int herr = 0;
  CHECK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
  const int steps_l = K / G * G;
  printf("{\"arm\": \"launch\", \"K\": %d, \"work_ns\": %d, \"us_per_step\": %.3f}\n", steps_l, work_ns,
         best_l * 1e3f / steps_l);
  printf("{\"arm\": \"persist\", \"K\": %d, \"work_ns\": %d, \"us_per_step\": %.3f, \"barrier_timeouts\": %d}\n", K,
         work_ns, best_p * 1e3f / K, herr);
  CHECK(hipGraphExecDestroy(exec));
  CHECK(hipGraphDestroy(graph));
  return herr;
}
