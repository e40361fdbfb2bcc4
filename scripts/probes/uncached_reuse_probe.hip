// Does device memory that was allocated UNCACHED (hipExtMallocWithFlags(...,
// hipDeviceMallocUncached): the communicator's xGMI / aux regions) and freed leave
// anything behind for the next allocation at the same addresses?  (Round-6 diagnostic
// for the intermittent corrupted-fresh-tensor failure, which follows the MNIST DP
// loopback tests -- they create and free such regions -- in the GPU suite.)
//
// Per round: an uncached region U is written and read by a kernel on every XCD and
// freed; then normal allocations of the same and other sizes are made (often landing
// on U's addresses), filled (by a kernel, or by a host-to-device copy), and every word
// is checked twice -- a kernel compares against the expected value, and a device-to-
// host copy is compared on the host.  Any difference means the kernels and the copy
// engine disagree about memory at a re-used address.
//   ./uncached_reuse_probe <seconds> [uncached_mb=8] [mode]
//   mode 0: an uncached U allocated and freed every round; 1: plain hipMalloc U (control);
//   2: one uncached U kept for the whole run (never freed), opened and closed through
//   its IPC handle in this process every round; 3: one uncached U kept, no IPC (the pool);
//   4: no U -- a world-1 RCCL communicator initialised, used once and destroyed every
//   round (does ncclCommDestroy leave the same state behind?)
// Build (mode 4 needs RCCL): ... -lrccl
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probes/uncached_reuse_probe.hip -o build/uncached_reuse_probe
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

__global__ void fill_kernel(unsigned* p, long n, unsigned v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v + (unsigned)i;
}

__global__ void touch_kernel(unsigned* p, long n, unsigned* sink) {
  unsigned acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    acc += p[i];
    p[i] = acc ^ 0xA5A5A5A5u;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void check_kernel(const unsigned* p, long n, unsigned v, unsigned long long* bad) {
  unsigned long long b = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    b += p[i] != v + (unsigned)i;
  if (b) atomicAdd(bad, b);
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? std::atof(argv[1]) : 60.0;
  const long ubytes = (argc > 2 ? std::atol(argv[2]) : 8) << 20;
  const int mode = argc > 3 ? std::atoi(argv[3]) : 0;
  unsigned long long* bad;
  unsigned* sink;
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&sink, 64));
  const double t_end = now_s() + seconds;
  long rounds = 0, checks = 0, reused = 0, kbad_total = 0, hbad_total = 0, bad_checks = 0;
  double beat = now_s() + 10;
  std::vector<unsigned> host;
  unsigned seed = 1;
  void* keep = nullptr;
  if (mode >= 2) CK(hipExtMallocWithFlags(&keep, (size_t)ubytes, hipDeviceMallocUncached));
  long ipc_same = 0;
  while (now_s() < t_end) {
    if (mode == 4) {
      ncclUniqueId id;
      ncclComm_t comm;
      if (ncclGetUniqueId(&id) != ncclSuccess || ncclCommInitRank(&comm, 1, id, 0) != ncclSuccess) {
        std::fprintf(stderr, "rccl init failed\n");
        return 2;
      }
      if (ncclAllReduce(sink, sink, 4, ncclFloat32, ncclSum, comm, 0) != ncclSuccess) return 2;
      CK(hipDeviceSynchronize());
      ncclCommDestroy(comm);
    }
    void* u = keep;
    if (mode == 0)
      CK(hipExtMallocWithFlags(&u, (size_t)ubytes, hipDeviceMallocUncached));
    else if (mode == 1)
      CK(hipMalloc(&u, (size_t)ubytes));
    if (mode != 4) {
      hipLaunchKernelGGL(fill_kernel, dim3(512), dim3(256), 0, 0, (unsigned*)u, ubytes / 4, 7u * seed);
      hipLaunchKernelGGL(touch_kernel, dim3(512), dim3(256), 0, 0, (unsigned*)u, ubytes / 4, sink);
      CK(hipDeviceSynchronize());
    }
    if (mode == 2) {  // the communicator's loopback: its own region through its own IPC handle
      hipIpcMemHandle_t h;
      CK(hipIpcGetMemHandle(&h, u));
      void* v = nullptr;
      CK(hipIpcOpenMemHandle(&v, h, hipIpcMemLazyEnablePeerAccess));
      hipLaunchKernelGGL(touch_kernel, dim3(512), dim3(256), 0, 0, (unsigned*)v, ubytes / 4, sink);
      CK(hipDeviceSynchronize());
      if (v != u) CK(hipIpcCloseMemHandle(v));
      else ++ipc_same;
    }
    if (mode <= 1) CK(hipFree(u));
    // normal allocations: the same size first (most likely at u), then others
    const long sizes[3] = {ubytes, ubytes / 2, ubytes + (1 << 20)};
    std::vector<void*> held;
    for (int k = 0; k < 3; ++k) {
      void* q = nullptr;
      CK(hipMalloc(&q, (size_t)sizes[k]));
      held.push_back(q);
      reused += q == u;
      const long n = sizes[k] / 4;
      const unsigned v = 0x1000u * (++seed);
      if (k == 1) {  // the copy engine writes, kernels check
        host.resize(n);
        for (long i = 0; i < n; ++i) host[i] = v + (unsigned)i;
        CK(hipMemcpy(q, host.data(), sizes[k], hipMemcpyHostToDevice));
      } else {  // a kernel writes, the copy engine reads
        hipLaunchKernelGGL(fill_kernel, dim3(512), dim3(256), 0, 0, (unsigned*)q, n, v);
      }
      CK(hipMemset(bad, 0, 8));
      hipLaunchKernelGGL(check_kernel, dim3(512), dim3(256), 0, 0, (const unsigned*)q, n, v, bad);
      unsigned long long kb = 0;
      CK(hipMemcpy(&kb, bad, 8, hipMemcpyDeviceToHost));
      host.assign(n, 0u);
      CK(hipMemcpy(host.data(), q, sizes[k], hipMemcpyDeviceToHost));
      long hb = 0, first = -1;
      for (long i = 0; i < n; ++i)
        if (host[i] != v + (unsigned)i) {
          if (first < 0) first = i;
          ++hb;
        }
      checks += 1;
      if (kb || hb) {
        if (kbad_total + hbad_total < 64LL * n)  // the first few in full
          std::printf("{\"bad\": true, \"round\": %ld, \"k\": %d, \"reused_addr\": %d, \"kernel_view_bad\": %llu, "
                      "\"copy_view_bad\": %ld, \"ptr\": \"%p\", \"first_bad_word\": %ld, \"got\": \"%08x\", "
                      "\"want\": \"%08x\"}\n",
                      rounds, k, (int)(q == u), kb, hb, q, first, first >= 0 ? host[first] : 0u,
                      first >= 0 ? v + (unsigned)first : 0u);
        std::fflush(stdout);
        kbad_total += (long)kb;
        hbad_total += hb;
        ++bad_checks;
      }
    }
    for (void* q : held) CK(hipFree(q));
    ++rounds;
    if (now_s() > beat) {
      beat = now_s() + 10;
      std::printf("{\"heartbeat\": %ld, \"checks\": %ld, \"reused\": %ld, \"kernel_bad\": %ld, \"copy_bad\": %ld}\n", rounds,
                  checks, reused, kbad_total, hbad_total);
      std::fflush(stdout);
    }
  }
  std::printf("{\"summary\": true, \"mode\": %d, \"rounds\": %ld, \"checks\": %ld, \"bad_checks\": %ld, "
              "\"reused_addresses\": %ld, \"kernel_bad_words\": %ld, \"copy_bad_words\": %ld, \"ipc_same_ptr\": %ld}\n",
              mode, rounds, checks, bad_checks, reused, kbad_total, hbad_total, ipc_same);
  return 0;
}
