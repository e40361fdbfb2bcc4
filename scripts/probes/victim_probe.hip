// Cross-process device-memory corruption detector (diagnostic, not part of the build).
//
// A "victim" process that keeps taking FRESH device memory from the driver (new
// hipMalloc chunks, the oldest released as it goes, so physical pages churn), fills it
// with a byte pattern and checks it on the device every `period_ms`.  Any changed byte
// was written by something that does not own that memory -- another process with a
// stale mapping of pages this process now owns.  Run it beside the multi-process GPU
// tests; each detection prints one JSON line with the wall time, so it can be matched
// against the test that was running.
//
//   ./victim_probe <seconds> [chunk_mb=256] [chunks=16] [period_ms=100]
// Build: hipcc --offload-arch=gfx950 -O2 scripts/probes/victim_probe.hip -o build/victim_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <thread>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

constexpr unsigned kPattern = 0x5A5A5A5Au;

// first changed word (index) and the count of changed words, per chunk
__global__ void scan_kernel(const unsigned* p, long n, unsigned long long* count, long long* first) {
  unsigned long long c = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    if (p[i] != kPattern) {
      ++c;
      atomicMin(reinterpret_cast<unsigned long long*>(first), (unsigned long long)i);
    }
  }
  if (c) atomicAdd(count, c);
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? std::atof(argv[1]) : 60.0;
  const long chunk = (argc > 2 ? std::atol(argv[2]) : 256) << 20;
  const int nchunks = argc > 3 ? std::atoi(argv[3]) : 16;
  const int period_ms = argc > 4 ? std::atoi(argv[4]) : 100;
  const long n = chunk / 4;
  std::deque<unsigned*> held;
  unsigned long long* cnt;
  long long* first;
  CK(hipMalloc(&cnt, 8));
  CK(hipMalloc(&first, 8));
  const double t_end = now_s() + seconds;
  long checks = 0, allocs = 0, hits = 0;
  double next_beat = 0.0;
  std::vector<unsigned> win(16);
  while (now_s() < t_end) {
    // churn: release the oldest chunk, take a fresh one (new physical pages)
    if ((int)held.size() >= nchunks) {
      CK(hipFree(held.front()));
      held.pop_front();
    }
    unsigned* p = nullptr;
    if (hipMalloc(&p, chunk) == hipSuccess) {
      CK(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(p), kPattern, n));
      held.push_back(p);
      ++allocs;
    }
    CK(hipDeviceSynchronize());
    for (size_t k = 0; k < held.size(); ++k) {
      unsigned long long c = 0;
      long long f = 0x7fffffffffffffffLL;
      CK(hipMemcpy(cnt, &c, 8, hipMemcpyHostToDevice));
      CK(hipMemcpy(first, &f, 8, hipMemcpyHostToDevice));
      hipLaunchKernelGGL(scan_kernel, dim3(1024), dim3(256), 0, 0, held[k], n, cnt, first);
      CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&f, first, 8, hipMemcpyDeviceToHost));
      ++checks;
      if (c) {
        ++hits;
        const long w0 = f - f % 4;
        CK(hipMemcpy(win.data(), held[k] + w0, 64, hipMemcpyDeviceToHost));
        std::printf("{\"t\": %.3f, \"chunk\": %zu, \"addr\": \"%p\", \"changed_words\": %llu, \"first_word\": %lld, "
                    "\"words\": [", now_s(), k, (void*)held[k], c, f);
        for (int i = 0; i < 16; ++i) std::printf("%s\"%08x\"", i ? "," : "", win[i]);
        std::printf("]}\n");
        std::fflush(stdout);
        // re-arm the chunk so one event is reported once
        CK(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(held[k]), kPattern, n));
        CK(hipDeviceSynchronize());
      }
    }
    if (now_s() >= next_beat) {  // heartbeat every 10 s (the run's liveness signal)
      next_beat = now_s() + 10.0;
      std::printf("{\"heartbeat\": %.3f, \"checks\": %ld, \"hits\": %ld}\n", now_s(), checks, hits);
      std::fflush(stdout);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(period_ms));
  }
  for (auto p : held) hipFree(p);
  std::printf("{\"summary\": true, \"t\": %.3f, \"checks\": %ld, \"allocs\": %ld, \"hits\": %ld}\n", now_s(), checks,
              allocs, hits);
  return 0;
}
