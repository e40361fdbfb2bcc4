// Native self-test of the comm engine, no Python / torch involved (SURVEY.md §5.2
// "debug build of the C++ extension with -fsanitize=address (host side)").
//
// Built by `python -m ray_lightning_accelerators_amd._build --selftest` twice:
// plain, and with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code
// only (`-Xarch_host -fsanitize=...`; device code is never instrumented).  The
// program forks into W ranks BEFORE any HIP call; every rank maps its peers' xGMI
// regions through IPC handles exchanged over a socketpair and drives the real
// kernels and host engines:
//   1. one-shot allreduce (ragged sizes, both slot parities),
//   2. two-shot allreduce, fp32 and bf16 wire (ragged sizes incl. empty chunks),
//   3. fusion engine: 40 requests of random sizes -> batches on the engine
//      thread, pack / allreduce / unpack with the post-scale, drain,
//   4. DDP reducer: 4 buckets over an arena, readiness in reverse order,
//   5. dead peer: one rank skips a collective; the other's bounded poll must
//      set the error word (no hang).
// With one GPU every rank uses device 0 (same protocol; the link is local); on a
// multi-GPU node rank r uses device r % count, i.e. real xGMI.
// Exit status 0 = every rank passed; the sanitizers abort on a host memory error,
// leak (LeakSanitizer) or UB.
#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "comm/communicator.h"
#include "comm/fusion_engine.h"
#include "comm/reducer.h"

using rla::comm::Communicator;
using rla::comm::FusionEngine;
using rla::comm::Reducer;

namespace {

#define CHECK(cond, ...)                                                    \
  do {                                                                      \
    if (!(cond)) {                                                          \
      std::fprintf(stderr, "[rank %d] check failed: %s: ", g_rank, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                                    \
      std::fprintf(stderr, "\n");                                           \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

int g_rank = 0;

void hip_ok(hipError_t e, const char* what) { CHECK(e == hipSuccess, "%s: %s", what, hipGetErrorString(e)); }

// ---- tiny all-to-all channel: a star through rank 0 over socketpairs
struct Channel {
  int rank, world;
  std::vector<int> fds;  // rank 0: fd per peer (index r); others: fds[0] to rank 0

  static void send_all(int fd, const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    while (n) {
      ssize_t k = write(fd, c, n);
      CHECK(k > 0, "socket write");
      c += k;
      n -= (size_t)k;
    }
  }
  static void recv_all(int fd, void* p, size_t n) {
    char* c = static_cast<char*>(p);
    while (n) {
      ssize_t k = read(fd, c, n);
      CHECK(k > 0, "socket read");
      c += k;
      n -= (size_t)k;
    }
  }
  static void send_str(int fd, const std::string& s) {
    uint64_t n = s.size();
    send_all(fd, &n, sizeof(n));
    send_all(fd, s.data(), n);
  }
  static std::string recv_str(int fd) {
    uint64_t n = 0;
    recv_all(fd, &n, sizeof(n));
    std::string s(n, '\0');
    recv_all(fd, &s[0], n);
    return s;
  }
  // every rank contributes one string, every rank gets all of them
  std::vector<std::string> all_gather(const std::string& mine) {
    std::vector<std::string> out(world);
    if (rank == 0) {
      out[0] = mine;
      for (int r = 1; r < world; ++r) out[r] = recv_str(fds[r]);
      for (int r = 1; r < world; ++r)
        for (int k = 0; k < world; ++k) send_str(fds[r], out[k]);
    } else {
      send_str(fds[0], mine);
      for (int k = 0; k < world; ++k) out[k] = recv_str(fds[0]);
    }
    return out;
  }
  void barrier() { all_gather(std::string(1, 'b')); }
};

std::vector<float> pattern(int64_t n, int rank) {
  std::vector<float> v(n);
  for (int64_t i = 0; i < n; ++i) v[i] = (float)(i % 97) * (rank + 1) + rank;
  return v;
}

float expect_at(int64_t i, int world) {
  return (float)(i % 97) * (world * (world + 1) / 2) + (float)(world * (world - 1) / 2);
}

void check_sum(const float* dev, int64_t n, int world, const char* what) {
  std::vector<float> h(n);
  hip_ok(hipMemcpy(h.data(), dev, n * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy D2H");
  for (int64_t i = 0; i < n; ++i)
    CHECK(h[i] == expect_at(i, world), "%s n=%lld: x[%lld]=%g want %g", what, (long long)n, (long long)i, h[i],
          expect_at(i, world));
}

int run_rank(Channel& ch) {
  const int rank = ch.rank, world = ch.world;
  int ndev = 0;
  hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  const int device = rank % (ndev > 0 ? ndev : 1);
  hip_ok(hipSetDevice(device), "hipSetDevice");
  hipStream_t s;
  hip_ok(hipStreamCreate(&s), "hipStreamCreate");

  Communicator comm(rank, world, device);
  comm.set_spin_limit(int64_t(1) << 22);
  const int64_t one_cap = 1 << 16;
  comm.xgmi_open(ch.all_gather(comm.xgmi_handle(one_cap)));
  comm.twoshot_open(ch.all_gather(comm.twoshot_handle(int64_t(1) << 21)));
  CHECK(comm.has_xgmi() && comm.has_twoshot(), "regions not open");

  float* buf = nullptr;
  const int64_t maxn = int64_t(1) << 21;
  hip_ok(hipMalloc(reinterpret_cast<void**>(&buf), maxn * sizeof(float)), "hipMalloc");

  // 1 + 2: one-shot, two-shot fp32, router
  const int64_t sizes[] = {1, 3, 4, 5, 255, 4099, 27882, 65536, 70001, 1000003};
  for (int pass = 0; pass < 2; ++pass) {
    for (int64_t n : sizes) {
      std::vector<float> h = pattern(n, rank);
      hip_ok(hipMemcpy(buf, h.data(), n * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy H2D");
      ch.barrier();
      const int route = comm.route(buf, n);
      CHECK(route == (n <= one_cap ? 0 : 1), "route(%lld)=%d", (long long)n, route);
      if (pass == 0) comm.allreduce_f32(buf, n, s);
      else comm.allreduce_twoshot(buf, n, false, s);  // two-shot for every size too
      hip_ok(hipStreamSynchronize(s), "sync");
      CHECK(comm.error_state() == 0, "error state after n=%lld", (long long)n);
      check_sum(buf, n, world, pass == 0 ? "routed" : "two-shot");
    }
  }
  // bf16 wire: small integers are exact in bf16
  {
    const int64_t n = 300007;
    std::vector<float> h(n, (float)(rank + 1));
    hip_ok(hipMemcpy(buf, h.data(), n * sizeof(float), hipMemcpyHostToDevice), "hipMemcpy H2D");
    CHECK(comm.allreduce_f32_bf16wire(buf, n, s), "bf16 wire refused");
    hip_ok(hipStreamSynchronize(s), "sync");
    hip_ok(hipMemcpy(h.data(), buf, n * sizeof(float), hipMemcpyDeviceToHost), "D2H");
    for (int64_t i = 0; i < n; ++i) CHECK(h[i] == world * (world + 1) / 2.f, "bf16 x[%lld]=%g", (long long)i, h[i]);
  }

  // 3: fusion engine (engine thread, pack kernel, post-scale)
  {
    std::mt19937 rng(1234);  // same sizes on every rank
    std::vector<int64_t> ns;
    int64_t total = 0;
    for (int k = 0; k < 40; ++k) {
      ns.push_back(1 + (int64_t)(rng() % 20000));
      total += (ns.back() + 3) / 4 * 4;
    }
    CHECK(total <= maxn, "fusion test too large");
    std::vector<float> h(total, (float)(rank + 1));
    hip_ok(hipMemcpy(buf, h.data(), total * sizeof(float), hipMemcpyHostToDevice), "H2D");
    FusionEngine eng(&comm, 64 << 10, device);
    std::vector<int64_t> handles;
    int64_t off = 0;
    for (int64_t n : ns) {
      handles.push_back(eng.submit(buf + off, n, 1.0f / world, s));
      off += (n + 3) / 4 * 4;
    }
    eng.flush();
    for (int64_t hd : handles) CHECK(eng.wait(hd, s), "unknown handle");
    eng.drain();
    hip_ok(hipStreamSynchronize(s), "sync");
    CHECK(eng.batches_executed() >= 2, "expected several fusion batches, got %lld", (long long)eng.batches_executed());
    std::vector<uint64_t> fp = {eng.fingerprint()};
    auto fps = ch.all_gather(std::string(reinterpret_cast<char*>(fp.data()), sizeof(uint64_t)));
    for (auto& f : fps) CHECK(f == fps[0], "fusion fingerprints differ across ranks");
    hip_ok(hipMemcpy(h.data(), buf, total * sizeof(float), hipMemcpyDeviceToHost), "D2H");
    off = 0;
    const float want = (world + 1) / 2.f;
    for (int64_t n : ns) {
      for (int64_t i = 0; i < n; ++i) CHECK(std::fabs(h[off + i] - want) < 1e-6f, "fusion value %g", h[off + i]);
      off += (n + 3) / 4 * 4;
    }
  }

  // 4: DDP reducer, 10 params in 4 buckets, readiness back to front
  {
    const int np = 10;
    std::vector<int64_t> poff(np + 1, 0);
    for (int p = 0; p < np; ++p) poff[p + 1] = poff[p] + 4 * (1000 + 3713 * p);
    const int64_t numel = poff[np];
    std::vector<int> pb(np);
    for (int p = 0; p < np; ++p) pb[p] = 3 - p * 4 / np;  // last params -> bucket 0
    std::vector<int64_t> bounds;
    for (int b = 0; b < 4; ++b) {
      int64_t lo = numel, hi = 0;
      for (int p = 0; p < np; ++p)
        if (pb[p] == b) {
          lo = std::min(lo, poff[p]);
          hi = std::max(hi, poff[p + 1]);
        }
      bounds.push_back(lo);
      bounds.push_back(hi);
    }
    std::vector<float> h = pattern(numel, rank);
    Reducer red(&comm, buf, numel, bounds, pb, device);
    for (int step = 0; step < 3; ++step) {
      hip_ok(hipMemcpy(buf, h.data(), numel * sizeof(float), hipMemcpyHostToDevice), "H2D");
      ch.barrier();
      red.prepare();
      for (int p = np - 1; p >= 0; --p) red.mark_ready(p, s);
      red.finish(s);
      hip_ok(hipStreamSynchronize(s), "sync");
      check_sum(buf, numel, world, "reducer");
    }
    CHECK(red.launched() == 12, "reducer launched %lld buckets", (long long)red.launched());
  }

  // 5: dead peer -- rank 1 never joins; rank 0's bounded poll must give up
  ch.barrier();
  comm.set_spin_limit(int64_t(1) << 14);
  if (rank == 0) {
    comm.allreduce_xgmi(buf, 1024, s);
    hip_ok(hipStreamSynchronize(s), "sync");
    CHECK(comm.error_state() == 1, "dead peer not detected (state %d)", comm.error_state());
  }
  ch.barrier();
  if (rank != 0) CHECK(comm.error_state() == 0, "healthy rank reports an error");

  hip_ok(hipFree(buf), "hipFree");
  hip_ok(hipStreamDestroy(s), "hipStreamDestroy");
  std::printf("[rank %d] comm selftest ok (device %d of %d)\n", rank, device, ndev);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "canary") == 0) {
    // proves the sanitizer build is live: a one-element heap overflow that ASan
    // must report (the plain build just exits 0)
    volatile char* p = new char[8];
    p[8] = 1;
    delete[] p;
    return 0;
  }
  const int world = argc > 1 ? std::atoi(argv[1]) : 2;
  if (world < 2 || world > rla::comm::kXgmiMaxRanks) {
    std::fprintf(stderr, "usage: %s [world 2..8]\n", argv[0]);
    return 2;
  }
  // fork every rank BEFORE any HIP call
  std::vector<int> child_fd(world, -1);
  std::vector<pid_t> pids;
  int my_rank = 0, my_fd = -1;
  for (int r = 1; r < world; ++r) {
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 3;
    pid_t pid = fork();
    if (pid < 0) return 3;
    if (pid == 0) {
      close(sv[0]);
      for (int k = 1; k < r; ++k) close(child_fd[k]);
      my_rank = r;
      my_fd = sv[1];
      pids.clear();
      break;
    }
    close(sv[1]);
    child_fd[r] = sv[0];
    pids.push_back(pid);
  }
  g_rank = my_rank;
  Channel ch{my_rank, world, {}};
  if (my_rank == 0) ch.fds = child_fd;
  else ch.fds = {my_fd};
  int rc = run_rank(ch);
  if (my_rank == 0) {
    for (pid_t p : pids) {
      int st = 0;
      waitpid(p, &st, 0);
      if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
    }
    std::printf(rc == 0 ? "comm selftest PASSED (world %d)\n" : "comm selftest FAILED (world %d)\n", world);
  }
  return rc;
}
