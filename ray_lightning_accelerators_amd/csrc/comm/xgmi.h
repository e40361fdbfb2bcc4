// Host-side view of the xGMI one-shot allreduce (csrc/comm/xgmi_allreduce.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rla {
namespace comm {

constexpr int kXgmiMaxRanks = 8;    // one node: 8 MI355X on a full xGMI mesh
constexpr int kXgmiMaxBlocks = 64;  // << 256 CUs: all blocks stay resident while they poll
// flags: [2 slots][kXgmiMaxBlocks][kXgmiMaxRanks] uint32, padded to 64 KiB
constexpr int64_t kXgmiFlagBytes = 64 * 1024;

// Auxiliary (kernel-driven exchange) region: flags [2 slots][kDpMaxBlocks][kXgmiMaxRanks]
// uint32 in the same 64 KiB header, then the same receive-area layout.
constexpr int kDpMaxBlocks = 128;

// Region of one rank: flags, then receive areas [2 slots][kXgmiMaxRanks][slot_stride] fp32.
inline int64_t xgmi_region_bytes(int64_t slot_stride_floats) {
  return kXgmiFlagBytes + 2 * (int64_t)kXgmiMaxRanks * slot_stride_floats * 4;
}

struct XgmiLaunch {
  float* x;
  int64_t n;
  char* regions[kXgmiMaxRanks];
  int rank, world;
  uint32_t* gen;
  int* error;
  int64_t slot_stride;
  int64_t spin_limit;
};

int xgmi_blocks_for(int64_t n);
int launch_xgmi_oneshot(const XgmiLaunch& l, hipStream_t stream);

}  // namespace comm
}  // namespace rla
