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

// Wave-positioned areas of the one-launch step's exchange protocols (mlp_step3.hip,
// "packed" and "owner"): one exchange UNIT per (block, wave) = 64 lanes x 4 values.
//   packed / reduce-scatter area: [2 slots][kXgmiMaxRanks srcs][kDpMaxUnits][64 lanes][2] 8-B granules
//     (two values per granule, the tag in the low mantissa bits of the first)
//   all-gather area:              [2 slots][kDpMaxUnits][64 lanes][4] 8-B {generation, fp32} granules
// A lane's granules are adjacent, so it moves them 16 B per instruction and every
// store instruction of a wave covers 1 KB contiguous bytes (whole 64-B lines over
// the link), not 64 scattered arena positions.
constexpr int kDpMaxUnits = kDpMaxBlocks * 8;
constexpr int64_t kDpPackedGranules = 2LL * kXgmiMaxRanks * kDpMaxUnits * 128;
constexpr int64_t kDpGatherGranules = 2LL * kDpMaxUnits * 256;
// receive-area stride (floats per (slot, rank)) that holds both areas behind the flag header
constexpr int64_t kDpUnitAreaFloats = (kDpPackedGranules + kDpGatherGranules) * 8 / (2 * kXgmiMaxRanks * 4);

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

// Two-shot (reduce-scatter + all-gather) region of one rank (xgmi_twoshot.hip):
// flags [2 slots][2 phases][kTwoShotMaxBlocks][kXgmiMaxRanks] uint32 in the 64 KiB
// header, then [2 slots][2 areas: scatter, gather][world][chunk_stride] wire elements.
// XgmiLaunch::slot_stride is the chunk stride there, in fp32 elements.
constexpr int kTwoShotMaxBlocks = 128;
inline int64_t twoshot_region_bytes(int64_t chunk_stride_floats, int world) {
  return kXgmiFlagBytes + 4 * (int64_t)world * chunk_stride_floats * 4;
}
struct TwoShotPlan {
  int64_t cs;    // chunk length (floats, multiple of 4); chunk c = [c*cs, min((c+1)*cs, n))
  int64_t per4;  // float4s of each chunk per block
  int blocks;
};
TwoShotPlan twoshot_plan(int64_t n, int world);
// bf16_wire: links carry bf16 (fp32 accumulate, result rounded to bf16 once)
int launch_xgmi_twoshot(const XgmiLaunch& l, bool bf16_wire, hipStream_t stream);

}  // namespace comm
}  // namespace rla
