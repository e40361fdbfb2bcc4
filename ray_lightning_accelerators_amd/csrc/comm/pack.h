#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rla {
namespace comm {

constexpr int kPackMax = 48;  // descriptors per launch (kernel-argument table < 1.3 KiB)

struct PackTable {
  const float* src[kPackMax];
  float* dst[kPackMax];
  int64_t n[kPackMax];
  int count;
  float scale;
};

void launch_pack(const PackTable& t, hipStream_t stream);

}  // namespace comm
}  // namespace rla
