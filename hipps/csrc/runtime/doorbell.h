// hipps runtime — device doorbell launcher (doorbell.hip), used by control.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hipps {
namespace rt {

constexpr int kMaxBell = 6;  // words stored by one doorbell launch

struct DoorbellArgs {
  int64_t* w[kMaxBell];  // device-visible addresses of control words (registered host memory)
  int64_t v[kMaxBell];
  const int64_t* src[kMaxBell];  // non-null: store *src (device memory, read in stream order) instead of v
  int n;
};

hipError_t launch_doorbell(hipStream_t stream, const DoorbellArgs& a);

}  // namespace rt
}  // namespace hipps
