// hipps runtime — stream-ordered doorbells written by the GPU itself.
//
// The async PS's control words (push / ack sequence numbers, published versions) live in a
// POSIX shared-memory block that every rank maps and registers with hipHostRegister, so the
// device can store into it.  A doorbell is a one-wavefront kernel enqueued on the stream that
// produced the data it announces: it starts only after the stream's earlier copies / kernels
// completed, and stores each word with a system-scope release so the host that polls the word
// (std::atomic acquire load) never sees the doorbell before the announced bytes.
//
// Round 1 rang these bells from hipLaunchHostFunc callbacks, which stall the stream for a host
// round trip per bell (one per pushed bucket and one per PS ack).  This kernel costs one
// launch slot and no host involvement.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "runtime/doorbell.h"

namespace hipps {
namespace rt {

__global__ __launch_bounds__(64) void k_doorbell(DoorbellArgs a) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < a.n; ++i)  // in order: e.g. slot version before the sequence word
    __hip_atomic_store(a.w[i], a.src[i] ? *a.src[i] : a.v[i], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_doorbell(hipStream_t stream, const DoorbellArgs& a) {
  hipLaunchKernelGGL(k_doorbell, dim3(1), dim3(64), 0, stream, a);
  return hipGetLastError();
}

}  // namespace rt
}  // namespace hipps
