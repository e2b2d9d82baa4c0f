// hipps — shared device helpers for the CDNA4 (gfx950) kernels.
//
// Every kernel in this library works on flat, 16-element-aligned buffers produced by the
// parameter/gradient store (hipps/parallel/flat.py): a model's parameters live in ONE fp32
// buffer, gradients in another, and codec payloads in device wire buffers.  That replaces the
// reference's per-tensor pickle path (mpi_comms.py:186-193) with a handful of launches per
// step over contiguous HBM.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace hipps {

constexpr int kBlock = 256;          // 4 waves of 64 lanes
constexpr int kMaxGrid = 256 * 8;    // 256 CUs x 8 resident blocks; grid-stride beyond
constexpr int kMaxSlots = 16;        // max dense sources fused into one aggregate/step launch

// ---- bf16 <-> f32 -------------------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  // hipcc lowers the plain cast to v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving).
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}

// ---- vector loads of 4 elements of a wire type into f32 -----------------------------------
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  __device__ __forceinline__ static float4 load(const float* p, int64_t i) {
    return *reinterpret_cast<const float4*>(p + i);
  }
  __device__ __forceinline__ static void store(float* p, int64_t i, float4 v) {
    *reinterpret_cast<float4*>(p + i) = v;
  }
  __device__ __forceinline__ static float load1(const float* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void store1(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Vec4<uint16_t> {  // bf16 stored as raw 16-bit
  __device__ __forceinline__ static float4 load(const uint16_t* p, int64_t i) {
    uint2 u = *reinterpret_cast<const uint2*>(p + i);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
  }
  __device__ __forceinline__ static void store(uint16_t* p, int64_t i, float4 v) {
    *reinterpret_cast<uint2*>(p + i) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  }
  __device__ __forceinline__ static float load1(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }
  __device__ __forceinline__ static void store1(uint16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
};

struct SlotPtrs {
  const void* p[kMaxSlots];
};

// ---- reading bytes another GPU wrote into this GPU's memory ---------------------------------
// The async PS's mailbox slots are plain (coarse-grained) hipMalloc memory that remote workers
// fill over xGMI; the PS learns of a message from a host-polled doorbell, so no HIP-level
// synchronisation tells this device's caches that the bytes changed.  A worker's mailbox ring is
// rewritten as it wraps, so this XCD's L2 (and the CU's L1) may still hold an older message's lines.
// The consumer therefore acquires at SYSTEM scope before its first load of the slot
// (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility"; cdna_hip_programming.md
// Guideline 16 consumer recipe): one wave issues the invalidate (buffer_inv sc0 sc1), waits for it
// to complete with an explicit vmcnt(0) (the fence's own wait sits BEFORE the invalidate), and the
// barrier holds the other waves until then.  Call it uniformly from every thread of the block.
__device__ __forceinline__ void acquire_remote_block() {
  if (threadIdx.x < 64) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// ---- launch geometry ----------------------------------------------------------------------
inline int grid_for(int64_t work_items, int block = kBlock) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (int)g;
}

// ---- counter-based RNG (splitmix64) for stochastic rounding --------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx) {
  return (float)(splitmix64(seed ^ (idx * 0xD1B54A32D192ED03ull)) >> 40) * (1.0f / 16777216.0f);
}

// ---- wave-level reductions (64 lanes) ------------------------------------------------------
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace hipps
