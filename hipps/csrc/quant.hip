// hipps — 8-bit block quantization codec (encode on the worker, fused dequant-accumulate on PS).
//
// Replaces the external `codings` QSGD-style encoder the reference calls from its hook
// (ps.py:65-66, 94) and the decode loop (ps.py:165-167).  Wire payload per message:
//   scales : float32[ceil(n / 256)]      (absmax / 127 per 256-element block)
//   q      : int8[n]
// = n + 4*ceil(n/256) bytes vs 4n for the reference's fp32 pickle (mpi_comms.py:186-193).
//
// One 64-lane wave owns one 256-element block (4 elements / lane, 16-byte loads): the block
// absmax is a 6-step __shfl_xor butterfly, no LDS.  Optional error feedback keeps the
// quantization residual on the worker (r <- x + r - deq(q)); optional stochastic rounding uses a
// counter-based hash so a message is reproducible from (seed, index).
#include "common.h"

#include <cstdlib>

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {

constexpr int kQBlock = 256;

__device__ __forceinline__ int8_t q8_round(float x, float inv, bool stochastic, uint64_t seed, int64_t idx) {
  float y = x * inv;
  y = stochastic ? floorf(y + uniform01(seed, (uint64_t)idx)) : rintf(y);
  y = fminf(127.f, fmaxf(-127.f, y));
  return (int8_t)(int)y;
}

// One wave per 256-element block; each wave takes kQUnroll consecutive blocks per iteration so
// every lane has 2 x kQUnroll 16-byte loads in flight (x and residual) before the first use.
constexpr int kQUnroll = 4;
__global__ __launch_bounds__(kBlock) void k_q8_encode(const float* __restrict__ x, float* __restrict__ resid,
                                                      int8_t* __restrict__ q, float* __restrict__ scales, int64_t n,
                                                      int stochastic, uint64_t seed) {
  const int lane = threadIdx.x & 63;
  const int64_t nblocks = (n + kQBlock - 1) / kQBlock;
  const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6) * kQUnroll;
  for (int64_t b0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kQUnroll; b0 < nblocks;
       b0 += wstride) {
    float v[kQUnroll][4];
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u) {
      const int64_t i = (b0 + u) * kQBlock + lane * 4;
      if (i + 4 <= n) {
        float4 t = *reinterpret_cast<const float4*>(x + i);
        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[u][j] = (i + j < n) ? x[i + j] : 0.f;
      }
    }
    if (resid) {
#pragma unroll
      for (int u = 0; u < kQUnroll; ++u) {
        const int64_t i = (b0 + u) * kQBlock + lane * 4;
        if (i + 4 <= n) {
          float4 r = *reinterpret_cast<const float4*>(resid + i);
          v[u][0] += r.x; v[u][1] += r.y; v[u][2] += r.z; v[u][3] += r.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[u][j] += (i + j < n) ? resid[i + j] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kQUnroll; ++u) {
      const int64_t b = b0 + u;
      if (b >= nblocks) break;
      const int64_t i = b * kQBlock + lane * 4;
      float amax = fmaxf(fmaxf(fabsf(v[u][0]), fabsf(v[u][1])), fmaxf(fabsf(v[u][2]), fabsf(v[u][3])));
      amax = wave_max(amax);
      const float scale = amax / 127.f;
      const float inv = amax > 0.f ? 127.f / amax : 0.f;
      int8_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = q8_round(v[u][j], inv, stochastic, seed, i + j);
      if (lane == 0) scales[b] = scale;
      if (i + 4 <= n) {
        *reinterpret_cast<char4*>(q + i) = make_char4(o[0], o[1], o[2], o[3]);
        if (resid)
          *reinterpret_cast<float4*>(resid + i) = make_float4(v[u][0] - o[0] * scale, v[u][1] - o[1] * scale,
                                                              v[u][2] - o[2] * scale, v[u][3] - o[3] * scale);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (i + j < n) {
            q[i + j] = o[j];
            if (resid) resid[i + j] = v[u][j] - o[j] * scale;
          }
      }
    }
  }
}

// Row form (the default): one 16-lane DPP row per 256-element block, 16 elements per lane as four
// 16-byte loads 64 elements apart (each load instruction covers four 256-byte runs), four blocks per
// wave per iteration.  The block absmax is 4 DPP steps inside the row instead of a 6-step
// cross-lane shuffle through LDS per block (6 LDS round trips per block in k_q8_encode), and the
// next iteration's x / residual loads are issued before this one's quantization (software
// pipelined: one HBM round trip exposed per wave, not per iteration).  Same element -> (block,
// scale, rounding index) mapping as k_q8_encode, so the message is bit-identical.
__device__ __forceinline__ float row16_max(float v) {
  // quad xor 1, quad xor 2, half-row mirror, row mirror: every lane of the 16-lane row ends with the
  // row's maximum
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
  return v;
}

__global__ __launch_bounds__(kBlock) void k_q8_encode_rows(const float* __restrict__ x, float* __restrict__ resid,
                                                           int8_t* __restrict__ q, float* __restrict__ scales,
                                                           int64_t n, int stochastic, uint64_t seed) {
  const int lane = threadIdx.x & 63, row = lane >> 4, rl = lane & 15;
  const int64_t nblocks = (n + kQBlock - 1) / kQBlock;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6) * 4;
  // element e = 4*j + k of this lane in block b: b*256 + 64*j + 4*rl + k
  auto load = [&](const float* src, int64_t b, float (&v)[16]) {
    const int64_t base = b * kQBlock + 4 * rl;
    if ((b + 1) * kQBlock <= n) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 t = *reinterpret_cast<const float4*>(src + base + 64 * j);
        v[4 * j] = t.x; v[4 * j + 1] = t.y; v[4 * j + 2] = t.z; v[4 * j + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t i = base + 64 * j + k;
          v[4 * j + k] = i < n ? src[i] : 0.f;
        }
    }
  };
  int64_t b0 = wave * 4;  // the wave's first block this iteration (wave-uniform)
  int64_t b = b0 + row;   // this row's block
  float xv[16], rv[16];
  if (b < nblocks) {
    load(x, b, xv);
    if (resid) load(resid, b, rv);
  }
  while (b0 < nblocks) {
    const int64_t b0n = b0 + wstride, bn = b0n + row;
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = resid ? xv[e] + rv[e] : xv[e];
    if (bn < nblocks) {  // the next iteration's operands in flight during this one's work
      load(x, bn, xv);
      if (resid) load(resid, bn, rv);
    }
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) amax = fmaxf(amax, fabsf(v[e]));
    amax = row16_max(amax);  // every lane of the wave is active here (wave-uniform loop)
    if (b < nblocks) {
      const float scale = amax / 127.f;
      const float inv = amax > 0.f ? 127.f / amax : 0.f;
      const int64_t base = b * kQBlock + 4 * rl;
      if (rl == 0) scales[b] = scale;
      const bool full = (b + 1) * kQBlock <= n;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t i = base + 64 * j;
        int8_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = q8_round(v[4 * j + k], inv, stochastic, seed, i + k);
        if (full) {
          *reinterpret_cast<char4*>(q + i) = make_char4(o[0], o[1], o[2], o[3]);
          if (resid)
            *reinterpret_cast<float4*>(resid + i) =
                make_float4(v[4 * j] - o[0] * scale, v[4 * j + 1] - o[1] * scale, v[4 * j + 2] - o[2] * scale,
                            v[4 * j + 3] - o[3] * scale);
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (i + k < n) {
              q[i + k] = o[k];
              if (resid) resid[i + k] = v[4 * j + k] - o[k] * scale;
            }
        }
      }
    }
    b0 = b0n;
    b = bn;
  }
}

// acc = gscale * sum_w deq(q_w, s_w) (rank order, 4 elements per lane), or with ``accumulate``
// acc = ((acc + g*deq_0) + g*deq_1) + ... -- each message on its own, no contraction: batch-
// invariant, as flat.hip k_aggregate
__global__ __launch_bounds__(kBlock) void k_q8_aggregate(SlotPtrs qs, SlotPtrs ss, int W, float gscale,
                                                         float* __restrict__ acc, int64_t n, int accumulate,
                                                         int acquire) {
  if (acquire) acquire_remote_block();  // a source slot was written by another GPU (common.h)
  const int64_t nv = (n + 3) >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t i = v << 2;
    const int64_t blk = i / kQBlock;
    if (accumulate) {
      if (i + 4 <= n) {
        float4 a = *reinterpret_cast<const float4*>(acc + i);
        for (int w = 0; w < W; ++w) {
          const char4 c = *reinterpret_cast<const char4*>(reinterpret_cast<const int8_t*>(qs.p[w]) + i);
          const float s = reinterpret_cast<const float*>(ss.p[w])[blk];
          a.x = __fadd_rn(a.x, __fmul_rn(__fmul_rn((float)c.x, s), gscale));
          a.y = __fadd_rn(a.y, __fmul_rn(__fmul_rn((float)c.y, s), gscale));
          a.z = __fadd_rn(a.z, __fmul_rn(__fmul_rn((float)c.z, s), gscale));
          a.w = __fadd_rn(a.w, __fmul_rn(__fmul_rn((float)c.w, s), gscale));
        }
        *reinterpret_cast<float4*>(acc + i) = a;
      } else {
        for (int j = 0; j < 4 && i + j < n; ++j) {
          float a = acc[i + j];
          for (int w = 0; w < W; ++w) {
            const int8_t* q = reinterpret_cast<const int8_t*>(qs.p[w]);
            const float s = reinterpret_cast<const float*>(ss.p[w])[blk];
            a = __fadd_rn(a, __fmul_rn(__fmul_rn((float)q[i + j], s), gscale));
          }
          acc[i + j] = a;
        }
      }
      continue;
    }
    float d[4] = {0.f, 0.f, 0.f, 0.f};
    const bool full = i + 4 <= n;
    for (int w = 0; w < W; ++w) {
      const int8_t* q = reinterpret_cast<const int8_t*>(qs.p[w]);
      const float s = reinterpret_cast<const float*>(ss.p[w])[blk];
      if (full) {
        char4 c = *reinterpret_cast<const char4*>(q + i);
        d[0] += c.x * s; d[1] += c.y * s; d[2] += c.z * s; d[3] += c.w * s;
      } else {
        for (int j = 0; j < 4; ++j)
          if (i + j < n) d[j] += q[i + j] * s;
      }
    }
    if (full) {
      float4 o = make_float4(d[0] * gscale, d[1] * gscale, d[2] * gscale, d[3] * gscale);
      if (accumulate) {
        float4 a = *reinterpret_cast<const float4*>(acc + i);
        o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
      }
      *reinterpret_cast<float4*>(acc + i) = o;
    } else {
      for (int j = 0; j < 4; ++j)
        if (i + j < n) acc[i + j] = (accumulate ? acc[i + j] : 0.f) + d[j] * gscale;
    }
  }
}

// ------------------------------------------------------------------------------------------
void q8_encode(at::Tensor x, c10::optional<at::Tensor> resid, at::Tensor q, at::Tensor scales, bool stochastic,
               int64_t seed) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == at::kFloat, "x: contiguous f32 device tensor");
  const int64_t n = x.numel();
  TORCH_CHECK(q.numel() == n && q.scalar_type() == at::kChar, "q must be int8[n]");
  TORCH_CHECK(scales.numel() == (n + kQBlock - 1) / kQBlock && scales.scalar_type() == at::kFloat,
              "scales must be f32[ceil(n/256)]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(q.data_ptr()) % 4 == 0,
              "x must be 16-byte and q 4-byte aligned");
  float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->numel() == n && resid->scalar_type() == at::kFloat && resid->is_contiguous(), "residual");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(resid->data_ptr()) % 16 == 0, "residual must be 16-byte aligned");
    rp = resid->data_ptr<float>();
  }
  const int64_t nblocks = (n + kQBlock - 1) / kQBlock;
  static const bool rows = [] {  // HIPPS_Q8_ENC=0: the one-wave-per-block kernel, for A/B
    const char* e = std::getenv("HIPPS_Q8_ENC");
    return !(e && e[0] == '0');
  }();
  const int grid = grid_for((nblocks + kQUnroll - 1) / kQUnroll * 64);
  if (rows)
    hipLaunchKernelGGL(k_q8_encode_rows, grid, kBlock, 0, c10::hip::getCurrentHIPStream(), x.data_ptr<float>(), rp,
                       (int8_t*)q.data_ptr(), scales.data_ptr<float>(), n, (int)stochastic, (uint64_t)seed);
  else
    hipLaunchKernelGGL(k_q8_encode, grid, kBlock, 0, c10::hip::getCurrentHIPStream(), x.data_ptr<float>(), rp,
                       (int8_t*)q.data_ptr(), scales.data_ptr<float>(), n, (int)stochastic, (uint64_t)seed);
}

void q8_aggregate(const std::vector<at::Tensor>& qs, const std::vector<at::Tensor>& ss, at::Tensor acc, double gscale,
                  bool accumulate, bool acquire) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat && acc.is_contiguous(), "acc: f32 device tensor");
  TORCH_CHECK(!qs.empty() && qs.size() == ss.size() && (int)qs.size() <= kMaxSlots, "1..16 (q, scale) pairs");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(acc.data_ptr()) % 16 == 0, "acc must be 16-byte aligned");
  const int64_t n = acc.numel();
  SlotPtrs qp{}, sp{};
  for (size_t w = 0; w < qs.size(); ++w) {
    TORCH_CHECK(qs[w].numel() == n && qs[w].scalar_type() == at::kChar, "q size/dtype");
    TORCH_CHECK(ss[w].numel() == (n + kQBlock - 1) / kQBlock && ss[w].scalar_type() == at::kFloat, "scale size");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(qs[w].data_ptr()) % 4 == 0, "q must be 4-byte aligned");
    qp.p[w] = qs[w].data_ptr();
    sp.p[w] = ss[w].data_ptr();
  }
  const int grid = grid_for((n + 3) >> 2);
  hipLaunchKernelGGL(k_q8_aggregate, grid, kBlock, 0, c10::hip::getCurrentHIPStream(), qp, sp, (int)qs.size(),
                     (float)gscale, acc.data_ptr<float>(), n, (int)accumulate, (int)acquire);
}

}  // namespace hipps
