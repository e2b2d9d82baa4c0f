// hipps — dense flat-buffer kernels: wire cast/pack, rank-ordered aggregate, fused optimizers.
//
// Reference parity:
//   K4  d_p = sum(grads)               ps.py:176       -> k_aggregate (fixed rank order, fp32 acc)
//   K5  SGD wd/momentum/nesterov/update ps.py:197-214  -> k_sgd   (one pass, fused with K4)
//   K6  Adam (reference eps placement)  ps.py:217-261  -> k_adam  (one pass, fused with K4)
//   K1/K2/K3 host staging + float cast  mpi_comms.py:32-58 -> k_convert (device-resident wire)
//
// All kernels are HBM-bound streams: 16-byte (fp32x4) or 8-byte (bf16x4) vector accesses per
// lane, grid capped at 8 blocks/CU with a grid-stride loop (cdna_hip_programming.md G11/G13).
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {

// ------------------------------------------------------------------------------------------
// element ops (scalar form; the vector loops apply them lane-wise).  fmaf mirrors ATen's
// add_(alpha, other) == fma(other, alpha, self) so results track torch to ~1 ulp.
// ------------------------------------------------------------------------------------------
struct SgdHp {
  float lr, wd, mom, damp;
  int nesterov, first;
  float la;  // look-ahead publish: pub = p - la * buf (delay-compensated async read, 0 = off)
};

__device__ __forceinline__ float sgd1(float& p, float& b, float d, const SgdHp& h, bool has_buf) {
  if (h.wd != 0.f) d = fmaf(h.wd, p, d);
  if (h.mom != 0.f && has_buf) {
    b = h.first ? d : fmaf(1.f - h.damp, d, b * h.mom);
    d = h.nesterov ? fmaf(h.mom, b, d) : b;
  }
  p = fmaf(-h.lr, d, p);
  return p;
}

struct AdamHp {
  float lr, b1, b2, eps, wd, step_size, bc2_sqrt;
  int amsgrad, torch_mode, step;
};

// bias-correction scalars for step t, in double like the host launcher (a chunk whose own step
// count equals the group's uses the host's values unchanged, so both paths agree bit for bit)
__device__ __forceinline__ void adam_bias(AdamHp& h, int t) {
  const double bc1 = 1.0 - pow((double)h.b1, (double)t), bc2 = 1.0 - pow((double)h.b2, (double)t);
  h.step_size = (float)(h.torch_mode ? (double)h.lr / bc1 : (double)h.lr * sqrt(bc2) / bc1);
  h.bc2_sqrt = (float)sqrt(bc2);
}

__device__ __forceinline__ float adam1(float& p, float& m, float& v, float* vmax, float g, const AdamHp& h) {
  if (h.wd != 0.f) g = fmaf(h.wd, p, g);
  m = fmaf(1.f - h.b1, g, m * h.b1);
  v = fmaf((1.f - h.b2) * g, g, v * h.b2);
  float vv = v;
  if (h.amsgrad) {
    vv = fmaxf(*vmax, v);
    *vmax = vv;
  }
  // reference (ps.py:255): denom = sqrt(v) + eps, step_size = lr*sqrt(bc2)/bc1
  // torch   (>=1.0)       : denom = sqrt(v)/sqrt(bc2) + eps, step_size = lr/bc1
  float denom = h.torch_mode ? (sqrtf(vv) / h.bc2_sqrt + h.eps) : (sqrtf(vv) + h.eps);
  p = fmaf(-h.step_size, m / denom, p);
  return p;
}

// Look-ahead publish for asynchronous readers (delay-compensated momentum, cf. DANA, Hakimi et
// al. 2019): a worker's gradient lands tau updates after the version it read, and those updates
// carry at least the momentum part lr * (mu + ... + mu^tau) * buf, so the PS publishes the
// parameters extrapolated by it; the fp32 master itself is unchanged.
__device__ __forceinline__ float4 lookahead4(float4 p, float4 b, float la) {
  return make_float4(fmaf(-la, b.x, p.x), fmaf(-la, b.y, p.y), fmaf(-la, b.z, p.z), fmaf(-la, b.w, p.w));
}

template <typename T>
__device__ __forceinline__ float4 sum_slots4(const SlotPtrs& g, int W, int64_t i, float gscale) {
  float4 d = Vec4<T>::load(reinterpret_cast<const T*>(g.p[0]), i);
  for (int w = 1; w < W; ++w) {  // fixed rank order -> bitwise identical on every rank
    float4 s = Vec4<T>::load(reinterpret_cast<const T*>(g.p[w]), i);
    d.x += s.x; d.y += s.y; d.z += s.z; d.w += s.w;
  }
  if (gscale != 1.f) { d.x *= gscale; d.y *= gscale; d.z *= gscale; d.w *= gscale; }
  return d;
}
template <typename T>
__device__ __forceinline__ float sum_slots1(const SlotPtrs& g, int W, int64_t i, float gscale) {
  float d = Vec4<T>::load1(reinterpret_cast<const T*>(g.p[0]), i);
  for (int w = 1; w < W; ++w) d += Vec4<T>::load1(reinterpret_cast<const T*>(g.p[w]), i);
  return gscale != 1.f ? d * gscale : d;
}

__device__ __forceinline__ void pub_store4(void* pub, int pub_mode, int64_t i, float4 v) {
  if (pub_mode == 1) Vec4<float>::store(reinterpret_cast<float*>(pub), i, v);
  else if (pub_mode == 2) Vec4<uint16_t>::store(reinterpret_cast<uint16_t*>(pub), i, v);
}
__device__ __forceinline__ void pub_store1(void* pub, int pub_mode, int64_t i, float v) {
  if (pub_mode == 1) reinterpret_cast<float*>(pub)[i] = v;
  else if (pub_mode == 2) reinterpret_cast<uint16_t*>(pub)[i] = f32_to_bf16(v);
}

// ------------------------------------------------------------------------------------------
// k_aggregate: acc = gscale * sum_w slot_w (rank order), or with ``accumulate`` (the async PS
// adding the messages that arrived) acc = (((acc + g*slot_0) + g*slot_1) + ...) -- each message
// added on its own, without contraction, so the result does not depend on how arriving messages
// were batched into launches (it did: identical messages summed as {a, a, a} or {a}, {a, a}
// rounded differently -- tests/test_multigpu.py's same-device determinism case failed once)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_aggregate(SlotPtrs g, int W, float gscale, float* __restrict__ acc,
                                                      int64_t n, int accumulate, int acquire) {
  if (acquire) acquire_remote_block();  // a source slot was written by another GPU (common.h)
  const int64_t nv = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t i = v << 2;
    float4 d;
    if (accumulate) {
      d = Vec4<float>::load(acc, i);
      for (int w = 0; w < W; ++w) {
        const float4 s = Vec4<T>::load(reinterpret_cast<const T*>(g.p[w]), i);
        d.x = __fadd_rn(d.x, __fmul_rn(s.x, gscale));
        d.y = __fadd_rn(d.y, __fmul_rn(s.y, gscale));
        d.z = __fadd_rn(d.z, __fmul_rn(s.z, gscale));
        d.w = __fadd_rn(d.w, __fmul_rn(s.w, gscale));
      }
    } else {
      d = sum_slots4<T>(g, W, i, gscale);
    }
    Vec4<float>::store(acc, i, d);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nv << 2) + threadIdx.x; i < n; i += blockDim.x) {
      if (accumulate) {
        float d = acc[i];
        for (int w = 0; w < W; ++w)
          d = __fadd_rn(d, __fmul_rn(Vec4<T>::load1(reinterpret_cast<const T*>(g.p[w]), i), gscale));
        acc[i] = d;
      } else {
        acc[i] = sum_slots1<T>(g, W, i, gscale);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// k_copy_acquire: dst = src (bytes), after a system-scope acquire -- stages bytes another GPU
// wrote into this device's memory (presence bytes, canaries, object-codec blobs of a remote
// worker's mailbox slot) into a private buffer that ordinary torch kernels may then read.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_copy_acquire(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         int64_t n) {
  acquire_remote_block();
  const int64_t nv = n >> 4, stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t v = t0; v < nv; v += stride)
    reinterpret_cast<uint4*>(dst)[v] = reinterpret_cast<const uint4*>(src)[v];
  for (int64_t i = (nv << 4) + t0; i < n; i += stride) dst[i] = src[i];
}

// ------------------------------------------------------------------------------------------
// k_convert: dst(Tout) = scale * src(Tin)   (f32->bf16 wire pack, bf16->f32 unpack, copies)
// ------------------------------------------------------------------------------------------
template <typename Tin, typename Tout>
__global__ __launch_bounds__(kBlock) void k_convert(const Tin* __restrict__ src, Tout* __restrict__ dst, int64_t n,
                                                    float scale) {
  // four 4-element groups per lane per iteration, all loads issued before the first store
  constexpr int U = 4;
  const int64_t nv = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v0 < nv; v0 += U * stride) {
    float4 d[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (v0 + u * stride < nv) d[u] = Vec4<Tin>::load(src, (v0 + u * stride) << 2);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v0 + u * stride >= nv) break;
      float4 e = d[u];
      if (scale != 1.f) { e.x *= scale; e.y *= scale; e.z *= scale; e.w *= scale; }
      Vec4<Tout>::store(dst, (v0 + u * stride) << 2, e);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nv << 2) + threadIdx.x; i < n; i += blockDim.x)
      Vec4<Tout>::store1(dst, i, Vec4<Tin>::load1(src, i) * scale);
  }
}

// ------------------------------------------------------------------------------------------
// k_sgd: decode + sum_W + weight decay + momentum/nesterov + update + publish, one pass.
// zero_src: when the gradient source is a single fp32 accumulator, clear it in the same pass
// (the async PS re-arms its accumulator without a separate memset).
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kBlock) void k_sgd(SlotPtrs g, int W, float gscale, float* __restrict__ p,
                                                float* __restrict__ buf, void* __restrict__ pub, int pub_mode,
                                                int zero_src, int64_t n, SgdHp h, const uint8_t* __restrict__ cmask,
                                                int* __restrict__ cstep) {
  const bool has_buf = buf != nullptr;
  const int64_t nv = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t i = v << 2;
    float4 pv = Vec4<float>::load(p, i);
    if (cmask && !cmask[i >> 4]) {  // parameter without a gradient this step: untouched (ps.py:178-179)
      if (zero_src) Vec4<float>::store((float*)g.p[0], i, make_float4(0.f, 0.f, 0.f, 0.f));
      if (h.la != 0.f && has_buf) pv = lookahead4(pv, Vec4<float>::load(buf, i), h.la);
      pub_store4(pub, pub_mode, i, pv);
      continue;
    }
    float4 d = sum_slots4<T>(g, W, i, gscale);
    if (zero_src) Vec4<float>::store((float*)g.p[0], i, make_float4(0.f, 0.f, 0.f, 0.f));
    SgdHp hc = h;
    if (cstep) {  // per-parameter first step (ps.py:203-205): this chunk's own update count
      const int cs = cstep[i >> 4];
      hc.first = cs == 0;
      if ((i & 15) == 0) cstep[i >> 4] = cs + 1;  // one lane per chunk; n % 16 == 0 (host check)
    }
    float4 b = has_buf && !hc.first ? Vec4<float>::load(buf, i) : make_float4(0.f, 0.f, 0.f, 0.f);
    sgd1(pv.x, b.x, d.x, hc, has_buf);
    sgd1(pv.y, b.y, d.y, hc, has_buf);
    sgd1(pv.z, b.z, d.z, hc, has_buf);
    sgd1(pv.w, b.w, d.w, hc, has_buf);
    Vec4<float>::store(p, i, pv);
    if (has_buf && h.mom != 0.f) Vec4<float>::store(buf, i, b);
    pub_store4(pub, pub_mode, i, h.la != 0.f && has_buf ? lookahead4(pv, b, h.la) : pv);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nv << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float d = sum_slots1<T>(g, W, i, gscale);
      if (zero_src) ((float*)g.p[0])[i] = 0.f;
      float pv = p[i];
      if (cmask && !cmask[i >> 4]) {
        pub_store1(pub, pub_mode, i, h.la != 0.f && has_buf ? fmaf(-h.la, buf[i], pv) : pv);
        continue;
      }
      float b = has_buf && !h.first ? buf[i] : 0.f;
      sgd1(pv, b, d, h, has_buf);
      p[i] = pv;
      if (has_buf && h.mom != 0.f) buf[i] = b;
      pub_store1(pub, pub_mode, i, h.la != 0.f && has_buf ? fmaf(-h.la, b, pv) : pv);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_adam(SlotPtrs g, int W, float gscale, float* __restrict__ p,
                                                 float* __restrict__ m, float* __restrict__ vv,
                                                 float* __restrict__ vmax, void* __restrict__ pub, int pub_mode,
                                                 int zero_src, int64_t n, AdamHp h, const uint8_t* __restrict__ cmask,
                                                 int* __restrict__ cstep) {
  const int64_t nv = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  float dummy = 0.f;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t i = v << 2;
    if (cmask && !cmask[i >> 4]) {
      if (zero_src) Vec4<float>::store((float*)g.p[0], i, make_float4(0.f, 0.f, 0.f, 0.f));
      pub_store4(pub, pub_mode, i, Vec4<float>::load(p, i));
      continue;
    }
    float4 d = sum_slots4<T>(g, W, i, gscale);
    if (zero_src) Vec4<float>::store((float*)g.p[0], i, make_float4(0.f, 0.f, 0.f, 0.f));
    float4 pv = Vec4<float>::load(p, i), mv = Vec4<float>::load(m, i), sv = Vec4<float>::load(vv, i);
    float4 xv = h.amsgrad ? Vec4<float>::load(vmax, i) : make_float4(0.f, 0.f, 0.f, 0.f);
    AdamHp hc = h;
    if (cstep) {  // per-parameter step (ps.py:241): a late-starting parameter is corrected for its own t
      const int t = cstep[i >> 4] + 1;
      if (t != h.step) adam_bias(hc, t);
      if ((i & 15) == 0) cstep[i >> 4] = t;
    }
    adam1(pv.x, mv.x, sv.x, &xv.x, d.x, hc);
    adam1(pv.y, mv.y, sv.y, &xv.y, d.y, hc);
    adam1(pv.z, mv.z, sv.z, &xv.z, d.z, hc);
    adam1(pv.w, mv.w, sv.w, &xv.w, d.w, hc);
    Vec4<float>::store(p, i, pv);
    Vec4<float>::store(m, i, mv);
    Vec4<float>::store(vv, i, sv);
    if (h.amsgrad) Vec4<float>::store(vmax, i, xv);
    pub_store4(pub, pub_mode, i, pv);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nv << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float d = sum_slots1<T>(g, W, i, gscale);
      if (zero_src) ((float*)g.p[0])[i] = 0.f;
      if (cmask && !cmask[i >> 4]) {
        pub_store1(pub, pub_mode, i, p[i]);
        continue;
      }
      float pv = p[i], mv = m[i], sv = vv[i];
      float* xp = h.amsgrad ? &vmax[i] : &dummy;
      adam1(pv, mv, sv, xp, d, h);
      p[i] = pv; m[i] = mv; vv[i] = sv;
      pub_store1(pub, pub_mode, i, pv);
    }
  }
}

// ------------------------------------------------------------------------------------------
// k_gather: multi-tensor gather of autograd-owned gradient tensors into a flat destination
// (fp32 flat gradient or a dense bf16/fp32 wire image), one launch per bucket instead of one
// accumulate kernel per parameter.  Source pointers travel in the kernel arguments (<= 256
// tensors per launch); the chunk table (tensor, src offset, dst offset, length) is static and
// device-resident.
// ------------------------------------------------------------------------------------------
constexpr int kGatherMax = 256;
struct GatherPtrs {
  const float* p[kGatherMax];
};

template <typename Tout>
__global__ __launch_bounds__(kBlock) void k_gather(GatherPtrs src, const int64_t* __restrict__ table, int64_t nchunks,
                                                   Tout* __restrict__ dst, float scale) {
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t* row = table + c * 4;
    const float* s = src.p[row[0]] + row[1];
    Tout* d = dst + row[2];
    const int64_t len = row[3];
    const bool vec = ((reinterpret_cast<uintptr_t>(s) & 15) == 0);
    const int64_t nv = vec ? (len >> 2) : 0;
    constexpr int U = 4;  // four 16-byte loads in flight per lane before any store
    for (int64_t v0 = threadIdx.x; v0 < nv; v0 += U * (int64_t)blockDim.x) {
      float4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (v0 + u * (int64_t)blockDim.x < nv) x[u] = Vec4<float>::load(s, (v0 + u * (int64_t)blockDim.x) << 2);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (v0 + u * (int64_t)blockDim.x < nv) {
          if (scale != 1.f) { x[u].x *= scale; x[u].y *= scale; x[u].z *= scale; x[u].w *= scale; }
          Vec4<Tout>::store(d, (v0 + u * (int64_t)blockDim.x) << 2, x[u]);
        }
    }
    for (int64_t i = (nv << 2) + threadIdx.x; i < len; i += blockDim.x) Vec4<Tout>::store1(d, i, s[i] * scale);
  }
}

// ------------------------------------------------------------------------------------------
// k_transpose_cast: dst[c * dst_ld + r] = bf16(src[r * src_ld + c]) over a list of fp32 matrix
// slices, one launch per weight refresh.  Feeds two backward operands: the 1x1-conv weights
// [Cout, Cin] -> [Cin, Cout] (the input-gradient GEMM's K-contiguous B operand), and every tap of
// a KxK weight (channels-last [Cout][KH][KW][Cin]) -> tap (KH-1-kh, KW-1-kw) of [Cin][KH][KW][Cout],
// i.e. rot180(W)^T for the stride-1 input gradient run as a forward convolution.  Without it,
// each layer pays one transpose (+flip) launch per backward.  64x64 tiles through LDS (row stride
// 65: conflict-free column reads); the tile table (src off, dst off, R, C, r0, c0, src_ld,
// dst_ld) is static and device-resident.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_transpose_cast(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                           const int64_t* __restrict__ tiles, int64_t ntiles) {
  __shared__ float t[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int64_t b = blockIdx.x; b < ntiles; b += gridDim.x) {
    const int64_t* row = tiles + b * 8;
    const float* s = src + row[0];
    uint16_t* d = dst + row[1];
    const int64_t R = row[2], C = row[3], r0 = row[4], c0 = row[5], sld = row[6], dld = row[7];
    for (int i = ty; i < 64; i += kBlock / 64) {
      const int64_t r = r0 + i, c = c0 + tx;
      t[i][tx] = (r < R && c < C) ? s[r * sld + c] : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += kBlock / 64) {
      const int64_t c = c0 + i, r = r0 + tx;
      if (c < C && r < R) d[c * dld + r] = f32_to_bf16(t[tx][i]);
    }
    __syncthreads();
  }
}

// ==========================================================================================
// host launchers
// ==========================================================================================
namespace {

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device (HIP) tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

enum class WireT { F32, BF16 };

WireT wire_of(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return WireT::F32;
  if (t.scalar_type() == at::kBFloat16) return WireT::BF16;
  TORCH_CHECK(false, "wire dtype must be float32 or bfloat16, got ", t.scalar_type());
}

SlotPtrs make_slots(const std::vector<at::Tensor>& slots, int64_t n, WireT& wt) {
  TORCH_CHECK(!slots.empty() && (int)slots.size() <= kMaxSlots, "1..", kMaxSlots, " gradient sources required");
  SlotPtrs s{};
  wt = wire_of(slots[0]);
  for (size_t w = 0; w < slots.size(); ++w) {
    check_dev(slots[w], "grad source");
    TORCH_CHECK(wire_of(slots[w]) == wt, "all gradient sources must share one dtype");
    TORCH_CHECK(slots[w].numel() == n, "gradient source ", w, " has ", slots[w].numel(), " elements, expected ", n);
    s.p[w] = slots[w].data_ptr();
  }
  return s;
}

// chunk mask: one byte per 16 flat elements (every parameter slot starts on a 16-element
// boundary, so a chunk never straddles two parameters); 0 = skip the chunk this step
const uint8_t* cmask_of(const c10::optional<at::Tensor>& mask, int64_t n) {
  if (!mask.has_value() || !mask->defined()) return nullptr;
  TORCH_CHECK(mask->is_cuda() && mask->is_contiguous() && mask->scalar_type() == at::kByte,
              "mask must be a contiguous uint8 device tensor");
  TORCH_CHECK(mask->numel() >= (n + 15) / 16, "mask has ", mask->numel(), " chunks, need ", (n + 15) / 16);
  return mask->data_ptr<uint8_t>();
}

// per-chunk update counts (int32, one per 16 elements): the per-parameter optimizer step of
// ps.py:203-205 (momentum first step) and ps.py:241 (Adam state['step'])
int* csteps_of(const c10::optional<at::Tensor>& cs, int64_t n) {
  if (!cs.has_value() || !cs->defined()) return nullptr;
  TORCH_CHECK(cs->is_cuda() && cs->is_contiguous() && cs->scalar_type() == at::kInt,
              "csteps must be a contiguous int32 device tensor");
  TORCH_CHECK(n % 16 == 0 && cs->numel() == n / 16, "csteps must hold one count per 16-element chunk of a "
              "16-aligned range (", cs->numel(), " vs n=", n, ")");
  return cs->data_ptr<int>();
}

int pub_mode_of(const c10::optional<at::Tensor>& pub, int64_t n) {
  if (!pub.has_value() || !pub->defined()) return 0;
  check_dev(*pub, "publish");
  TORCH_CHECK(pub->numel() == n, "publish buffer size mismatch");
  return wire_of(*pub) == WireT::F32 ? 1 : 2;
}

}  // namespace

void aggregate(const std::vector<at::Tensor>& slots, at::Tensor acc, double gscale, bool accumulate, bool acquire) {
  check_dev(acc, "acc");
  TORCH_CHECK(acc.scalar_type() == at::kFloat, "acc must be float32");
  const int64_t n = acc.numel();
  WireT wt;
  SlotPtrs s = make_slots(slots, n, wt);
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = grid_for(n >> 2);
  if (wt == WireT::F32)
    hipLaunchKernelGGL(k_aggregate<float>, grid, kBlock, 0, stream, s, (int)slots.size(), (float)gscale,
                       acc.data_ptr<float>(), n, (int)accumulate, (int)acquire);
  else
    hipLaunchKernelGGL(k_aggregate<uint16_t>, grid, kBlock, 0, stream, s, (int)slots.size(), (float)gscale,
                       acc.data_ptr<float>(), n, (int)accumulate, (int)acquire);
}

void copy_acquire(at::Tensor src, at::Tensor dst) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.scalar_type() == at::kByte && dst.scalar_type() == at::kByte,
              "copy_acquire: uint8 device tensors");
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && src.numel() == dst.numel(), "copy_acquire: sizes");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "copy_acquire: 16-byte aligned buffers");
  const int64_t n = src.numel();
  if (n == 0) return;
  hipLaunchKernelGGL(k_copy_acquire, grid_for((n + 15) >> 4), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     src.data_ptr<uint8_t>(), dst.data_ptr<uint8_t>(), n);
}

void convert(at::Tensor src, at::Tensor dst, double scale) {
  check_dev(src, "src");
  check_dev(dst, "dst");
  const int64_t n = src.numel();
  TORCH_CHECK(dst.numel() == n, "convert size mismatch");
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = grid_for(n >> 2);
  const WireT a = wire_of(src), b = wire_of(dst);
  const float sc = (float)scale;
  if (a == WireT::F32 && b == WireT::BF16)
    hipLaunchKernelGGL((k_convert<float, uint16_t>), grid, kBlock, 0, stream, src.data_ptr<float>(),
                       (uint16_t*)dst.data_ptr(), n, sc);
  else if (a == WireT::BF16 && b == WireT::F32)
    hipLaunchKernelGGL((k_convert<uint16_t, float>), grid, kBlock, 0, stream, (const uint16_t*)src.data_ptr(),
                       dst.data_ptr<float>(), n, sc);
  else if (a == WireT::F32 && b == WireT::F32)
    hipLaunchKernelGGL((k_convert<float, float>), grid, kBlock, 0, stream, src.data_ptr<float>(),
                       dst.data_ptr<float>(), n, sc);
  else
    hipLaunchKernelGGL((k_convert<uint16_t, uint16_t>), grid, kBlock, 0, stream, (const uint16_t*)src.data_ptr(),
                       (uint16_t*)dst.data_ptr(), n, sc);
}

void gather_flat(const std::vector<at::Tensor>& srcs, at::Tensor table, at::Tensor dst, double scale) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= kGatherMax, "1..256 source tensors per gather");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.dim() == 2 && table.size(1) == 4,
              "table must be a device int64 [nchunks, 4]");
  check_dev(dst, "dst");
  GatherPtrs p{};
  for (size_t i = 0; i < srcs.size(); ++i) {
    TORCH_CHECK(srcs[i].is_cuda() && srcs[i].scalar_type() == at::kFloat, "gather sources must be f32 device tensors");
    TORCH_CHECK(srcs[i].is_non_overlapping_and_dense(), "gather source must be dense");
    p.p[i] = srcs[i].data_ptr<float>();
  }
  const int64_t nchunks = table.size(0);
  if (nchunks == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = (int)std::min<int64_t>(nchunks, kMaxGrid);
  if (wire_of(dst) == WireT::F32)
    hipLaunchKernelGGL(k_gather<float>, grid, kBlock, 0, stream, p, table.data_ptr<int64_t>(), nchunks,
                       dst.data_ptr<float>(), (float)scale);
  else
    hipLaunchKernelGGL(k_gather<uint16_t>, grid, kBlock, 0, stream, p, table.data_ptr<int64_t>(), nchunks,
                       (uint16_t*)dst.data_ptr(), (float)scale);
}

void transpose_cast(at::Tensor src, at::Tensor dst, at::Tensor tiles) {
  check_dev(src, "src");
  check_dev(dst, "dst");
  TORCH_CHECK(src.scalar_type() == at::kFloat && src.is_contiguous(), "src must be a contiguous f32 flat buffer");
  TORCH_CHECK(dst.scalar_type() == at::kBFloat16 && dst.is_contiguous(), "dst must be a contiguous bf16 flat buffer");
  TORCH_CHECK(tiles.is_cuda() && tiles.scalar_type() == at::kLong && tiles.dim() == 2 && tiles.size(1) == 8,
              "tiles must be a device int64 [ntiles, 8]");
  const int64_t ntiles = tiles.size(0);
  if (ntiles == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = (int)std::min<int64_t>(ntiles, kMaxGrid);
  hipLaunchKernelGGL(k_transpose_cast, grid, kBlock, 0, stream, src.data_ptr<float>(), (uint16_t*)dst.data_ptr(),
                     tiles.data_ptr<int64_t>(), ntiles);
}

void sgd_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, c10::optional<at::Tensor> buf,
              c10::optional<at::Tensor> pub, bool zero_src, double lr, double wd, double momentum, double dampening,
              bool nesterov, bool first, c10::optional<at::Tensor> mask, c10::optional<at::Tensor> csteps,
              double lookahead) {
  check_dev(p, "param");
  TORCH_CHECK(p.scalar_type() == at::kFloat, "param master must be float32");
  const int64_t n = p.numel();
  WireT wt;
  SlotPtrs s = make_slots(grads, n, wt);
  float* bp = nullptr;
  if (buf.has_value() && buf->defined()) {
    check_dev(*buf, "momentum_buffer");
    TORCH_CHECK(buf->numel() == n && buf->scalar_type() == at::kFloat, "momentum buffer mismatch");
    bp = buf->data_ptr<float>();
  }
  TORCH_CHECK(momentum == 0.0 || bp != nullptr, "momentum != 0 requires a momentum buffer");
  TORCH_CHECK(!zero_src || (grads.size() == 1 && wt == WireT::F32), "zero_src needs a single fp32 source");
  const int pm = pub_mode_of(pub, n);
  void* pp = pm ? pub->data_ptr() : nullptr;
  SgdHp h{(float)lr, (float)wd, (float)momentum, (float)dampening, (int)nesterov, (int)first, (float)lookahead};
  TORCH_CHECK(lookahead == 0.0 || bp != nullptr, "a look-ahead publish needs the momentum buffer");
  const uint8_t* cm = cmask_of(mask, n);
  int* cs = csteps_of(csteps, n);
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = grid_for(n >> 2);
  if (wt == WireT::F32)
    hipLaunchKernelGGL(k_sgd<float>, grid, kBlock, 0, stream, s, (int)grads.size(), (float)gscale,
                       p.data_ptr<float>(), bp, pp, pm, (int)zero_src, n, h, cm, cs);
  else
    hipLaunchKernelGGL(k_sgd<uint16_t>, grid, kBlock, 0, stream, s, (int)grads.size(), (float)gscale,
                       p.data_ptr<float>(), bp, pp, pm, (int)zero_src, n, h, cm, cs);
}

void adam_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, at::Tensor exp_avg,
               at::Tensor exp_avg_sq, c10::optional<at::Tensor> max_exp_avg_sq, c10::optional<at::Tensor> pub,
               bool zero_src, double lr, double beta1, double beta2, double eps, double wd, int64_t step,
               bool amsgrad, bool torch_mode, c10::optional<at::Tensor> mask, c10::optional<at::Tensor> csteps) {
  check_dev(p, "param");
  check_dev(exp_avg, "exp_avg");
  check_dev(exp_avg_sq, "exp_avg_sq");
  const int64_t n = p.numel();
  TORCH_CHECK(exp_avg.numel() == n && exp_avg_sq.numel() == n, "adam state size mismatch");
  WireT wt;
  SlotPtrs s = make_slots(grads, n, wt);
  float* xp = nullptr;
  if (amsgrad) {
    TORCH_CHECK(max_exp_avg_sq.has_value() && max_exp_avg_sq->defined(), "amsgrad needs max_exp_avg_sq");
    check_dev(*max_exp_avg_sq, "max_exp_avg_sq");
    xp = max_exp_avg_sq->data_ptr<float>();
  }
  TORCH_CHECK(!zero_src || (grads.size() == 1 && wt == WireT::F32), "zero_src needs a single fp32 source");
  const int pm = pub_mode_of(pub, n);
  void* pp = pm ? pub->data_ptr() : nullptr;
  const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
  const double step_size = torch_mode ? lr / bc1 : lr * std::sqrt(bc2) / bc1;
  AdamHp h{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd, (float)step_size, (float)std::sqrt(bc2),
           (int)amsgrad, (int)torch_mode, (int)step};
  const uint8_t* cm = cmask_of(mask, n);
  int* cs = csteps_of(csteps, n);
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = grid_for(n >> 2);
  if (wt == WireT::F32)
    hipLaunchKernelGGL(k_adam<float>, grid, kBlock, 0, stream, s, (int)grads.size(), (float)gscale,
                       p.data_ptr<float>(), exp_avg.data_ptr<float>(), exp_avg_sq.data_ptr<float>(), xp, pp, pm,
                       (int)zero_src, n, h, cm, cs);
  else
    hipLaunchKernelGGL(k_adam<uint16_t>, grid, kBlock, 0, stream, s, (int)grads.size(), (float)gscale,
                       p.data_ptr<float>(), exp_avg.data_ptr<float>(), exp_avg_sq.data_ptr<float>(), xp, pp, pm,
                       (int)zero_src, n, h, cm, cs);
}

}  // namespace hipps
