// hipps — fused elementwise ops of the Llama block (SwiGLU gate, rotary position embedding).
//
// PyTorch's eager route for ``silu(w1 h) * w3 h`` is two forward kernels and four backward
// kernels over [tokens, ffn] bf16 tensors (silu, mul; mul x2, silu_backward, and the autocast
// bookkeeping), and ``_rope`` (strided halves, four multiplies, add / sub, stack) is seven
// kernels per q or k in each direction, with bf16 cos / sin tables and a bf16 rounding after
// every op.  Here each is ONE pass: 16-byte loads / stores of 8 bf16 per lane, fp32 math, one
// rounding per output.
//   swiglu fwd   c = silu(a) * b                             read a, b   write c
//   swiglu bwd   da = g * b * s * (1 + a (1 - s)), db = g * silu(a)   (s = sigmoid(a))
//   rope         y[2i] = x[2i] cos - x[2i+1] sin, y[2i+1] = x[2i] sin + x[2i+1] cos, per position
//                (sign = -1: the backward, rotation by -theta), fp32 cos / sin tables [S, hd/2]
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {

namespace {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ __launch_bounds__(kBlock) void k_swiglu_fwd(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                       uint16_t* __restrict__ c, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    const u32x4 va = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + i);
    const u32x4 vb = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + i);
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a0 = lo(va[j]), a1 = hi(va[j]);
      o[j] = pack_bf16x2(a0 * sigm(a0) * lo(vb[j]), a1 * sigm(a1) * hi(vb[j]));
    }
    reinterpret_cast<u32x4*>(c)[i] = o;
  }
}

__global__ __launch_bounds__(kBlock) void k_swiglu_bwd(const uint16_t* __restrict__ g, const uint16_t* __restrict__ a,
                                                       const uint16_t* __restrict__ b, uint16_t* __restrict__ da,
                                                       uint16_t* __restrict__ db, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    const u32x4 vg = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g) + i);
    const u32x4 va = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + i);
    const u32x4 vb = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b) + i);
    u32x4 oa, ob;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float r[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float x = h ? hi(va[j]) : lo(va[j]), y = h ? hi(vb[j]) : lo(vb[j]), gg = h ? hi(vg[j]) : lo(vg[j]);
        const float s = sigm(x);
        r[0][h] = gg * y * s * (1.f + x * (1.f - s));
        r[1][h] = gg * x * s;
      }
      oa[j] = pack_bf16x2(r[0][0], r[0][1]);
      ob[j] = pack_bf16x2(r[1][0], r[1][1]);
    }
    reinterpret_cast<u32x4*>(da)[i] = oa;
    reinterpret_cast<u32x4*>(db)[i] = ob;
  }
}

// Packed gate / up projection (one [rows, 2F] GEMM output: a = columns [0, F), b = [F, 2F)):
// c[m] = silu(a[m]) * b[m] with row strides (elements) ys for the input, cs for the output; the
// backward writes da / db straight into the packed [rows, 2F] gradient
__global__ __launch_bounds__(kBlock) void k_swiglu_fwd_rows(const uint16_t* __restrict__ y, int64_t ys, int F,
                                                            uint16_t* __restrict__ c, int64_t cs, int64_t rows) {
  const int w8 = F >> 3;
  const int64_t n8 = rows * w8;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    const int64_t m = i / w8;
    const int c0 = (int)(i - m * w8) * 8;
    const uint16_t* ya = y + m * ys + c0;
    const u32x4 va = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ya));
    const u32x4 vb = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ya + F));
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a0 = lo(va[j]), a1 = hi(va[j]);
      o[j] = pack_bf16x2(a0 * sigm(a0) * lo(vb[j]), a1 * sigm(a1) * hi(vb[j]));
    }
    *reinterpret_cast<u32x4*>(c + m * cs + c0) = o;
  }
}

__global__ __launch_bounds__(kBlock) void k_swiglu_bwd_rows(const uint16_t* __restrict__ g, int64_t gs,
                                                            const uint16_t* __restrict__ y, int64_t ys, int F,
                                                            uint16_t* __restrict__ dy, int64_t ds, int64_t rows) {
  const int w8 = F >> 3;
  const int64_t n8 = rows * w8;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    const int64_t m = i / w8;
    const int c0 = (int)(i - m * w8) * 8;
    const uint16_t* ya = y + m * ys + c0;
    const u32x4 vg = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g + m * gs + c0));
    const u32x4 va = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ya));
    const u32x4 vb = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ya + F));
    u32x4 oa, ob;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float r[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float x = h ? hi(va[j]) : lo(va[j]), yy = h ? hi(vb[j]) : lo(vb[j]), gg = h ? hi(vg[j]) : lo(vg[j]);
        const float sg = sigm(x);
        r[0][h] = gg * yy * sg * (1.f + x * (1.f - sg));
        r[1][h] = gg * x * sg;
      }
      oa[j] = pack_bf16x2(r[0][0], r[0][1]);
      ob[j] = pack_bf16x2(r[1][0], r[1][1]);
    }
    uint16_t* d = dy + m * ds + c0;
    *reinterpret_cast<u32x4*>(d) = oa;
    *reinterpret_cast<u32x4*>(d + F) = ob;
  }
}

// x, y: [rows = B*S, W = heads*hd] bf16 with row strides xs / ys (elements; in place allowed),
// row m is position m % S; cs, sn: fp32 [S, hd/2]
__global__ __launch_bounds__(kBlock) void k_rope(const uint16_t* x, uint16_t* y, const float* __restrict__ cs,
                                                 const float* __restrict__ sn, int64_t n8, int w8, int S, int hd,
                                                 float sign, int64_t xs, int64_t ys) {
  const int half = hd >> 1;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
    const int64_t m = i / w8;
    const int c0 = (int)(i - m * w8) * 8;
    const int s = (int)(m % S);
    const int p0 = (c0 % hd) >> 1;
    const float4 cv = *reinterpret_cast<const float4*>(cs + (int64_t)s * half + p0);
    const float4 sv = *reinterpret_cast<const float4*>(sn + (int64_t)s * half + p0);
    const float cc[4] = {cv.x, cv.y, cv.z, cv.w};
    const float ss[4] = {sign * sv.x, sign * sv.y, sign * sv.z, sign * sv.w};
    const u32x4 v = *reinterpret_cast<const u32x4*>(x + m * xs + c0);
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x0 = lo(v[j]), x1 = hi(v[j]);
      o[j] = pack_bf16x2(x0 * cc[j] - x1 * ss[j], x0 * ss[j] + x1 * cc[j]);
    }
    *reinterpret_cast<u32x4*>(y + m * ys + c0) = o;
  }
}

void check_bf16_flat(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), what,
              ": contiguous bf16 device tensor");
  TORCH_CHECK(t.numel() % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, what,
              ": numel % 8 == 0 and 16-byte aligned");
}
}  // namespace

void swiglu_forward(at::Tensor a, at::Tensor b, at::Tensor c) {
  check_bf16_flat(a, "swiglu a");
  check_bf16_flat(b, "swiglu b");
  check_bf16_flat(c, "swiglu c");
  TORCH_CHECK(a.numel() == b.numel() && a.numel() == c.numel(), "swiglu: sizes");
  const int64_t n8 = a.numel() / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(k_swiglu_fwd, grid_for(n8), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)a.data_ptr(), (const uint16_t*)b.data_ptr(), (uint16_t*)c.data_ptr(), n8);
}

void swiglu_backward(at::Tensor g, at::Tensor a, at::Tensor b, at::Tensor da, at::Tensor db) {
  for (auto* t : {&g, &a, &b, &da, &db}) check_bf16_flat(*t, "swiglu backward operand");
  TORCH_CHECK(g.numel() == a.numel() && a.numel() == b.numel() && da.numel() == a.numel() && db.numel() == a.numel(),
              "swiglu backward: sizes");
  const int64_t n8 = a.numel() / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(k_swiglu_bwd, grid_for(n8), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)g.data_ptr(), (const uint16_t*)a.data_ptr(), (const uint16_t*)b.data_ptr(),
                     (uint16_t*)da.data_ptr(), (uint16_t*)db.data_ptr(), n8);
}

// x, y: [B*S, W] (W = heads * hd); cs / sn fp32 [>= S, hd/2] contiguous
namespace {
// a [rows, W] bf16 view with contiguous rows of 16-byte multiples at a 16-byte aligned row stride
void check_rows(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.stride(1) == 1 &&
                  t.size(1) % 8 == 0 && t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              what, ": bf16 [rows, cols] with unit column stride, cols and row stride multiples of 8, 16-byte aligned");
}
}  // namespace

// c = silu(y[:, :F]) * y[:, F:] for a packed [rows, 2F] gate / up projection (c [rows, F])
void swiglu_rows_forward(at::Tensor y, at::Tensor c) {
  check_rows(y, "swiglu y");
  check_rows(c, "swiglu c");
  const int64_t rows = y.size(0), F = c.size(1);
  TORCH_CHECK(y.size(1) == 2 * F && c.size(0) == rows && F % 8 == 0, "swiglu: y [rows, 2F], c [rows, F]");
  if (rows == 0) return;
  hipLaunchKernelGGL(k_swiglu_fwd_rows, grid_for(rows * F / 8), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)y.data_ptr(), y.stride(0), (int)F, (uint16_t*)c.data_ptr(), c.stride(0), rows);
}

// dy [rows, 2F] (packed da | db) from g [rows, F] and the packed projection y
void swiglu_rows_backward(at::Tensor g, at::Tensor y, at::Tensor dy) {
  check_rows(g, "swiglu g");
  check_rows(y, "swiglu y");
  check_rows(dy, "swiglu dy");
  const int64_t rows = y.size(0), F = g.size(1);
  TORCH_CHECK(y.size(1) == 2 * F && dy.sizes() == y.sizes() && g.size(0) == rows, "swiglu backward: sizes");
  if (rows == 0) return;
  hipLaunchKernelGGL(k_swiglu_bwd_rows, grid_for(rows * F / 8), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)g.data_ptr(), g.stride(0), (const uint16_t*)y.data_ptr(), y.stride(0), (int)F,
                     (uint16_t*)dy.data_ptr(), dy.stride(0), rows);
}

void rope_apply(at::Tensor x, at::Tensor y, at::Tensor cs, at::Tensor sn, int64_t S, int64_t hd, double sign) {
  TORCH_CHECK(x.dim() == 2 && y.dim() == 2, "rope: x, y must be [B*S, heads*hd] (row strides allowed)");
  check_rows(x, "rope x");
  check_rows(y, "rope y");
  TORCH_CHECK(x.sizes() == y.sizes(), "rope: sizes");
  TORCH_CHECK(hd % 8 == 0 && S > 0, "rope: head dim must be a multiple of 8");
  const int64_t W = x.size(-1);
  TORCH_CHECK(W % hd == 0 && x.size(0) % S == 0, "rope: x must be [B*S, heads*hd]");
  for (auto* t : {&cs, &sn}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->dim() == 2 &&
                    t->size(0) >= S && t->size(1) == hd / 2,
                "rope: cos / sin tables must be fp32 [S, hd/2]");
  }
  const int64_t n8 = x.numel() / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(k_rope, grid_for(n8), kBlock, 0, c10::hip::getCurrentHIPStream(), (const uint16_t*)x.data_ptr(),
                     (uint16_t*)y.data_ptr(), cs.data_ptr<float>(), sn.data_ptr<float>(), n8, (int)(W / 8), (int)S,
                     (int)hd, (float)sign, x.stride(0), y.stride(0));
}

}  // namespace hipps
