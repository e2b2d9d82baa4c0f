// hipps — 3x3 / stride-2 / pad-1 max pooling for channels-last bf16 activations (the ResNet stem).
//
// PyTorch's NHWC max_pool2d backward scatters through int64 indices: 0.62 ms per ResNet-50 step
// at bs256 (profiles/bench_n1_steady_r1b.txt), the forward 0.26 ms.  Both passes are pure
// bandwidth (~0.5 GB each), i.e. ~0.1 ms each at HBM speed.
//
// forward : one lane = one output pixel x 8 channels (16 B loads/stores).  The argmax is kept as
//           a 4-bit tap code (kh*3 + kw) per channel, 8 codes in one uint32 per lane: 1/4 of the
//           output bytes instead of 4x (int64 indices).  Ties and NaNs follow PyTorch's rule
//           (first maximum in scan order; a NaN always wins), so values and gradients match it.
// BN variant (the ResNet stem): the input is a training BatchNorm's INPUT and each tap is read as
//           bf16(max(x * scale[c] + shift[c], 0)) -- the BN apply kernel's exact rounding -- so the
//           BN + ReLU output (411 MB at batch 256) is never written or re-read; pooled values and
//           tap codes are bit-identical to apply-then-pool.
// backward: gather form, no atomics: one lane = one input pixel x 8 channels.  With k=3, s=2,
//           p=1 an input row h lies in the windows oh in [h>>1, (h+1)>>1] (1 or 2 of them), so a
//           lane checks at most 4 windows' codes and sums the matching dy in fp32.
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdlib>

namespace hipps {

namespace {
__device__ __forceinline__ void ld8(const uint16_t* p, float v[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ void st8(uint16_t* p, const float v[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                            pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
}
}  // namespace

template <typename I, bool BN = false>
__global__ __launch_bounds__(kBlock) void k_maxpool3s2_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                           uint32_t* __restrict__ code, int64_t total, int H, int W,
                                                           int Ho, int Wo, int G, const float* __restrict__ scale,
                                                           const float* __restrict__ shift) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= total) return;
  // 32-bit index decomposition when the grid fits (the int64 div/mod sequence dominated)
  I p = (I)v;
  const int g = (int)(p % (I)G);
  p /= (I)G;
  const int wo = (int)(p % (I)Wo);
  p /= (I)Wo;
  const int ho = (int)(p % (I)Ho);
  const int64_t n = (int64_t)(p / (I)Ho);
  float m[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = -INFINITY;
    sc[j] = BN ? scale[g * 8 + j] : 1.f;
    sh[j] = BN ? shift[g * 8 + j] : 0.f;
  }
  // all 9 taps' loads issue together: out-of-range taps read a clamped (valid) address and are
  // skipped in the compare (a branch around each load serialised them: 159 us per batch-256 stem
  // pool, profiles/r4/r4e/steady.txt)
  float xv[9][8];
  bool ok[9];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int h = 2 * ho - 1 + kh;
    const int hc = min(max(h, 0), H - 1);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int w = 2 * wo - 1 + kw;
      const int wc = min(max(w, 0), W - 1);
      ok[kh * 3 + kw] = h >= 0 && h < H && w >= 0 && w < W;
      ld8(x + (((n * H + hc) * W + wc) * G + g) * 8, xv[kh * 3 + kw]);
    }
  }
  uint32_t c = 0;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    if (BN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[t][j] = bf16_to_f32(f32_to_bf16(fmaxf(fmaf(xv[t][j], sc[j], sh[j]), 0.f)));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (ok[t] && (xv[t][j] > m[j] || __builtin_isnan(xv[t][j]))) {
        m[j] = xv[t][j];
        c = (c & ~(15u << (4 * j))) | ((uint32_t)t << (4 * j));
      }
    }
  }
  st8(y + v * 8, m);
  code[v] = c;
}

// Two horizontally adjacent outputs per lane (wo = 2 wp, 2 wp + 1): their windows share the middle
// input column, so 3 x 5 taps are loaded (and, BN variant, normalised) instead of 2 x 9.  Per
// output the same scan order, ties and NaN rule as k_maxpool3s2_fwd, so values and codes are equal.
template <typename I, bool BN = false>
__global__ __launch_bounds__(kBlock) void k_maxpool3s2_fwd2(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                            uint32_t* __restrict__ code, int64_t total, int H, int W,
                                                            int Ho, int Wo, int G, const float* __restrict__ scale,
                                                            const float* __restrict__ shift) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= total) return;
  const int Wp = (Wo + 1) >> 1;
  I p = (I)v;
  const int g = (int)(p % (I)G);
  p /= (I)G;
  const int wp = (int)(p % (I)Wp);
  p /= (I)Wp;
  const int ho = (int)(p % (I)Ho);
  const int64_t n = (int64_t)(p / (I)Ho);
  const int wo0 = 2 * wp;
  const bool two = wo0 + 1 < Wo;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = BN ? scale[g * 8 + j] : 1.f;
    sh[j] = BN ? shift[g * 8 + j] : 0.f;
  }
  float xv[3][5][8];
  bool okr[3], okc[5];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int h = 2 * ho - 1 + kh;
    okr[kh] = h >= 0 && h < H;
    const int hc = min(max(h, 0), H - 1);
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const int w = 2 * wo0 - 1 + c;
      okc[c] = w >= 0 && w < W;
      const int wc = min(max(w, 0), W - 1);
      ld8(x + (((n * H + hc) * W + wc) * G + g) * 8, xv[kh][c]);
    }
  }
  if (BN) {
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int c = 0; c < 5; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          xv[kh][c][j] = bf16_to_f32(f32_to_bf16(fmaxf(fmaf(xv[kh][c][j], sc[j], sh[j]), 0.f)));
  }
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    if (o == 1 && !two) break;
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    uint32_t cd = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int c = 2 * o + kw;
        const bool ok = okr[kh] && okc[c];
        const uint32_t t = kh * 3 + kw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (ok && (xv[kh][c][j] > m[j] || __builtin_isnan(xv[kh][c][j]))) {
            m[j] = xv[kh][c][j];
            cd = (cd & ~(15u << (4 * j))) | (t << (4 * j));
          }
        }
      }
    }
    const int64_t out = ((n * Ho + ho) * Wo + wo0 + o) * G + g;
    st8(y + out * 8, m);
    code[out] = cd;
  }
}

template <typename I>
__global__ __launch_bounds__(kBlock) void k_maxpool3s2_bwd(const uint16_t* __restrict__ dy,
                                                           const uint32_t* __restrict__ code,
                                                           uint16_t* __restrict__ dx, int64_t total, int H, int W,
                                                           int Ho, int Wo, int G) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= total) return;
  I p = (I)v;
  const int g = (int)(p % (I)G);
  p /= (I)G;
  const int w = (int)(p % (I)W);
  p /= (I)W;
  const int h = (int)(p % (I)H);
  const int64_t n = (int64_t)(p / (I)H);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  // candidate windows (h>>1 | (h>>1)+1) x (w>>1 | (w>>1)+1), the +1 ones only for odd h / w inside
  // the pooled map: a static 2x2 with predicates, so the 4 code / dy loads issue together (the
  // data-dependent loop serialised them: 280 us per batch-256 stem pool backward, profiles/r4/r4e/
  // steady.txt).  Same (oh, ow) summation order as that loop; absent windows add +0.
  const int oh0 = h >> 1, ow0 = w >> 1;
  const bool h1 = (h & 1) && oh0 + 1 < Ho, w1 = (w & 1) && ow0 + 1 < Wo;
  uint32_t c[4];
  uint4 d[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool okk = (!(k >> 1) || h1) && (!(k & 1) || w1);
    const int64_t o = okk ? ((n * Ho + oh0 + (k >> 1)) * Wo + ow0 + (k & 1)) * G + g : 0;
    const uint32_t cv = code[o];
    d[k] = *reinterpret_cast<const uint4*>(dy + o * 8);
    c[k] = okk ? cv : 0xffffffffu;  // tap 15 never matches
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t t = (uint32_t)((h - 2 * (oh0 + (k >> 1)) + 1) * 3 + (w - 2 * (ow0 + (k & 1)) + 1));
    const uint32_t dw[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dv = __uint_as_float(j & 1 ? dw[j >> 1] & 0xffff0000u : dw[j >> 1] << 16);
      acc[j] += ((c[k] >> (4 * j)) & 15u) == t ? dv : 0.f;
    }
  }
  st8(dx + v * 8, acc);
}

// x: [N, C, H, W] channels-last bf16 (C % 8 == 0); y: [N, C, Ho, Wo] channels-last bf16;
// code: int32 [N*Ho*Wo*C/8] (4-bit tap codes).  scale / shift (optional, f32 [C]): pool
// relu(x * scale + shift) instead of x (x is a BatchNorm input, see the BN variant above).
void maxpool3s2_forward(at::Tensor x, at::Tensor y, at::Tensor code, c10::optional<at::Tensor> scale,
                        c10::optional<at::Tensor> shift) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool: x must be channels-last bf16 NCHW");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0 && H >= 1 && W >= 1, "maxpool: C % 8 == 0");
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.dim() == 4 && y.size(0) == N && y.size(1) == C &&
                  y.size(2) == Ho && y.size(3) == Wo && y.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool: y must be channels-last bf16 [N, C, Ho, Wo]");
  const int64_t total = N * Ho * Wo * (C / 8);
  TORCH_CHECK(code.is_cuda() && code.scalar_type() == at::kInt && code.is_contiguous() && code.numel() == total,
              "maxpool: code must be int32[N*Ho*Wo*C/8]");
  for (const at::Tensor* t : {&x, &y, &code})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "maxpool: 16-byte aligned tensors");
  TORCH_CHECK(x.numel() < (int64_t(1) << 40) && (total + kBlock - 1) / kBlock < (int64_t(1) << 31), "maxpool: size");
  const bool bn = scale.has_value() && scale->defined();
  const float *sc = nullptr, *sh = nullptr;
  if (bn) {
    TORCH_CHECK(shift.has_value() && shift->defined(), "maxpool: scale needs shift");
    for (const c10::optional<at::Tensor>* v : {&scale, &shift})
      TORCH_CHECK((*v)->is_cuda() && (*v)->scalar_type() == at::kFloat && (*v)->is_contiguous() && (*v)->numel() == C,
                  "maxpool: scale / shift must be f32 [C]");
    sc = scale->data_ptr<float>();
    sh = shift->data_ptr<float>();
  }
  if (total == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  // two outputs per lane (k_maxpool3s2_fwd2); HIPPS_POOL_PAIR=0: one per lane
  static const bool pair = [] {
    const char* e = std::getenv("HIPPS_POOL_PAIR");
    return !(e && e[0] == '0');
  }();
  const int64_t items = pair ? N * Ho * ((Wo + 1) / 2) * (C / 8) : total;
  const int grid = (int)((items + kBlock - 1) / kBlock);
#define HIPPS_MP(K, I, B)                                                                                     \
  hipLaunchKernelGGL((K<I, B>), grid, kBlock, 0, stream, (const uint16_t*)x.data_ptr(), (uint16_t*)y.data_ptr(), \
                     (uint32_t*)code.data_ptr(), items, (int)H, (int)W, (int)Ho, (int)Wo, (int)(C / 8), sc, sh)
  if (pair) {
    if (total < (int64_t(1) << 31)) {
      if (bn) HIPPS_MP(k_maxpool3s2_fwd2, uint32_t, true); else HIPPS_MP(k_maxpool3s2_fwd2, uint32_t, false);
    } else {
      if (bn) HIPPS_MP(k_maxpool3s2_fwd2, int64_t, true); else HIPPS_MP(k_maxpool3s2_fwd2, int64_t, false);
    }
  } else if (total < (int64_t(1) << 31)) {
    if (bn) HIPPS_MP(k_maxpool3s2_fwd, uint32_t, true); else HIPPS_MP(k_maxpool3s2_fwd, uint32_t, false);
  } else {
    if (bn) HIPPS_MP(k_maxpool3s2_fwd, int64_t, true); else HIPPS_MP(k_maxpool3s2_fwd, int64_t, false);
  }
#undef HIPPS_MP
}

// dy: [N, C, Ho, Wo] channels-last bf16; dx: [N, C, H, W] channels-last bf16 (fully written).
void maxpool3s2_backward(at::Tensor dy, at::Tensor code, at::Tensor dx) {
  TORCH_CHECK(dx.is_cuda() && dx.scalar_type() == at::kBFloat16 && dx.dim() == 4 &&
                  dx.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool bwd: dx must be channels-last bf16");
  const int64_t N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  TORCH_CHECK(C % 8 == 0, "maxpool bwd: C % 8 == 0");
  const int64_t Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N &&
                  dy.size(1) == C && dy.size(2) == Ho && dy.size(3) == Wo &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool bwd: dy must be channels-last bf16");
  TORCH_CHECK(code.is_cuda() && code.scalar_type() == at::kInt && code.is_contiguous() &&
                  code.numel() == N * Ho * Wo * (C / 8), "maxpool bwd: code size");
  for (const at::Tensor* t : {&dy, &dx, &code})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "maxpool bwd: 16-byte aligned tensors");
  const int64_t total = N * H * W * (C / 8);
  TORCH_CHECK(dx.numel() < (int64_t(1) << 40) && (total + kBlock - 1) / kBlock < (int64_t(1) << 31),
              "maxpool bwd: size");
  if (total == 0) return;
  const int grid = (int)((total + kBlock - 1) / kBlock);
  auto stream = c10::hip::getCurrentHIPStream();
  if (total < (int64_t(1) << 31))
    hipLaunchKernelGGL(k_maxpool3s2_bwd<uint32_t>, grid, kBlock, 0, stream, (const uint16_t*)dy.data_ptr(),
                       (const uint32_t*)code.data_ptr(), (uint16_t*)dx.data_ptr(), total, (int)H, (int)W, (int)Ho,
                       (int)Wo, (int)(C / 8));
  else
    hipLaunchKernelGGL(k_maxpool3s2_bwd<int64_t>, grid, kBlock, 0, stream, (const uint16_t*)dy.data_ptr(),
                       (const uint32_t*)code.data_ptr(), (uint16_t*)dx.data_ptr(), total, (int)H, (int)W, (int)Ho,
                       (int)Wo, (int)(C / 8));
}

}  // namespace hipps
