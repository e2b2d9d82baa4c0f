// hipps — LayerNorm (BERT's 25 norms per step) and RMSNorm (Llama) over the last dim of [rows, D].
//
// PyTorch's route under autocast (hipps/models/transformer.py _ln) casts the fp32 weight and bias
// to bf16 every forward, runs the forward at ~1.7 TB/s, and the backward as an input-gradient
// kernel (~1.5 TB/s) plus two gamma/beta reduction kernels and the casts of their results.  Here:
//   forward   one wave per row, the row held in registers (D/8 16-byte chunks over 64 lanes),
//             two-pass mean / variance in fp32, fp32 weight and bias read directly; writes y
//             (bf16) and the row's mean / rstd (fp32) for the backward
//   backward  one wave per row as well: dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy w;
//             each workgroup also sums dy xhat and dy over its rows per column into a partial
//             row, and a second kernel folds the partial rows in a fixed order into the fp32
//             weight / bias gradients (deterministic)
#include "common.h"

#include <type_traits>

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <algorithm>

namespace hipps {

namespace {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kLnWaves = 4;  // rows in flight per workgroup

template <int N> __device__ __forceinline__ float wsum_n(float v) {  // sum over aligned groups of N lanes
#pragma unroll
  for (int o = N / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(v[j] << 16);
    f[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
  }
}

// NC: 16-byte chunks per lane (D <= 512 * NC; D <= 2048 keeps the backward's LDS at <= 64 KB)
template <int NC>
__global__ __launch_bounds__(64 * kLnWaves) void k_ln_fwd(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, uint16_t* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nch = D >> 3;
  const uint16_t* xr = x + row * D;
  float v[NC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      unpack8(*reinterpret_cast<const u32x4*>(xr + ch * 8), v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  const float mu = wsum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (lane + 64 * c < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[c][j] - mu;
        q += d * d;
      }
    }
  }
  const float rs = rsqrtf(wsum(q) / D + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      const float4 w0 = *reinterpret_cast<const float4*>(w + ch * 8), w1 = *reinterpret_cast<const float4*>(w + ch * 8 + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(b + ch * 8), b1 = *reinterpret_cast<const float4*>(b + ch * 8 + 4);
      const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = pack_bf16x2((v[c][2 * j] - mu) * rs * ww[2 * j] + bb[2 * j],
                           (v[c][2 * j + 1] - mu) * rs * ww[2 * j + 1] + bb[2 * j + 1]);
      *reinterpret_cast<u32x4*>(y + row * D + ch * 8) = o;
    }
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

// rows [blockIdx.x * rpb, +rpb): dx per row; per-column sums of dy * xhat and dy over those rows
// -> part[blockIdx.x] (2 x D floats: dgamma partial, dbeta partial)
// DXS: a third column sum, of the bf16 dx written (the bias gradient of the Linear whose output
// this LayerNorm normalised -- BERT's attn_out / out: their colsum pass over dx is saved)
// LPR (lanes per row) 32: each half-wave takes a row -- D = 768's 96 chunks as 3 per lane on
// 32 lanes instead of 2 on half of 64 (half the lanes idle in the second chunk)
template <int NC, bool DXS = false, int LPR = 64>
__global__ __launch_bounds__(64 * kLnWaves) void k_ln_bwd(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          const float* __restrict__ w, uint16_t* __restrict__ dx,
                                                          float* __restrict__ part, int64_t R, int D, int rpb) {
  constexpr int NK = DXS ? 3 : 2;
  extern __shared__ float red[];  // [kLnWaves][NK][D]
  const int lane64 = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int RPW = 64 / LPR;                 // rows per wave at a time
  const int lane = lane64 & (LPR - 1), hrow = lane64 / LPR;
  const int nch = D >> 3;
  float ww[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + LPR * c;
    const int cc = ch < nch ? ch : 0;
    const float4 w0 = *reinterpret_cast<const float4*>(w + cc * 8), w1 = *reinterpret_cast<const float4*>(w + cc * 8 + 4);
    ww[c][0] = w0.x; ww[c][1] = w0.y; ww[c][2] = w0.z; ww[c][3] = w0.w;
    ww[c][4] = w1.x; ww[c][5] = w1.y; ww[c][6] = w1.z; ww[c][7] = w1.w;
  }
  float dg[NC][8], db[NC][8], dsx[DXS ? NC : 1][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[c][j] = db[c][j] = 0.f;
#pragma unroll
  for (int c = 0; c < (DXS ? NC : 1); ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dsx[c][j] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < R ? r0 + rpb : R;
  // software pipelined: the next row's x / dy / statistics are in flight while this row is
  // reduced and written (one row per wave at a time left each wave a chain of HBM round trips:
  // 30 us per BERT-base call, ~2.5 TB/s)
  u32x4 nx[NC], ndy[NC];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t row) {
    if (row < r1) {
      nmu = mean[row];
      nrs = rstd[row];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = lane + LPR * c;
        if (ch < nch) {
          nx[c] = *reinterpret_cast<const u32x4*>(x + row * D + ch * 8);
          ndy[c] = *reinterpret_cast<const u32x4*>(dy + row * D + ch * 8);
        }
      }
    }
  };
  fetch(r0 + wv * RPW + hrow);
  for (int64_t row = r0 + wv * RPW + hrow; row < r1; row += kLnWaves * RPW) {
    const float mu = nmu, rs = nrs;
    u32x4 cx[NC], cdy[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      cx[c] = nx[c];
      cdy[c] = ndy[c];
    }
    fetch(row + kLnWaves * RPW);
    float xh[NC][8], g[NC][8], gy[NC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + LPR * c;
      if (ch < nch) {
        float xv[8];
        unpack8(cx[c], xv);
        unpack8(cdy[c], gy[c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xv[j] - mu) * rs;
          g[c][j] = gy[c][j] * ww[c][j];
          s1 += g[c][j];
          s2 += g[c][j] * xh[c][j];
        }
      }
    }
    const float m1 = wsum_n<LPR>(s1) / D, m2 = wsum_n<LPR>(s2) / D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + LPR * c;
      if (ch < nch) {
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = pack_bf16x2(rs * (g[c][2 * j] - m1 - xh[c][2 * j] * m2),
                             rs * (g[c][2 * j + 1] - m1 - xh[c][2 * j + 1] * m2));
        *reinterpret_cast<u32x4*>(dx + row * D + ch * 8) = o;
        if constexpr (DXS) {  // the stored (bf16-rounded) values, as a colsum over dx would read them
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            dsx[DXS ? c : 0][2 * j] += __uint_as_float(o[j] << 16);
            dsx[DXS ? c : 0][2 * j + 1] += __uint_as_float(o[j] & 0xffff0000u);
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          dg[c][j] += gy[c][j] * xh[c][j];
          db[c][j] += gy[c][j];
        }
      }
    }
  }
  // fold the waves' column sums in a fixed order (LPR 32: the two half-waves' first, lane l + l^32)
  if constexpr (LPR == 32) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dg[c][j] += __shfl_xor(dg[c][j], 32, 64);
        db[c][j] += __shfl_xor(db[c][j], 32, 64);
        if constexpr (DXS) dsx[DXS ? c : 0][j] += __shfl_xor(dsx[DXS ? c : 0][j], 32, 64);
      }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + LPR * c;
    if (ch < nch && hrow == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wv * NK) * D + ch * 8 + j] = dg[c][j];
        red[(wv * NK + 1) * D + ch * 8 + j] = db[c][j];
        if constexpr (DXS) red[(wv * NK + 2) * D + ch * 8 + j] = dsx[DXS ? c : 0][j];
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NK * D; i += 64 * kLnWaves) {
    const int k = i / D, col = i - k * D;
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kLnWaves; ++q) a += red[(q * NK + k) * D + col];
    part[(int64_t)blockIdx.x * NK * D + i] = a;
  }
}

// out[k * D + col] = sum_p part[p][k][col] (k = 0: dgamma, 1: dbeta when nk == 2), fixed order.
// 64 columns per workgroup of 16 waves; wave w sums partial rows w, w + 16, ... with 8 loads in
// flight (D = 768 gives only 24 workgroups: with 4 waves of 4 loads each the fold was a chain of
// dependent HBM round trips, 24 us per call on BERT-base)
constexpr int kFoldWaves = 16;
__global__ __launch_bounds__(64 * kFoldWaves) void k_ln_fold(const float* __restrict__ part, int P, int D, int nk,
                                                             float* __restrict__ dw, float* __restrict__ dbias,
                                                             float* __restrict__ dsum = nullptr) {
  __shared__ float red[kFoldWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;  // over nk * D
  const int ii = i < nk * D ? i : 0;
  const int64_t rs = (int64_t)nk * D;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int p = wv;
  for (; p + 7 * kFoldWaves < P; p += 8 * kFoldWaves) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = part[(int64_t)(p + kFoldWaves * j) * rs + ii];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  for (; p < P; p += kFoldWaves) acc[0] += part[(int64_t)p * rs + ii];
  red[wv][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (wv == 0 && i < nk * D) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kFoldWaves; ++q) a += red[q][lane];
    if (i < D) dw[i] = a;
    else if (i < 2 * D) dbias[i - D] = a;
    else dsum[i - 2 * D] = a;
  }
}

// ---- RMSNorm (Llama): y = x * rsqrt(mean(x^2) + eps) * w, x fp32 (the residual stream) or bf16 --
template <typename TX> struct Ld8;
template <> struct Ld8<float> {
  __device__ __forceinline__ static void load(const float* p, float* f) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  __device__ __forceinline__ static void store(float* p, const float* f) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
  }
};
template <> struct Ld8<uint16_t> {
  __device__ __forceinline__ static void load(const uint16_t* p, float* f) { unpack8(*reinterpret_cast<const u32x4*>(p), f); }
  __device__ __forceinline__ static void store(uint16_t* p, const float* f) {
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(f[2 * j], f[2 * j + 1]);
    *reinterpret_cast<u32x4*>(p) = o;
  }
};

__device__ __forceinline__ void load_w8(const float* w, float* f) { Ld8<float>::load(w, f); }

// NC <= 8: D <= 4096
template <int NC, typename TX>
__global__ __launch_bounds__(64 * kLnWaves) void k_rms_fwd(const TX* __restrict__ x, const float* __restrict__ w,
                                                           uint16_t* __restrict__ y, float* __restrict__ rstd_out,
                                                           int64_t R, int D, float eps,
                                                           const uint16_t* __restrict__ addy,
                                                           float* __restrict__ xsum) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kLnWaves + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nch = D >> 3;
  float v[NC][8];
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      Ld8<TX>::load(x + row * D + ch * 8, v[c]);
      if (addy) {  // fused residual add: x + addy (bf16) is normalised and written out (fp32)
        float a[8];
        unpack8(*reinterpret_cast<const u32x4*>(addy + row * D + ch * 8), a);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += a[j];
        Ld8<float>::store(xsum + row * D + ch * 8, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) q += v[c][j] * v[c][j];
    }
  }
  const float rs = rsqrtf(wsum(q) / D + eps);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float ww[8], o[8];
      load_w8(w + ch * 8, ww);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rs * ww[j];
      Ld8<uint16_t>::store(y + row * D + ch * 8, o);
    }
  }
  if (lane == 0) rstd_out[row] = rs;
}

// dx = rs (g - xhat mean(g xhat)), g = dy w, xhat = x rs; dw partial = sum_rows dy xhat.  Two
// passes over each row (the second re-reads it from cache) keep the registers to w + dw sums.
template <int NC, typename TX>
__global__ __launch_bounds__(64 * kLnWaves) void k_rms_bwd(const uint16_t* __restrict__ dy, const TX* __restrict__ x,
                                                           const float* __restrict__ rstd, const float* __restrict__ w,
                                                           TX* __restrict__ dx, float* __restrict__ part, int64_t R,
                                                           int D, int rpb, const float* __restrict__ dres,
                                                           uint16_t* __restrict__ dx16) {
  extern __shared__ float red[];  // [kLnWaves][D]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nch = D >> 3;
  float ww[NC][8], dg[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    load_w8(w + (ch < nch ? ch : 0) * 8, ww[c]);
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[c][j] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < R ? r0 + rpb : R;
  // fp32 rows of D <= 2048 (Llama-3-1B): the row stays in registers between the two passes and
  // the next row's x / dy / rstd are in flight while this one is reduced and written (the
  // two-pass re-read form ran ~2.9 TB/s); D = 4096 keeps the re-read form (register budget)
  constexpr bool REG = NC <= 4 && std::is_same<TX, float>::value;
  if constexpr (REG) {
    float4 nx[NC][2];
    u32x4 ndy[NC];
    float nrs = 0.f;
    auto fetch = [&](int64_t row) {
      if (row < r1) {
        nrs = rstd[row];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int ch = lane + 64 * c;
          if (ch < nch) {
            const float* xp = reinterpret_cast<const float*>(x) + row * D + ch * 8;
            nx[c][0] = *reinterpret_cast<const float4*>(xp);
            nx[c][1] = *reinterpret_cast<const float4*>(xp + 4);
            ndy[c] = *reinterpret_cast<const u32x4*>(dy + row * D + ch * 8);
          }
        }
      }
    };
    fetch(r0 + wv);
    for (int64_t row = r0 + wv; row < r1; row += kLnWaves) {
      const float rs = nrs;
      float xv[NC][8], gy[NC][8];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        xv[c][0] = nx[c][0].x; xv[c][1] = nx[c][0].y; xv[c][2] = nx[c][0].z; xv[c][3] = nx[c][0].w;
        xv[c][4] = nx[c][1].x; xv[c][5] = nx[c][1].y; xv[c][6] = nx[c][1].z; xv[c][7] = nx[c][1].w;
        unpack8(ndy[c], gy[c]);
      }
      fetch(row + kLnWaves);
      float gr[NC][8];
      if (dres) {  // this row's residual gradient, issued before the reduction
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int ch = lane + 64 * c;
          if (ch < nch) Ld8<float>::load(dres + row * D + ch * 8, gr[c]);
        }
      }
      float s2 = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (lane + 64 * c < nch) {
#pragma unroll
          for (int j = 0; j < 8; ++j) s2 += gy[c][j] * ww[c][j] * xv[c][j] * rs;
        }
      }
      const float m2 = wsum(s2) / D;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = lane + 64 * c;
        if (ch < nch) {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xh = xv[c][j] * rs;
            o[j] = rs * (gy[c][j] * ww[c][j] - xh * m2);
            dg[c][j] += gy[c][j] * xh;
          }
          if (dres) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += gr[c][j];
          }
          Ld8<TX>::store(dx + row * D + ch * 8, o);
          if (dx16) Ld8<uint16_t>::store(dx16 + row * D + ch * 8, o);
        }
      }
    }
  }
  for (int64_t row = r0 + wv; !REG && row < r1; row += kLnWaves) {
    const float rs = rstd[row];
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        float xv[8], gy[8];
        Ld8<TX>::load(x + row * D + ch * 8, xv);
        unpack8(*reinterpret_cast<const u32x4*>(dy + row * D + ch * 8), gy);
#pragma unroll
        for (int j = 0; j < 8; ++j) s2 += gy[j] * ww[c][j] * xv[j] * rs;
      }
    }
    const float m2 = wsum(s2) / D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        float xv[8], gy[8], o[8];
        Ld8<TX>::load(x + row * D + ch * 8, xv);
        unpack8(*reinterpret_cast<const u32x4*>(dy + row * D + ch * 8), gy);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = xv[j] * rs;
          o[j] = rs * (gy[j] * ww[c][j] - xh * m2);
          dg[c][j] += gy[j] * xh;
        }
        if (dres) {  // the residual stream's own gradient joins here (fused residual add backward)
          float g[8];
          Ld8<float>::load(dres + row * D + ch * 8, g);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += g[j];
        }
        Ld8<TX>::store(dx + row * D + ch * 8, o);
        if (dx16) Ld8<uint16_t>::store(dx16 + row * D + ch * 8, o);  // bf16 twin for the bf16 branch
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wv * D + ch * 8 + j] = dg[c][j];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += 64 * kLnWaves) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kLnWaves; ++q) a += red[q * D + i];
    part[(int64_t)blockIdx.x * D + i] = a;
  }
}

void ln_check(const at::Tensor& x, int64_t D, int64_t dmax = 2048) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "layer_norm: contiguous bf16");
  TORCH_CHECK(D % 8 == 0 && D >= 8 && D <= dmax && x.numel() % D == 0, "norm: D % 8 == 0, D <= ", dmax);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "layer_norm: 16-byte aligned");
}

void ln_param_check(const at::Tensor& p, int64_t D, const char* what) {
  TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat && p.is_contiguous() && p.numel() == D &&
                  reinterpret_cast<uintptr_t>(p.data_ptr()) % 16 == 0,
              "layer_norm: ", what, " must be a 16-byte aligned fp32 [D]");
}
}  // namespace

void ln_forward(at::Tensor x, at::Tensor w, at::Tensor b, at::Tensor y, at::Tensor mean, at::Tensor rstd, double eps) {
  const int64_t D = x.size(-1);
  ln_check(x, D);
  ln_check(y, D);
  ln_param_check(w, D, "weight");
  ln_param_check(b, D, "bias");
  const int64_t R = x.numel() / D;
  TORCH_CHECK(y.numel() == x.numel() && mean.numel() == R && rstd.numel() == R && mean.scalar_type() == at::kFloat &&
                  rstd.scalar_type() == at::kFloat,
              "layer_norm: output sizes");
  if (R == 0) return;
  const int grid = (int)((R + kLnWaves - 1) / kLnWaves);
  auto st = c10::hip::getCurrentHIPStream();
  const int nc = (int)((D / 8 + 63) / 64);
#define HIPPS_LNF(NCc)                                                                                              \
  hipLaunchKernelGGL(k_ln_fwd<NCc>, grid, 64 * kLnWaves, 0, st, (const uint16_t*)x.data_ptr(), w.data_ptr<float>(), \
                     b.data_ptr<float>(), (uint16_t*)y.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), R,   \
                     (int)D, (float)eps)
  if (nc <= 1) HIPPS_LNF(1);
  else if (nc <= 2) HIPPS_LNF(2);
  else HIPPS_LNF(4);
#undef HIPPS_LNF
}

// dxsum (optional): fp32 [D] column sum of the bf16 dx written (a Linear's bias gradient)
void ln_backward(at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor rstd, at::Tensor w, at::Tensor dx,
                 at::Tensor dw, at::Tensor db, c10::optional<at::Tensor> dxsum) {
  const int64_t D = x.size(-1);
  ln_check(x, D);
  ln_check(dy, D);
  ln_check(dx, D);
  ln_param_check(w, D, "weight");
  ln_param_check(dw, D, "weight gradient");
  ln_param_check(db, D, "bias gradient");
  const int64_t R = x.numel() / D;
  TORCH_CHECK(dy.numel() == x.numel() && dx.numel() == x.numel() && mean.numel() == R && rstd.numel() == R,
              "layer_norm backward: sizes");
  if (R == 0) {
    dw.zero_();
    db.zero_();
    return;
  }
  // partial rows: enough workgroups to fill the chip, >= 16 rows each
  int64_t P = std::min<int64_t>(1024, std::max<int64_t>(1, R / 16));
  const int rpb = (int)((R + P - 1) / P);
  P = (R + rpb - 1) / rpb;
  const bool dxs = dxsum.has_value() && dxsum->defined();
  if (dxs) ln_param_check(*dxsum, D, "dx column sum");
  const int nk = dxs ? 3 : 2;
  at::Tensor part = at::empty({P, nk, D}, dw.options());
  auto st = c10::hip::getCurrentHIPStream();
  const size_t lds = (size_t)kLnWaves * nk * D * sizeof(float);
  const int nc = (int)((D / 8 + 63) / 64);
#define HIPPS_LNB(NCc, DX)                                                                                            \
  hipLaunchKernelGGL((k_ln_bwd<NCc, DX>), (int)P, 64 * kLnWaves, lds, st, (const uint16_t*)dy.data_ptr(),            \
                     (const uint16_t*)x.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(), w.data_ptr<float>(), \
                     (uint16_t*)dx.data_ptr(), part.data_ptr<float>(), R, (int)D, rpb)
  // opt-in (HIPPS_LN_HALF=1): a row per half-wave, 3 chunks per lane for D 520..768 -- measured
  // slower in the BERT-base step (803.4 / 804.0 k vs 813.4 / 813.8 k tokens/s, same box,
  // profiles/r6/ab_ln_half/): the 64-lane form's idle half-chunk costs less than the half-wave
  // form's extra row state and cross-half fold
  static const bool half = [] {
    const char* e = std::getenv("HIPPS_LN_HALF");
    return e && e[0] == '1';
  }();
  if (half && D / 8 > 64 && D / 8 <= 96) {  // D 520..768: a row per half-wave, 3 chunks per lane
    if (dxs)
      hipLaunchKernelGGL((k_ln_bwd<3, true, 32>), (int)P, 64 * kLnWaves, lds, st, (const uint16_t*)dy.data_ptr(),
                         (const uint16_t*)x.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                         w.data_ptr<float>(), (uint16_t*)dx.data_ptr(), part.data_ptr<float>(), R, (int)D, rpb);
    else
      hipLaunchKernelGGL((k_ln_bwd<3, false, 32>), (int)P, 64 * kLnWaves, lds, st, (const uint16_t*)dy.data_ptr(),
                         (const uint16_t*)x.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                         w.data_ptr<float>(), (uint16_t*)dx.data_ptr(), part.data_ptr<float>(), R, (int)D, rpb);
  } else if (dxs) {
    if (nc <= 1) HIPPS_LNB(1, true);
    else if (nc <= 2) HIPPS_LNB(2, true);
    else HIPPS_LNB(4, true);
  } else {
    if (nc <= 1) HIPPS_LNB(1, false);
    else if (nc <= 2) HIPPS_LNB(2, false);
    else HIPPS_LNB(4, false);
  }
#undef HIPPS_LNB
  hipLaunchKernelGGL(k_ln_fold, (int)((nk * D + 63) / 64), 64 * kFoldWaves, 0, st, part.data_ptr<float>(), (int)P, (int)D,
                     nk, dw.data_ptr<float>(), db.data_ptr<float>(), dxs ? dxsum->data_ptr<float>() : nullptr);
}

// x: fp32 or bf16 [rows, D] (D % 8 == 0, D <= 4096); y bf16; rstd fp32 [rows]
// add (optional): bf16 [rows, D] added to x (fp32) first; the sum is written to xsum (fp32)
void rms_forward(at::Tensor x, at::Tensor w, at::Tensor y, at::Tensor rstd, double eps, c10::optional<at::Tensor> add,
                 c10::optional<at::Tensor> xsum) {
  const int64_t D = x.size(-1);
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16) && x.is_contiguous() &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "rms_norm: x must be a contiguous 16-byte aligned fp32 / bf16 device tensor");
  TORCH_CHECK(D % 8 == 0 && D >= 8 && D <= 4096, "rms_norm: D % 8 == 0, D <= 4096");
  ln_check(y, D, 4096);
  ln_param_check(w, D, "weight");
  const int64_t R = x.numel() / D;
  TORCH_CHECK(y.numel() == x.numel() && rstd.numel() == R && rstd.scalar_type() == at::kFloat, "rms_norm: sizes");
  const uint16_t* addp = nullptr;
  float* xsp = nullptr;
  if (add.has_value()) {
    TORCH_CHECK(x.scalar_type() == at::kFloat && xsum.has_value(), "rms_norm(add): fp32 x and an xsum output");
    ln_check(*add, D, 4096);
    TORCH_CHECK(add->numel() == x.numel() && xsum->numel() == x.numel() && xsum->scalar_type() == at::kFloat &&
                    xsum->is_contiguous() && reinterpret_cast<uintptr_t>(xsum->data_ptr()) % 16 == 0,
                "rms_norm(add): add / xsum sizes");
    addp = (const uint16_t*)add->data_ptr();
    xsp = xsum->data_ptr<float>();
  }
  if (R == 0) return;
  const int grid = (int)((R + kLnWaves - 1) / kLnWaves);
  auto st = c10::hip::getCurrentHIPStream();
  const int nc = (int)((D / 8 + 63) / 64);
  const bool f32 = x.scalar_type() == at::kFloat;
#define HIPPS_RMSF(NCc)                                                                                                \
  do {                                                                                                                 \
    if (f32)                                                                                                           \
      hipLaunchKernelGGL((k_rms_fwd<NCc, float>), grid, 64 * kLnWaves, 0, st, x.data_ptr<float>(), w.data_ptr<float>(), \
                         (uint16_t*)y.data_ptr(), rstd.data_ptr<float>(), R, (int)D, (float)eps, addp, xsp);        \
    else                                                                                                               \
      hipLaunchKernelGGL((k_rms_fwd<NCc, uint16_t>), grid, 64 * kLnWaves, 0, st, (const uint16_t*)x.data_ptr(),        \
                         w.data_ptr<float>(), (uint16_t*)y.data_ptr(), rstd.data_ptr<float>(), R, (int)D, (float)eps,   \
                         nullptr, nullptr);                                                                            \
  } while (0)
  if (nc <= 1) HIPPS_RMSF(1);
  else if (nc <= 2) HIPPS_RMSF(2);
  else if (nc <= 4) HIPPS_RMSF(4);
  else HIPPS_RMSF(8);
#undef HIPPS_RMSF
}

// dy bf16; x / dx fp32 or bf16 (same dtype); dw fp32 [D]
// dres (optional, fp32 x only): added to dx; dx16 (optional): a bf16 copy of the final dx
void rms_backward(at::Tensor dy, at::Tensor x, at::Tensor rstd, at::Tensor w, at::Tensor dx, at::Tensor dw,
                  c10::optional<at::Tensor> dres, c10::optional<at::Tensor> dx16) {
  const int64_t D = x.size(-1);
  TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16) && x.is_contiguous() &&
                  dx.scalar_type() == x.scalar_type() && dx.is_contiguous() && dx.numel() == x.numel() &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dx.data_ptr()) % 16 == 0,
              "rms_norm backward: x / dx");
  TORCH_CHECK(D % 8 == 0 && D >= 8 && D <= 4096, "rms_norm: D % 8 == 0, D <= 4096");
  ln_check(dy, D, 4096);
  ln_param_check(w, D, "weight");
  ln_param_check(dw, D, "weight gradient");
  const int64_t R = x.numel() / D;
  TORCH_CHECK(dy.numel() == x.numel() && rstd.numel() == R, "rms_norm backward: sizes");
  const float* dresp = nullptr;
  uint16_t* dx16p = nullptr;
  if (dres.has_value()) {
    TORCH_CHECK(x.scalar_type() == at::kFloat && dres->scalar_type() == at::kFloat && dres->is_contiguous() &&
                    dres->numel() == x.numel() && reinterpret_cast<uintptr_t>(dres->data_ptr()) % 16 == 0,
                "rms_norm backward: dres must be fp32 contiguous, aligned, x's size (fp32 x)");
    dresp = dres->data_ptr<float>();
  }
  if (dx16.has_value()) {
    TORCH_CHECK(x.scalar_type() == at::kFloat, "rms_norm backward: dx16 needs fp32 x");
    ln_check(*dx16, D, 4096);
    TORCH_CHECK(dx16->numel() == x.numel(), "rms_norm backward: dx16 size");
    dx16p = (uint16_t*)dx16->data_ptr();
  }
  if (R == 0) {
    dw.zero_();
    return;
  }
  // 4..16 rows per workgroup: >= 2 workgroups per CU at 2048 rows (Llama-3-8B, D 4096), where
  // 16-row blocks left 128 workgroups for 256 CUs (144 us per call, < 1 TB/s)
  const int rpb = (int)std::min<int64_t>(16, std::max<int64_t>(4, R / 1024));
  const int64_t P = (R + rpb - 1) / rpb;
  at::Tensor part = at::empty({P, D}, dw.options());
  auto st = c10::hip::getCurrentHIPStream();
  const size_t lds = (size_t)kLnWaves * D * sizeof(float);
  const int nc = (int)((D / 8 + 63) / 64);
  const bool f32 = x.scalar_type() == at::kFloat;
#define HIPPS_RMSB(NCc)                                                                                               \
  do {                                                                                                                \
    if (f32)                                                                                                          \
      hipLaunchKernelGGL((k_rms_bwd<NCc, float>), (int)P, 64 * kLnWaves, lds, st, (const uint16_t*)dy.data_ptr(),     \
                         x.data_ptr<float>(), rstd.data_ptr<float>(), w.data_ptr<float>(), dx.data_ptr<float>(),      \
                         part.data_ptr<float>(), R, (int)D, rpb, dresp, dx16p);                                       \
    else                                                                                                              \
      hipLaunchKernelGGL((k_rms_bwd<NCc, uint16_t>), (int)P, 64 * kLnWaves, lds, st, (const uint16_t*)dy.data_ptr(),  \
                         (const uint16_t*)x.data_ptr(), rstd.data_ptr<float>(), w.data_ptr<float>(),                  \
                         (uint16_t*)dx.data_ptr(), part.data_ptr<float>(), R, (int)D, rpb, nullptr, nullptr);          \
  } while (0)
  if (nc <= 1) HIPPS_RMSB(1);
  else if (nc <= 2) HIPPS_RMSB(2);
  else if (nc <= 4) HIPPS_RMSB(4);
  else HIPPS_RMSB(8);
#undef HIPPS_RMSB
  hipLaunchKernelGGL(k_ln_fold, (int)((D + 63) / 64), 64 * kFoldWaves, 0, st, part.data_ptr<float>(), (int)P, (int)D, 1,
                     dw.data_ptr<float>(), dw.data_ptr<float>(), nullptr);
}

}  // namespace hipps
