// hipps — fused training BatchNorm (+ residual add) (+ ReLU) for channels-last bf16 activations.
//
// Why: on MI355X the ResNet-50 worker step (ps_async, bs256) spends 14.9 ms in MIOpen BatchNorm
// and 8.5 ms in eager ReLU / add / relu-backward kernels out of 40.7 ms (profiles/
// bench_n1_steady_kernels.txt): ~20 HBM passes over 5.7 GB of activations.  Fusing the
// activation into the normalisation and recomputing the ReLU mask in the backward cuts that to
// ~9 passes.
//
// Layout: x is [M, C] with M = N*H*W rows and C contiguous (channels_last), C % 8 == 0,
// C <= 2048.  Each lane moves 8 channels (16 bytes) per access; a 256-thread workgroup is
// G = C/8 channel groups x R = 256/G row lanes, so a lane's channel group never changes and its
// per-channel constants live in registers for the whole grid-stride loop.
//
// Forward:  reduce (sum, sumsq per channel; fp32 lanes -> per-WG partials)   1 read
//           finalize (fp64 combine; mean, invstd, running stats, scale/shift)
//           apply  y = act(x*scale + shift [+ res])                         1 read (+res) 1 write
// Backward: reduce (sum dz, sum dz*xhat; dz = dy * relu'(.), mask recomputed from x, or read
//           from y when a residual was fused)                               2-3 reads
//           finalize (dgamma, dbeta, dx = a*dz + k1*x + k0 coefficients)
//           apply  dx (+ dres = dz)                                          2-3 reads 1-2 writes
// Partials are combined in a fixed order, so results are deterministic run to run.
#include "common.h"

#include <cstdlib>

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {

constexpr int kMaxC = 2048;

__device__ __forceinline__ void load8(const uint16_t* p, float v[8]) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ void store8(uint16_t* p, const float v[8]) {
  *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                            pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
}
__device__ __forceinline__ void load8f(const float* p, float v[8]) {
  float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

enum MaskMode { MASK_NONE = 0, MASK_X = 1, MASK_Y = 2, MASK_BITS = 3 };
// MASK_BITS: the forward wrote one byte per 8 channels (bit j = output channel c0+j > 0); the
// backward reads 1/16 of the bytes that re-reading the bf16 output (MASK_Y) would cost.

// ---- per-channel reductions -> partial[c][rb] (channel-major, two arrays) ------------------
// FWD: a += x, b += x*x.   BWD: dz = dy*mask; a += dz, b += dz*(x-mean)*invstd.
// Each lane keeps UNR rows (up to 3*UNR x 16 B) in flight before consuming them: one load per
// iteration left these passes at 3.2-3.9 TB/s (profiles/bench_n1_steady_fusedbn.txt).  The mask
// mode is a template parameter so each variant only holds the registers it needs (the runtime
// switch cost 186 VGPRs in the backward = 2 waves/SIMD; profiles/bn_regs.txt).
template <bool BWD, int MODE>
__device__ __forceinline__ void reduce_row(const float xv[8], const float* d, const float* yv, uint32_t mb,
                                           const float mu[8], const float is[8], const float sc[8],
                                           const float sh[8], float sa[8], float sb[8]) {
  if (!BWD) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sa[j] += xv[j]; sb[j] = fmaf(xv[j], xv[j], sb[j]); }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dz = d[j];
      if (MODE == MASK_BITS) dz = ((mb >> j) & 1u) ? dz : 0.f;
      else if (MODE == MASK_Y) dz = yv[j] > 0.f ? dz : 0.f;
      else if (MODE == MASK_X) dz = fmaf(xv[j], sc[j], sh[j]) > 0.f ? dz : 0.f;
      sa[j] += dz;
      sb[j] = fmaf(dz, (xv[j] - mu[j]) * is[j], sb[j]);
    }
  }
}

template <bool BWD, int MODE, int UNR>
__global__ __launch_bounds__(kBlock) void k_bn_reduce(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                                      const uint16_t* __restrict__ y,
                                                      const uint8_t* __restrict__ mbits,
                                                      const float* __restrict__ mean, const float* __restrict__ invstd,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      int64_t M, int C, int64_t rows_per_wg, int nrb,
                                                      float* __restrict__ pa, float* __restrict__ pb) {
  __shared__ float la[kBlock * 8], lb[kBlock * 8];
  constexpr bool need_y = BWD && MODE == MASK_Y;
  constexpr bool need_b = BWD && MODE == MASK_BITS;
  constexpr bool need_ss = BWD && MODE == MASK_X;
  const int G = C >> 3, R = kBlock / G;
  const int g = threadIdx.x % G, r = threadIdx.x / G;
  const int c0 = g * 8;
  float sa[8], sb[8], mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j] = 0.f; sb[j] = 0.f; mu[j] = 0.f; is[j] = 0.f; sc[j] = 0.f; sh[j] = 0.f; }
  if (BWD) {
    load8f(mean + c0, mu);
    load8f(invstd + c0, is);
    if (need_ss) { load8f(scale + c0, sc); load8f(shift + c0, sh); }
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r1 = min(M, r0 + rows_per_wg);
  int64_t row = r0 + r;
  for (; row + (UNR - 1) * (int64_t)R < r1; row += UNR * (int64_t)R) {
    float xv[UNR][8], d[BWD ? UNR : 1][8], yv[need_y ? UNR : 1][8];
    uint32_t mb[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t rr = row + u * (int64_t)R;
      const int64_t off = rr * C + c0;
      load8(x + off, xv[u]);
      if (BWD) load8(dy + off, d[BWD ? u : 0]);
      if (need_y) load8(y + off, yv[need_y ? u : 0]);
      mb[u] = need_b ? (uint32_t)mbits[rr * G + g] : 0u;
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      reduce_row<BWD, MODE>(xv[u], d[BWD ? u : 0], yv[need_y ? u : 0], mb[u], mu, is, sc, sh, sa, sb);
  }
  for (; row < r1; row += R) {
    const int64_t off = row * C + c0;
    float xv[8], d[8], yv[8];
    load8(x + off, xv);
    if (BWD) load8(dy + off, d);
    if (need_y) load8(y + off, yv);
    const uint32_t mb = need_b ? (uint32_t)mbits[row * G + g] : 0u;
    reduce_row<BWD, MODE>(xv, d, yv, mb, mu, is, sc, sh, sa, sb);
  }
  // combine the R row lanes of each channel group through LDS
#pragma unroll
  for (int j = 0; j < 8; ++j) { la[r * C + c0 + j] = sa[j]; lb[r * C + c0 + j] = sb[j]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBlock) {
    float a = 0.f, b = 0.f;
    for (int q = 0; q < R; ++q) { a += la[q * C + c]; b += lb[q * C + c]; }
    pa[(int64_t)c * nrb + blockIdx.x] = a;
    pb[(int64_t)c * nrb + blockIdx.x] = b;
  }
}

// Combine partial[c][rb] over rb: one workgroup per channel, the 256 lanes read consecutive
// partials (coalesced), fp64 sums, shuffle tree per wave + fixed-order combine of the 4 waves.
// (v1 looped serially per channel: 180-270 us per call, profiles/bn_micro_r1.txt; v2 used one
// wave per channel: 12 us per call on the 1x1-GEMM partials, nrb = M/128 = 6272 on layer1,
// profiles/bench_n1_steady_r1c.txt.)
constexpr int kFinCh = 1;
// WPC (nrb <= 512, the deep layers' partials): one wave per channel, 4 channels per block -- the
// block-per-channel form spent most of its ~5 us on 2048 mostly idle workgroups there
template <bool WPC, int U>
__device__ __forceinline__ bool combine_partials(const float* __restrict__ pa, const float* __restrict__ pb, int nrb,
                                                 int C, double& s, double& q, int& c) {
  __shared__ double red[2][kBlock / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  c = WPC ? blockIdx.x * (kBlock / 64) + wv : blockIdx.x;
  double a = 0.0, b = 0.0;
  if (c < C) {
    const float* ra = pa + (int64_t)c * nrb;
    const float* rb = pb + (int64_t)c * nrb;
    // 2*U independent loads in flight per lane: the partials were just written by the producer
    // and mostly sit in MALL / HBM (a layer-1 GEMM's are 12.8 MB), so the kernel's time is the
    // number of dependent round trips (nrb / (U*256)); out-of-range lanes load a clamped index and
    // add zero (a branch around each load would wait per element).  Each lane's sum keeps its
    // fixed order.
    constexpr int L = WPC ? 64 : kBlock;
    for (int i0 = WPC ? lane : (int)threadIdx.x; i0 < nrb; i0 += U * L) {
      float va[U], vb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u * L, nrb - 1);
        va[u] = ra[i];
        vb[u] = rb[i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool in = i0 + u * L < nrb;
        a += in ? (double)va[u] : 0.0;
        b += in ? (double)vb[u] : 0.0;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if constexpr (WPC) {
    s = a;
    q = b;
    return lane == 0 && c < C;
  } else {
    if (lane == 0) { red[0][wv] = a; red[1][wv] = b; }
    __syncthreads();
    s = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    q = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    return threadIdx.x == 0 && c < C;
  }
}

// forward finalize: stats + running stats + per-channel scale/shift
template <bool WPC, int U = 12>
__global__ __launch_bounds__(kBlock) void k_bn_finalize_fwd(const float* __restrict__ pa, const float* __restrict__ pb,
                                                            int nrb, int C, int64_t M, const float* __restrict__ w,
                                                            const float* __restrict__ bias, float eps, float momentum,
                                                            float* __restrict__ running_mean,
                                                            float* __restrict__ running_var, float* __restrict__ mean,
                                                            float* __restrict__ invstd, float* __restrict__ scale,
                                                            float* __restrict__ shift) {
  double s, q;
  int c;
  if (!combine_partials<WPC, U>(pa, pb, nrb, C, s, q, c)) return;
  const double m = s / (double)M;
  double var = q / (double)M - m * m;
  if (var < 0.0) var = 0.0;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = (float)m;
  invstd[c] = is;
  const float wc = w ? w[c] : 1.f, bc = bias ? bias[c] : 0.f;
  scale[c] = wc * is;
  shift[c] = bc - (float)m * wc * is;
  if (running_mean) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)m;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
  }
}

// backward finalize: dgamma, dbeta and dx = a*dz + k1*x + k0 coefficients
template <bool WPC, int U = 12>
__global__ __launch_bounds__(kBlock) void k_bn_finalize_bwd(const float* __restrict__ pa, const float* __restrict__ pb,
                                                            int nrb, int C, int64_t M, const float* __restrict__ w,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, float* __restrict__ dw,
                                                            float* __restrict__ db, float* __restrict__ ca,
                                                            float* __restrict__ ck1, float* __restrict__ ck0) {
  double s, q;
  int c;
  if (!combine_partials<WPC, U>(pa, pb, nrb, C, s, q, c)) return;
  if (dw) dw[c] = (float)q;
  if (db) db[c] = (float)s;
  const double is = invstd[c];
  const double a = (w ? (double)w[c] : 1.0) * is;
  const double k1 = -a * is * q / (double)M;
  const double k0 = -a * s / (double)M - k1 * (double)mean[c];
  ca[c] = (float)a;
  ck1[c] = (float)k1;
  ck0[c] = (float)k0;
}

// wave-per-channel finalize: measured no faster in the step (the ~5 us per call is launch
// latency, not the combine), so it is off (kWpcMax = 0); kept for the micro-benchmarks
constexpr int kWpcMax = 0;
// loads in flight per lane in the combine: 2*12 (HIPPS_BN_FIN_U=4: the round-3 depth, for A/B)
static bool fin_shallow() {
  static const bool v = [] { const char* e = std::getenv("HIPPS_BN_FIN_U"); return e && std::atoi(e) == 4; }();
  return v;
}
static void fin_fwd(hipStream_t st, const float* pa, const float* pb, int nrb, int C, int64_t M, const float* w,
                    const float* bias, float eps, float mom, float* rm, float* rv, float* mean, float* invstd,
                    float* scale, float* shift) {
  if (nrb <= kWpcMax)
    hipLaunchKernelGGL(k_bn_finalize_fwd<true>, (C + kBlock / 64 - 1) / (kBlock / 64), kBlock, 0, st, pa, pb, nrb, C, M,
                       w, bias, eps, mom, rm, rv, mean, invstd, scale, shift);
  else if (fin_shallow())
    hipLaunchKernelGGL((k_bn_finalize_fwd<false, 4>), C, kBlock, 0, st, pa, pb, nrb, C, M, w, bias, eps, mom, rm, rv,
                       mean, invstd, scale, shift);
  else
    hipLaunchKernelGGL(k_bn_finalize_fwd<false>, C, kBlock, 0, st, pa, pb, nrb, C, M, w, bias, eps, mom, rm, rv, mean,
                       invstd, scale, shift);
}
static void fin_bwd(hipStream_t st, const float* pa, const float* pb, int nrb, int C, int64_t M, const float* w,
                    const float* mean, const float* invstd, float* dw, float* db, float* ca, float* ck1, float* ck0) {
  if (nrb <= kWpcMax)
    hipLaunchKernelGGL(k_bn_finalize_bwd<true>, (C + kBlock / 64 - 1) / (kBlock / 64), kBlock, 0, st, pa, pb, nrb, C, M,
                       w, mean, invstd, dw, db, ca, ck1, ck0);
  else if (fin_shallow())
    hipLaunchKernelGGL((k_bn_finalize_bwd<false, 4>), C, kBlock, 0, st, pa, pb, nrb, C, M, w, mean, invstd, dw, db, ca,
                       ck1, ck0);
  else
    hipLaunchKernelGGL(k_bn_finalize_bwd<false>, C, kBlock, 0, st, pa, pb, nrb, C, M, w, mean, invstd, dw, db, ca, ck1,
                       ck0);
}

// y = act(x*scale + shift [+ res]); with rsc/rsh the residual is itself a pre-BN tensor whose
// BN is applied in the same pass: res*rsc + rsh (a ResNet downsample branch, never materialised).
// UNR vectors in flight per lane (UNR = 4 on the small layer-3/4 tensors measured no faster in the
// step, so every call site uses 1).
template <int UNR = 1>
__global__ __launch_bounds__(kBlock) void k_bn_apply_fwd(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                         uint16_t* __restrict__ y, uint8_t* __restrict__ mbits,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int64_t M, int C, int relu,
                                                         const float* __restrict__ rsc = nullptr,
                                                         const float* __restrict__ rsh = nullptr, int pack_bits = 1) {
  const int G = C >> 3;
  const int64_t V = M * (int64_t)G, stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(v0 % G) * 8;  // fixed per lane: stride is a multiple of G
  float sc[8], sh[8], rs[8], rh[8];
  load8f(scale + c0, sc);
  load8f(shift + c0, sh);
  if (rsc) {
    load8f(rsc + c0, rs);
    load8f(rsh + c0, rh);
  }
  auto body = [&](float* xv, float* rv, int64_t v) {
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = fmaf(xv[j], sc[j], sh[j]);
    if (res) {
      if (rsc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) rv[j] = fmaf(rv[j], rs[j], rh[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] += rv[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[j] = fmaxf(xv[j], 0.f);
    }
    store8(y + v * 8, xv);
    if (mbits) {
      uint32_t b = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) b |= (xv[j] > 0.f ? 1u : 0u) << j;
      // a full wave's 64 bytes as 16 dword stores (4 lanes' bytes gathered by DPP-free shuffles)
      // instead of 64 byte stores; the last, partial wave of the tensor stores bytes
      const int lane = threadIdx.x & 63;
      // (UNR == 2 splits a wave between its paired and remainder loops: bytes only)
      if (pack_bits && UNR != 2 && v - lane + 63 < V) {
        const uint32_t b1 = __shfl_down(b, 1, 64), b2 = __shfl_down(b, 2, 64), b3 = __shfl_down(b, 3, 64);
        if ((lane & 3) == 0) *reinterpret_cast<uint32_t*>(mbits + v) = b | (b1 << 8) | (b2 << 16) | (b3 << 24);
      } else {
        mbits[v] = (uint8_t)b;
      }
    }
  };
  int64_t v = v0;
  if constexpr (UNR == 3) {
    // software pipeline: the next vector's loads are issued before this one's stores, so the
    // wait for them (vmcnt counts stores too, in issue order) never waits for a store to land
    float xa[8], ra[8];
    if (v < V) {
      load8(x + v * 8, xa);
      if (res) load8(res + v * 8, ra);
    }
    for (; v < V; v += stride) {
      const int64_t vn = v + stride;
      float xb[8], rb[8];
      if (vn < V) {
        load8(x + vn * 8, xb);
        if (res) load8(res + vn * 8, rb);
      }
      body(xa, ra, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xa[j] = xb[j];
        ra[j] = rb[j];
      }
    }
    return;
  }
  if constexpr (UNR == 2) {
    for (; v + (UNR - 1) * stride < V; v += UNR * stride) {
      float xv[UNR][8], rv[UNR][8];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        load8(x + (v + u * stride) * 8, xv[u]);
        if (res) load8(res + (v + u * stride) * 8, rv[u]);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) body(xv[u], rv[u], v + u * stride);
    }
  }
  for (; v < V; v += stride) {
    float xv[8], rv[8];
    load8(x + v * 8, xv);
    if (res) load8(res + v * 8, rv);
    body(xv, rv, v);
  }
}

// dx = a*dz + k1*x + k0, dz = dy * mask;  dres = dz (when a residual was fused).  UNR vectors
// in flight per lane.
template <int MODE, int UNR = 2>
__global__ __launch_bounds__(kBlock) void k_bn_apply_bwd(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ y,
                                                         const uint8_t* __restrict__ mbits,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, const float* __restrict__ ca,
                                                         const float* __restrict__ ck1, const float* __restrict__ ck0,
                                                         uint16_t* __restrict__ dx, uint16_t* __restrict__ dres,
                                                         int64_t M, int C) {
  constexpr int mask_mode = MODE;
  const int G = C >> 3;
  const int64_t V = M * (int64_t)G, stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(v0 % G) * 8;
  float a[8], k1[8], k0[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = 0.f; sh[j] = 0.f; }
  load8f(ca + c0, a);
  load8f(ck1 + c0, k1);
  load8f(ck0 + c0, k0);
  if (mask_mode == MASK_X) { load8f(scale + c0, sc); load8f(shift + c0, sh); }
  auto body = [&](const float* d_in, const float* xv, const float* yv, uint32_t mb, int64_t off) {
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dz = d_in[j];
      if (mask_mode == MASK_BITS) dz = ((mb >> j) & 1u) ? dz : 0.f;
      else if (mask_mode == MASK_Y) dz = yv[j] > 0.f ? dz : 0.f;
      else if (mask_mode == MASK_X) dz = fmaf(xv[j], sc[j], sh[j]) > 0.f ? dz : 0.f;
      d[j] = dz;
    }
    if (dres) store8(dres + off, d);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(a[j], d[j], fmaf(k1[j], xv[j], k0[j]));
    store8(dx + off, o);
  };
  constexpr bool need_y = mask_mode == MASK_Y, need_b = mask_mode == MASK_BITS;
  int64_t v = v0;
  if constexpr (UNR == 0) {
    // software pipeline (HIPPS_BN_PIPE=1): the next vector's loads go out before this vector's
    // stores, so waiting for them never waits on a store (vmcnt counts both, in issue order)
    float d0[8], x0[8], y0[8];
    uint32_t m0 = 0;
    if (v < V) {
      load8(dy + v * 8, d0);
      load8(x + v * 8, x0);
      if (need_y) load8(y + v * 8, y0);
      m0 = need_b ? (uint32_t)mbits[v] : 0u;
    }
    for (; v < V; v += stride) {
      const int64_t vn = v + stride;
      float d1[8], x1[8], y1[8];
      uint32_t m1 = 0;
      if (vn < V) {
        load8(dy + vn * 8, d1);
        load8(x + vn * 8, x1);
        if (need_y) load8(y + vn * 8, y1);
        m1 = need_b ? (uint32_t)mbits[vn] : 0u;
      }
      body(d0, x0, y0, m0, v * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        d0[j] = d1[j];
        x0[j] = x1[j];
        y0[j] = y1[j];
      }
      m0 = m1;
    }
    return;
  }
  constexpr int UN = UNR > 0 ? UNR : 1;  // (UNR == 0 returned above)
  for (; v + (UN - 1) * stride < V; v += UN * stride) {  // UNR vectors in flight per lane
    float d[UN][8], xv[UN][8], yv[need_y ? UN : 1][8];
    uint32_t mb[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int64_t o = (v + u * stride) * 8;
      load8(dy + o, d[u]);
      load8(x + o, xv[u]);
      if (need_y) load8(y + o, yv[need_y ? u : 0]);
      mb[u] = need_b ? (uint32_t)mbits[v + u * stride] : 0u;
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) body(d[u], xv[u], yv[need_y ? u : 0], mb[u], (v + u * stride) * 8);
  }
  for (; v < V; v += stride) {
    float d0[8], x0[8], y0[8];
    const int64_t o0 = v * 8;
    load8(dy + o0, d0);
    load8(x + o0, x0);
    if (need_y) load8(y + o0, y0);
    const uint32_t m0 = need_b ? (uint32_t)mbits[v] : 0u;
    body(d0, x0, y0, m0, o0);
  }
}

// Backward of z = relu(bn3(x3) + bnd(xd)) (ResNet downsample block), pass 1: with dz' = dz * bits,
// dx3 = a3*dz' + k1*x3 + k0 (bn3's apply) and, in the same pass, the downsample BN's reduction
// (sum dz', sum dz' * (xd - mean_d) * invstd_d) into per-WG partials -- the residual gradient dz'
// is never written (pass 2 recomputes it from dz and the bits).
template <int UNR>
__global__ __launch_bounds__(kBlock) void k_bn_bwd_dual(const uint16_t* __restrict__ dz, const uint16_t* __restrict__ x3,
                                                        const uint16_t* __restrict__ xd,
                                                        const uint8_t* __restrict__ mbits,
                                                        const float* __restrict__ ca, const float* __restrict__ ck1,
                                                        const float* __restrict__ ck0, const float* __restrict__ meand,
                                                        const float* __restrict__ invstdd, uint16_t* __restrict__ dx3,
                                                        int64_t M, int C, int64_t rows_per_wg, int nrb,
                                                        float* __restrict__ pa, float* __restrict__ pb) {
  __shared__ float la[kBlock * 8], lb[kBlock * 8];
  const int G = C >> 3, R = kBlock / G;
  const int g = threadIdx.x % G, r = threadIdx.x / G;
  const int c0 = g * 8;
  float sa[8], sb[8], a[8], k1[8], k0[8], mu[8], is[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sa[j] = 0.f; sb[j] = 0.f; }
  load8f(ca + c0, a);
  load8f(ck1 + c0, k1);
  load8f(ck0 + c0, k0);
  load8f(meand + c0, mu);
  load8f(invstdd + c0, is);
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t r1 = min(M, r0 + rows_per_wg);
  auto body = [&](const float* d, const float* xv, const float* xr, uint32_t mb, int64_t off) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dzm = ((mb >> j) & 1u) ? d[j] : 0.f;
      o[j] = fmaf(a[j], dzm, fmaf(k1[j], xv[j], k0[j]));
      sa[j] += dzm;
      sb[j] = fmaf(dzm, (xr[j] - mu[j]) * is[j], sb[j]);
    }
    store8(dx3 + off, o);
  };
  int64_t row = r0 + r;
  for (; row + (UNR - 1) * (int64_t)R < r1; row += UNR * (int64_t)R) {
    float d[UNR][8], xv[UNR][8], xr[UNR][8];
    uint32_t mb[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int64_t rr = row + u * (int64_t)R;
      const int64_t off = rr * C + c0;
      load8(dz + off, d[u]);
      load8(x3 + off, xv[u]);
      load8(xd + off, xr[u]);
      mb[u] = (uint32_t)mbits[rr * G + g];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) body(d[u], xv[u], xr[u], mb[u], (row + u * (int64_t)R) * C + c0);
  }
  for (; row < r1; row += R) {
    const int64_t off = row * C + c0;
    float d[8], xv[8], xr[8];
    load8(dz + off, d);
    load8(x3 + off, xv);
    load8(xd + off, xr);
    body(d, xv, xr, (uint32_t)mbits[row * G + g], off);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { la[r * C + c0 + j] = sa[j]; lb[r * C + c0 + j] = sb[j]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBlock) {
    float s0 = 0.f, s1 = 0.f;
    for (int q = 0; q < R; ++q) { s0 += la[q * C + c]; s1 += lb[q * C + c]; }
    pa[(int64_t)c * nrb + blockIdx.x] = s0;
    pb[(int64_t)c * nrb + blockIdx.x] = s1;
  }
}

// ==========================================================================================
namespace {
void check_act(const at::Tensor& t, const char* n, int64_t numel) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, n, " must be a bf16 device tensor");
  TORCH_CHECK(t.numel() == numel, n, " size mismatch");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, n, " must be 16-byte aligned");
}
void check_vec(const at::Tensor& t, const char* n, int C) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == C, n,
              " must be a contiguous f32 device vector of length C");
}
int64_t pick_rows(int64_t M, int C, int& nrb) {
  const int G = C / 8, R = kBlock / G;
  const int64_t vec = M * G;
  int64_t want = vec / (kBlock * 16);  // >= 16 vectors per lane
  want = std::max<int64_t>(1, std::min<int64_t>(want, 1024));
  int64_t rows = (M + want - 1) / want;
  rows = (rows + R - 1) / R * R;
  nrb = (int)((M + rows - 1) / rows);
  return rows;
}
int apply_grid(int64_t M, int C) {
  const int64_t V = M * (C / 8);
  return grid_for(V);
}
// forward apply: UNR vectors in flight per lane on the large (>= 4 M-vector, layer-1/2) tensors
// when HIPPS_BN_APPLY_UNR=2 (A/B; 1 measured no slower on the layer-3/4 sizes)
typedef void (*ApplyFwdFn)(const uint16_t*, const uint16_t*, uint16_t*, uint8_t*, const float*, const float*, int64_t,
                           int, int, const float*, const float*, int);
// the ReLU mask bytes of a full wave as 16 dword stores (HIPPS_BN_BITS_PACK=0: 64 byte stores, A/B)
int bits_pack() {
  static const int on = [] {
    const char* e = std::getenv("HIPPS_BN_BITS_PACK");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on;
}
ApplyFwdFn apply_fwd_kernel(int64_t M, int C) {
  static const int unr = [] {
    const char* e = std::getenv("HIPPS_BN_APPLY_UNR");
    return e ? std::atoi(e) : 1;
  }();
  if (unr == 2 && M * (C / 8) >= (int64_t(4) << 20)) return k_bn_apply_fwd<2>;
  if (unr == 3) return k_bn_apply_fwd<3>;  // software-pipelined (A/B)
  return k_bn_apply_fwd<1>;
}
// HIPPS_BN_PIPE=1: the software-pipelined backward apply (k_bn_apply_bwd<MODE, 0>) -- A/B
bool bn_pipe() {
  static const bool on = [] {
    const char* e = std::getenv("HIPPS_BN_PIPE");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return on;
}
}  // namespace

namespace {
// forward finalize (stats -> running stats, scale/shift) + apply, from channel-major partials
void finalize_apply_fwd(const at::Tensor& part, int nrb, const at::Tensor& x, const uint16_t* rp, at::Tensor& y,
                        uint8_t* mo, at::Tensor& weight, at::Tensor& bias, float* rm, float* rv, at::Tensor& mean,
                        at::Tensor& invstd, at::Tensor& scale, at::Tensor& shift, int64_t M, int64_t C, double eps,
                        double momentum, bool relu, hipStream_t stream) {
  const float* pa = part.data_ptr<float>();
  const float* pb = pa + C * (int64_t)nrb;
  fin_fwd( stream, pa, pb, nrb, (int)C, M,
                     weight.data_ptr<float>(), bias.data_ptr<float>(), (float)eps, (float)momentum, rm, rv,
                     mean.data_ptr<float>(), invstd.data_ptr<float>(), scale.data_ptr<float>(),
                     shift.data_ptr<float>());
  hipLaunchKernelGGL(apply_fwd_kernel(M, (int)C), apply_grid(M, (int)C), kBlock, 0, stream, (const uint16_t*)x.data_ptr(), rp,
                     (uint16_t*)y.data_ptr(), mo, scale.data_ptr<float>(), shift.data_ptr<float>(), M, (int)C,
                     (int)relu, nullptr, nullptr, bits_pack());
}
}  // namespace

// x: [M, C] bf16 view (channels-last storage).  Returns nothing; fills y, mean, invstd,
// scale, shift and updates running stats in place.
void bn_forward_train(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y, at::Tensor weight, at::Tensor bias,
                      c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var, at::Tensor mean,
                      at::Tensor invstd, at::Tensor scale, at::Tensor shift, int64_t C, double eps, double momentum,
                      bool relu, c10::optional<at::Tensor> mask_out) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC && C >= 8, "fused BN needs C % 8 == 0 and 8 <= C <= 2048");
  const int64_t M = x.numel() / C;
  check_act(x, "x", M * C);
  check_act(y, "y", M * C);
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_act(*res, "residual", M * C);
    rp = (const uint16_t*)res->data_ptr();
  }
  for (auto* t : {&weight, &bias, &mean, &invstd, &scale, &shift}) check_vec(*t, "per-channel vector", (int)C);
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    check_vec(*running_mean, "running_mean", (int)C);
    check_vec(*running_var, "running_var", (int)C);
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  int nrb;
  const int64_t rows = pick_rows(M, (int)C, nrb);
  auto part = at::empty({2, C, (int64_t)nrb}, weight.options());
  auto stream = c10::hip::getCurrentHIPStream();
  uint8_t* mo = nullptr;
  if (mask_out.has_value() && mask_out->defined()) {
    TORCH_CHECK(mask_out->is_cuda() && mask_out->scalar_type() == at::kByte && mask_out->numel() == M * C / 8,
                "mask_out must be uint8[M*C/8]");
    mo = (uint8_t*)mask_out->data_ptr();
  }
  hipLaunchKernelGGL((k_bn_reduce<false, MASK_NONE, 8>), nrb, kBlock, 0, stream, (const uint16_t*)x.data_ptr(),
                     nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, M, (int)C, rows, nrb,
                     part[0].data_ptr<float>(), part[1].data_ptr<float>());
  finalize_apply_fwd(part, nrb, x, rp, y, mo, weight, bias, rm, rv, mean, invstd, scale, shift, M, C, eps, momentum,
                     relu, stream);
}

// Finalize only, from a producer's partial sums part [2, C, nrb] over M rows: mean, invstd, scale,
// shift and the running stats; no pass over the activations (the stem's max pool applies them).
void bn_finalize_partials(at::Tensor part, int64_t nrb, int64_t M, at::Tensor weight, at::Tensor bias,
                          c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
                          at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift, int64_t C, double eps,
                          double momentum) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC && C >= 8, "fused BN needs C % 8 == 0 and 8 <= C <= 2048");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.numel() == 2 * C * nrb,
              "bn_finalize_partials: part must be f32 [2, C, nrb]");
  TORCH_CHECK(M > 0 && nrb > 0 && nrb < (int64_t(1) << 31), "bn_finalize_partials: sizes");
  for (auto* t : {&weight, &bias, &mean, &invstd, &scale, &shift}) check_vec(*t, "per-channel vector", (int)C);
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    check_vec(*running_mean, "running_mean", (int)C);
    check_vec(*running_var, "running_var", (int)C);
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  fin_fwd( c10::hip::getCurrentHIPStream(),
                     part[0].data_ptr<float>(), part[1].data_ptr<float>(), (int)nrb, (int)C, M,
                     weight.data_ptr<float>(), bias.data_ptr<float>(), (float)eps, (float)momentum, rm, rv,
                     mean.data_ptr<float>(), invstd.data_ptr<float>(), scale.data_ptr<float>(),
                     shift.data_ptr<float>());
}

// Backward finalize only, from a producer's partials part [2, C, nrb] (a = sum dz', b = sum dz' x-hat
// over M rows): dweight, dbias and coef [3, C] = (a, k1, k0) of dx = a*dz' + k1*x + k0.  The stem's
// fused pool backward (stem.hip) reduces and applies on its own.
void bn_finalize_bwd_partials(at::Tensor part, int64_t nrb, int64_t M, at::Tensor weight, at::Tensor mean,
                              at::Tensor invstd, at::Tensor dweight, at::Tensor dbias, at::Tensor coef) {
  const int64_t C = weight.numel();
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC && C >= 8, "fused BN needs C % 8 == 0 and 8 <= C <= 2048");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.numel() == 2 * C * nrb,
              "bn_finalize_bwd_partials: part must be f32 [2, C, nrb]");
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 3 * C,
              "bn_finalize_bwd_partials: coef must be f32 [3, C]");
  for (auto* t : {&weight, &mean, &invstd, &dweight, &dbias}) check_vec(*t, "per-channel vector", (int)C);
  fin_bwd( c10::hip::getCurrentHIPStream(),
                     part[0].data_ptr<float>(), part[1].data_ptr<float>(), (int)nrb, (int)C, M,
                     weight.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                     dweight.data_ptr<float>(), dbias.data_ptr<float>(), coef[0].data_ptr<float>(),
                     coef[1].data_ptr<float>(), coef[2].data_ptr<float>());
}

// Statistics only (reduce + finalize): mean, invstd, scale, shift and the running stats, no apply
// pass -- the consuming 1x1 conv applies scale/shift + ReLU in its operand prologue (gemm.hip).
void bn_forward_stats(at::Tensor x, at::Tensor weight, at::Tensor bias, c10::optional<at::Tensor> running_mean,
                      c10::optional<at::Tensor> running_var, at::Tensor mean, at::Tensor invstd, at::Tensor scale,
                      at::Tensor shift, int64_t C, double eps, double momentum) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC && C >= 8, "fused BN needs C % 8 == 0 and 8 <= C <= 2048");
  const int64_t M = x.numel() / C;
  check_act(x, "x", M * C);
  for (auto* t : {&weight, &bias, &mean, &invstd, &scale, &shift}) check_vec(*t, "per-channel vector", (int)C);
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    check_vec(*running_mean, "running_mean", (int)C);
    check_vec(*running_var, "running_var", (int)C);
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  int nrb;
  const int64_t rows = pick_rows(M, (int)C, nrb);
  auto part = at::empty({2, C, (int64_t)nrb}, weight.options());
  auto stream = c10::hip::getCurrentHIPStream();
  hipLaunchKernelGGL((k_bn_reduce<false, MASK_NONE, 8>), nrb, kBlock, 0, stream, (const uint16_t*)x.data_ptr(),
                     nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, M, (int)C, rows, nrb,
                     part[0].data_ptr<float>(), part[1].data_ptr<float>());
  fin_fwd( stream, part[0].data_ptr<float>(),
                     part[1].data_ptr<float>(), nrb, (int)C, M, weight.data_ptr<float>(), bias.data_ptr<float>(),
                     (float)eps, (float)momentum, rm, rv, mean.data_ptr<float>(), invstd.data_ptr<float>(),
                     scale.data_ptr<float>(), shift.data_ptr<float>());
}

// eval / affine-only apply with given scale/shift
void bn_apply(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y, at::Tensor scale, at::Tensor shift, int64_t C,
              bool relu) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC, "fused BN needs C % 8 == 0 and C <= 2048");
  const int64_t M = x.numel() / C;
  check_act(x, "x", M * C);
  check_act(y, "y", M * C);
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_act(*res, "residual", M * C);
    rp = (const uint16_t*)res->data_ptr();
  }
  check_vec(scale, "scale", (int)C);
  check_vec(shift, "shift", (int)C);
  hipLaunchKernelGGL(apply_fwd_kernel(M, (int)C), apply_grid(M, (int)C), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)x.data_ptr(), rp, (uint16_t*)y.data_ptr(), nullptr, scale.data_ptr<float>(),
                     shift.data_ptr<float>(), M, (int)C, (int)relu, nullptr, nullptr, bits_pack());
}

// returns nothing; writes dx (and dres), dweight, dbias
void bn_backward(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> y, int64_t mask_mode, at::Tensor weight,
                 at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift, at::Tensor dx,
                 c10::optional<at::Tensor> dres, at::Tensor dweight, at::Tensor dbias, int64_t C,
                 c10::optional<at::Tensor> mask_in) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC, "fused BN needs C % 8 == 0 and C <= 2048");
  TORCH_CHECK(mask_mode >= MASK_NONE && mask_mode <= MASK_BITS, "bad mask mode");
  const int64_t M = x.numel() / C;
  check_act(dy, "dy", M * C);
  check_act(x, "x", M * C);
  check_act(dx, "dx", M * C);
  const uint16_t* yp = nullptr;
  if (mask_mode == MASK_Y) {
    TORCH_CHECK(y.has_value() && y->defined(), "mask from y needs y");
    check_act(*y, "y", M * C);
    yp = (const uint16_t*)y->data_ptr();
  }
  const uint8_t* mbp = nullptr;
  if (mask_mode == MASK_BITS) {
    TORCH_CHECK(mask_in.has_value() && mask_in->defined() && mask_in->scalar_type() == at::kByte &&
                    mask_in->numel() == M * C / 8, "MASK_BITS needs a uint8[M*C/8] mask");
    mbp = (const uint8_t*)mask_in->data_ptr();
  }
  uint16_t* drp = nullptr;
  if (dres.has_value() && dres->defined()) {
    check_act(*dres, "dres", M * C);
    drp = (uint16_t*)dres->data_ptr();
  }
  for (auto* t : {&weight, &mean, &invstd, &scale, &shift, &dweight, &dbias}) check_vec(*t, "per-channel vector", (int)C);
  int nrb;
  const int64_t rows = pick_rows(M, (int)C, nrb);
  auto part = at::empty({2, C, (int64_t)nrb}, weight.options());
  auto coef = at::empty({3, C}, weight.options());
  auto stream = c10::hip::getCurrentHIPStream();
  auto red = [&](auto kern) {
    hipLaunchKernelGGL(kern, nrb, kBlock, 0, stream, (const uint16_t*)x.data_ptr(), (const uint16_t*)dy.data_ptr(), yp,
                       mbp, mean.data_ptr<float>(), invstd.data_ptr<float>(), scale.data_ptr<float>(),
                       shift.data_ptr<float>(), M, (int)C, rows, nrb, part[0].data_ptr<float>(),
                       part[1].data_ptr<float>());
  };
  switch (mask_mode) {
    case MASK_NONE: red(k_bn_reduce<true, MASK_NONE, 4>); break;
    case MASK_X: red(k_bn_reduce<true, MASK_X, 4>); break;
    case MASK_Y: red(k_bn_reduce<true, MASK_Y, 4>); break;
    default: red(k_bn_reduce<true, MASK_BITS, 4>); break;
  }
  fin_bwd( stream, part[0].data_ptr<float>(),
                     part[1].data_ptr<float>(), nrb, (int)C, M, weight.data_ptr<float>(), mean.data_ptr<float>(),
                     invstd.data_ptr<float>(), dweight.data_ptr<float>(), dbias.data_ptr<float>(),
                     coef[0].data_ptr<float>(), coef[1].data_ptr<float>(), coef[2].data_ptr<float>());
  auto app = [&](auto kern) {
    hipLaunchKernelGGL(kern, apply_grid(M, (int)C), kBlock, 0, stream, (const uint16_t*)dy.data_ptr(),
                       (const uint16_t*)x.data_ptr(), yp, mbp, scale.data_ptr<float>(), shift.data_ptr<float>(),
                       coef[0].data_ptr<float>(), coef[1].data_ptr<float>(), coef[2].data_ptr<float>(),
                       (uint16_t*)dx.data_ptr(), drp, M, (int)C);
  };
  if (bn_pipe()) {
    switch (mask_mode) {
      case MASK_NONE: app(k_bn_apply_bwd<MASK_NONE, 0>); break;
      case MASK_X: app(k_bn_apply_bwd<MASK_X, 0>); break;
      case MASK_Y: app(k_bn_apply_bwd<MASK_Y, 0>); break;
      default: app(k_bn_apply_bwd<MASK_BITS, 0>); break;
    }
    return;
  }
  switch (mask_mode) {
    case MASK_NONE: app(k_bn_apply_bwd<MASK_NONE>); break;
    case MASK_X: app(k_bn_apply_bwd<MASK_X>); break;
    case MASK_Y: app(k_bn_apply_bwd<MASK_Y>); break;
    default: app(k_bn_apply_bwd<MASK_BITS>); break;
  }
}

}  // namespace hipps

namespace hipps {
// Forward BN whose batch statistics were already reduced by the producer (conv1x1 epilogue):
// part = f32 [2, C, nrb] channel-major partial sums / sums of squares.
void bn_forward_partials(at::Tensor part, int64_t nrb, at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y,
                         at::Tensor weight, at::Tensor bias, c10::optional<at::Tensor> running_mean,
                         c10::optional<at::Tensor> running_var, at::Tensor mean, at::Tensor invstd, at::Tensor scale,
                         at::Tensor shift, int64_t C, double eps, double momentum, bool relu,
                         c10::optional<at::Tensor> mask_out) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC && C >= 8, "fused BN needs C % 8 == 0 and 8 <= C <= 2048");
  const int64_t M = x.numel() / C;
  check_act(x, "x", M * C);
  check_act(y, "y", M * C);
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.numel() == 2 * C * nrb,
              "part must be f32 [2, C, nrb]");
  const uint16_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    check_act(*res, "residual", M * C);
    rp = (const uint16_t*)res->data_ptr();
  }
  for (auto* t : {&weight, &bias, &mean, &invstd, &scale, &shift}) check_vec(*t, "per-channel vector", (int)C);
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    check_vec(*running_mean, "running_mean", (int)C);
    check_vec(*running_var, "running_var", (int)C);
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  uint8_t* mo = nullptr;
  if (mask_out.has_value() && mask_out->defined()) {
    TORCH_CHECK(mask_out->is_cuda() && mask_out->scalar_type() == at::kByte && mask_out->numel() == M * C / 8,
                "mask_out must be uint8[M*C/8]");
    mo = (uint8_t*)mask_out->data_ptr();
  }
  finalize_apply_fwd(part, (int)nrb, x, rp, y, mo, weight, bias, rm, rv, mean, invstd, scale, shift, M, C, eps,
                     momentum, relu, c10::hip::getCurrentHIPStream());
}
}  // namespace hipps

namespace hipps {
// Backward BN whose reduction (sum dz, sum dz*x-hat per channel) was already done by the
// producer of dy -- the 1x1 dgrad GEMM epilogue (gemm.hip, BnBwdTap): finalize + apply only,
// i.e. one pass over dy and x instead of two.  part = f32 [2, C, nrb] channel-major partials.
void bn_backward_partials(at::Tensor part, int64_t nrb, at::Tensor dy, at::Tensor x, int64_t mask_mode,
                          at::Tensor weight, at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift,
                          at::Tensor dx, c10::optional<at::Tensor> dres, at::Tensor dweight, at::Tensor dbias, int64_t C,
                          c10::optional<at::Tensor> mask_in, int64_t unr) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC, "fused BN needs C % 8 == 0 and C <= 2048");
  TORCH_CHECK(mask_mode == MASK_NONE || mask_mode == MASK_X || mask_mode == MASK_BITS, "bad mask mode");
  TORCH_CHECK(unr == 0 || unr == 2 || unr == 4, "bn_backward_partials: unr 0 (auto), 2 or 4");
  // 0: 4 vectors in flight per lane on small tensors (latency-bound: layer-4 BN 15.9 -> 11.5 us),
  // 2 on large ones (layer-2 BN 115 vs 126 us), tools/bench_bn_dual.py
  if (unr == 0) unr = (int64_t)x.numel() <= (int64_t(1) << 24) ? 4 : 2;
  const int64_t M = x.numel() / C;
  check_act(dy, "dy", M * C);
  check_act(x, "x", M * C);
  check_act(dx, "dx", M * C);
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.numel() == 2 * C * nrb,
              "part must be f32 [2, C, nrb]");
  const uint8_t* mbp = nullptr;
  if (mask_mode == MASK_BITS) {
    TORCH_CHECK(mask_in.has_value() && mask_in->defined() && mask_in->scalar_type() == at::kByte &&
                    mask_in->numel() == M * C / 8, "MASK_BITS needs a uint8[M*C/8] mask");
    mbp = (const uint8_t*)mask_in->data_ptr();
  }
  uint16_t* drp = nullptr;
  if (dres.has_value() && dres->defined()) {
    check_act(*dres, "dres", M * C);
    drp = (uint16_t*)dres->data_ptr();
  }
  for (auto* t : {&weight, &mean, &invstd, &scale, &shift, &dweight, &dbias}) check_vec(*t, "per-channel vector", (int)C);
  auto coef = at::empty({3, C}, weight.options());
  auto stream = c10::hip::getCurrentHIPStream();
  const float* pa = part.data_ptr<float>();
  fin_bwd( stream, pa, pa + C * nrb,
                     (int)nrb, (int)C, M, weight.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                     dweight.data_ptr<float>(), dbias.data_ptr<float>(), coef[0].data_ptr<float>(),
                     coef[1].data_ptr<float>(), coef[2].data_ptr<float>());
  auto app = [&](auto kern) {
    hipLaunchKernelGGL(kern, apply_grid(M, (int)C), kBlock, 0, stream, (const uint16_t*)dy.data_ptr(),
                       (const uint16_t*)x.data_ptr(), nullptr, mbp, scale.data_ptr<float>(), shift.data_ptr<float>(),
                       coef[0].data_ptr<float>(), coef[1].data_ptr<float>(), coef[2].data_ptr<float>(),
                       (uint16_t*)dx.data_ptr(), drp, M, (int)C);
  };
  if (bn_pipe()) {
    switch (mask_mode) {
      case MASK_NONE: app(k_bn_apply_bwd<MASK_NONE, 0>); break;
      case MASK_X: app(k_bn_apply_bwd<MASK_X, 0>); break;
      default: app(k_bn_apply_bwd<MASK_BITS, 0>); break;
    }
  } else if (unr == 4) {
    switch (mask_mode) {
      case MASK_NONE: app(k_bn_apply_bwd<MASK_NONE, 4>); break;
      case MASK_X: app(k_bn_apply_bwd<MASK_X, 4>); break;
      default: app(k_bn_apply_bwd<MASK_BITS, 4>); break;
    }
  } else {
    switch (mask_mode) {
      case MASK_NONE: app(k_bn_apply_bwd<MASK_NONE>); break;
      case MASK_X: app(k_bn_apply_bwd<MASK_X>); break;
      default: app(k_bn_apply_bwd<MASK_BITS>); break;
    }
  }
}
}  // namespace hipps

namespace hipps {
// z = relu(bn3(x3) + bnd(xd)) for a ResNet downsample block, both BNs' statistics from their
// producers' epilogues (part3 [2, C, nrb3], partd [2, C, nrbd]): two finalizes and ONE apply pass
// that reads x3 and the pre-BN downsample output xd -- the downsample BN's output is never
// written or re-read.  mask: uint8 [M*C/8] ReLU bits of z.
void bn_dual_forward(at::Tensor part3, int64_t nrb3, at::Tensor partd, int64_t nrbd, at::Tensor x3, at::Tensor xd,
                     at::Tensor z, at::Tensor mask, at::Tensor w3, at::Tensor b3, at::Tensor rm3, at::Tensor rv3,
                     at::Tensor mean3, at::Tensor invstd3, at::Tensor scale3, at::Tensor shift3, at::Tensor wd,
                     at::Tensor bd, at::Tensor rmd, at::Tensor rvd, at::Tensor meand, at::Tensor invstdd,
                     at::Tensor scaled, at::Tensor shiftd, int64_t C, double eps3, double mom3, double epsd,
                     double momd) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC && C >= 8, "fused BN needs C % 8 == 0 and 8 <= C <= 2048");
  const int64_t M = x3.numel() / C;
  check_act(x3, "x3", M * C);
  check_act(xd, "xd", M * C);
  check_act(z, "z", M * C);
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.numel() == M * C / 8, "mask: uint8[M*C/8]");
  for (const at::Tensor* p : {&part3, &partd})
    TORCH_CHECK(p->is_cuda() && p->scalar_type() == at::kFloat && p->is_contiguous(), "partials: f32");
  TORCH_CHECK(part3.numel() == 2 * C * nrb3 && partd.numel() == 2 * C * nrbd, "partials: [2, C, nrb]");
  for (auto* t : {&w3, &b3, &rm3, &rv3, &mean3, &invstd3, &scale3, &shift3, &wd, &bd, &rmd, &rvd, &meand, &invstdd,
                  &scaled, &shiftd})
    check_vec(*t, "per-channel vector", (int)C);
  auto stream = c10::hip::getCurrentHIPStream();
  auto fin = [&](const at::Tensor& part, int64_t nrb, at::Tensor& w, at::Tensor& b, at::Tensor& rm, at::Tensor& rv,
                 at::Tensor& mean, at::Tensor& invstd, at::Tensor& scale, at::Tensor& shift, double eps, double mom) {
    const float* pa = part.data_ptr<float>();
    fin_fwd( stream, pa, pa + C * nrb,
                       (int)nrb, (int)C, M, w.data_ptr<float>(), b.data_ptr<float>(), (float)eps, (float)mom,
                       rm.data_ptr<float>(), rv.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                       scale.data_ptr<float>(), shift.data_ptr<float>());
  };
  fin(part3, nrb3, w3, b3, rm3, rv3, mean3, invstd3, scale3, shift3, eps3, mom3);
  fin(partd, nrbd, wd, bd, rmd, rvd, meand, invstdd, scaled, shiftd, epsd, momd);
  hipLaunchKernelGGL(apply_fwd_kernel(M, (int)C), apply_grid(M, (int)C), kBlock, 0, stream, (const uint16_t*)x3.data_ptr(),
                     (const uint16_t*)xd.data_ptr(), (uint16_t*)z.data_ptr(), (uint8_t*)mask.data_ptr(),
                     scale3.data_ptr<float>(), shift3.data_ptr<float>(), M, (int)C, 1, scaled.data_ptr<float>(),
                     shiftd.data_ptr<float>(), bits_pack());
}

// Backward of bn_dual_forward: dx3 (bn3's input gradient), dxd (the downsample BN's), the four
// affine gradients.  part3: bn3's backward reduction from the consumer's dgrad epilogue
// (BNGradTap) or none (reduced here).  Passes: [reduce bn3] -> finalize -> dx3 + the downsample
// BN's reduction in one pass (k_bn_bwd_dual) -> finalize -> dxd.
void bn_dual_backward(c10::optional<at::Tensor> part3, int64_t nrb3, at::Tensor dz, at::Tensor x3, at::Tensor xd,
                      at::Tensor mask, at::Tensor w3, at::Tensor mean3, at::Tensor invstd3, at::Tensor wd,
                      at::Tensor meand, at::Tensor invstdd, at::Tensor dx3, at::Tensor dxd, at::Tensor dw3,
                      at::Tensor db3, at::Tensor dwd, at::Tensor dbd, int64_t C, int64_t unr) {
  TORCH_CHECK(C % 8 == 0 && C <= kMaxC && C >= 8, "fused BN needs C % 8 == 0 and 8 <= C <= 2048");
  const int64_t M = x3.numel() / C;
  for (auto* t : {&dz, &x3, &xd, &dx3, &dxd}) check_act(*t, "activation", M * C);
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.numel() == M * C / 8, "mask: uint8[M*C/8]");
  for (auto* t : {&w3, &mean3, &invstd3, &wd, &meand, &invstdd, &dw3, &db3, &dwd, &dbd})
    check_vec(*t, "per-channel vector", (int)C);
  auto stream = c10::hip::getCurrentHIPStream();
  const auto* mbp = (const uint8_t*)mask.data_ptr();
  int nrb;
  const int64_t rows = pick_rows(M, (int)C, nrb);
  at::Tensor p3;
  int64_t n3 = nrb3;
  if (part3.has_value() && part3->defined()) {
    p3 = *part3;
    TORCH_CHECK(p3.is_cuda() && p3.scalar_type() == at::kFloat && p3.is_contiguous() && p3.numel() == 2 * C * nrb3,
                "part3: f32 [2, C, nrb3]");
  } else {
    p3 = at::empty({2, C, (int64_t)nrb}, w3.options());
    n3 = nrb;
    hipLaunchKernelGGL((k_bn_reduce<true, MASK_BITS, 4>), nrb, kBlock, 0, stream, (const uint16_t*)x3.data_ptr(),
                       (const uint16_t*)dz.data_ptr(), nullptr, mbp, mean3.data_ptr<float>(), invstd3.data_ptr<float>(),
                       nullptr, nullptr, M, (int)C, rows, nrb, p3[0].data_ptr<float>(), p3[1].data_ptr<float>());
  }
  auto coef3 = at::empty({3, C}, w3.options());
  auto coefd = at::empty({3, C}, w3.options());
  auto pd = at::empty({2, C, (int64_t)nrb}, w3.options());
  auto finb = [&](const float* pa, int64_t n, at::Tensor& w, at::Tensor& mean, at::Tensor& invstd, at::Tensor& dw,
                  at::Tensor& db, at::Tensor& coef) {
    fin_bwd( stream, pa, pa + C * n, (int)n,
                       (int)C, M, w.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                       dw.data_ptr<float>(), db.data_ptr<float>(), coef[0].data_ptr<float>(), coef[1].data_ptr<float>(),
                       coef[2].data_ptr<float>());
  };
  finb(p3.data_ptr<float>(), n3, w3, mean3, invstd3, dw3, db3, coef3);
  auto dual = [&](auto kern) {
    hipLaunchKernelGGL(kern, nrb, kBlock, 0, stream, (const uint16_t*)dz.data_ptr(), (const uint16_t*)x3.data_ptr(),
                       (const uint16_t*)xd.data_ptr(), mbp, coef3[0].data_ptr<float>(), coef3[1].data_ptr<float>(),
                       coef3[2].data_ptr<float>(), meand.data_ptr<float>(), invstdd.data_ptr<float>(),
                       (uint16_t*)dx3.data_ptr(), M, (int)C, rows, nrb, pd[0].data_ptr<float>(), pd[1].data_ptr<float>());
  };
  TORCH_CHECK(unr == 2 || unr == 4 || unr == 8, "bn_dual_backward: unr 2, 4 or 8");
  if (unr == 2) dual(k_bn_bwd_dual<2>);
  else if (unr == 8) dual(k_bn_bwd_dual<8>);
  else dual(k_bn_bwd_dual<4>);
  finb(pd.data_ptr<float>(), nrb, wd, meand, invstdd, dwd, dbd, coefd);
  auto appk = bn_pipe() ? k_bn_apply_bwd<MASK_BITS, 0> : k_bn_apply_bwd<MASK_BITS>;
  hipLaunchKernelGGL(appk, apply_grid(M, (int)C), kBlock, 0, stream,
                     (const uint16_t*)dz.data_ptr(), (const uint16_t*)xd.data_ptr(), nullptr, mbp, nullptr, nullptr,
                     coefd[0].data_ptr<float>(), coefd[1].data_ptr<float>(), coefd[2].data_ptr<float>(),
                     (uint16_t*)dxd.data_ptr(), nullptr, M, (int)C);
}
}  // namespace hipps
