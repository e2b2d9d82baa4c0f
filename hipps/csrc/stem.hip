// hipps — ResNet stem: 7x7 / stride 2 / pad 3 convolution of a 3-channel channels-last bf16 image
// into 64 channels, forward (with the next BatchNorm's batch statistics in the epilogue) and weight
// gradient, both on v_mfma_f32_16x16x32_bf16.
//
// Cin = 3 makes this a GEMM with a 147-long reduction (k = (ky*7 + kx)*3 + c, the physical order of
// a channels-last [64, 3, 7, 7] weight) over M = images*112*112 rows.  Library implicit-GEMM
// kernels tile that K poorly (MIOpen: 366 us forward / 350 us weight gradient + zero fills at
// batch 256, about 10 % of MFMA peak, profiles/bench_n1_steady_r2c.txt); the useful floor is the
// HBM traffic: 411 MB of bf16 output (forward) or dy (weight gradient) plus 77 MB of input.
//
// Both kernels stage whole input ROWS in LDS: one output row reads 7 input rows, and in NHWC a
// 7-pixel window of one input row is 21 CONSECUTIVE bf16 values (kx, c) -- so the forward's
// B fragment (8 consecutive k of one output pixel) is 8 consecutive LDS elements.  Each ky gets
// its own 32-deep k step (21 real values, 11 zero-weighted ones; compute is not the bound here).
//
// Forward:  C[cout][px] = W[cout][k] * X[k][px]: lanes own output pixels, so the epilogue's
// BatchNorm statistics are a 16-lane reduction; the weight fragments (7 ky x 4 cout tiles) stay
// in registers for the whole block.  Weight gradient: dW[cout][k] = sum_px dy[px][cout] X[px][k],
// dy staged per output row and read transposed (ds_read_b64_tr_b16), X gathered from the staged
// rows; per-block fp32 slabs + a fixed-order sum (deterministic).
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kCout = 64, kTaps = 7, kKS = 21;  // 7x7 taps, 7*3 values per (ky) row
constexpr int kK = kTaps * kKS;                  // 147
constexpr int kSRG = 8;                          // forward: output rows per block
constexpr int kSRows = 2 * kSRG + 5;             // forward: staged input rows
constexpr int kLead = 16;                        // LDS row: 16 zero elements before column 0

// LDS element of output pixel wo's window start (input column 2*wo - 3, channel 0) within a staged
// row: kLead + 3 * (2*wo - 3) = 6*wo + 7 (odd: fragments are read as 5 dwords + funnel shifts)
__device__ __forceinline__ int win0(int wo) { return 6 * wo + kLead - 9; }

// 8 consecutive bf16 at an ODD element offset e of a 4-byte-aligned LDS row (5 dword reads + funnel
// shifts), masked per lane group: q = 2 keeps k 16..20 (21..23 are the next pixel's values),
// q = 3 (k 24..31) is zero.  Branch-free: q is lane-dependent, so an if on it would serialize both
// paths and their LDS reads under exec masks.
struct OddMask {
  uint32_t m01, m2, m3;
};
__device__ __forceinline__ OddMask odd_mask(int q) {
  return OddMask{q < 3 ? ~0u : 0u, q < 2 ? ~0u : (q == 2 ? 0xffffu : 0u), q < 2 ? ~0u : 0u};
}
__device__ __forceinline__ bf16x8 lds_frag_odd(const uint16_t* base, int e, const OddMask& m) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(base) + ((e - 1) >> 1);
  const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
  const u32x4 v{__builtin_amdgcn_alignbit(d1, d0, 16) & m.m01, __builtin_amdgcn_alignbit(d2, d1, 16) & m.m01,
                __builtin_amdgcn_alignbit(d3, d2, 16) & m.m2, __builtin_amdgcn_alignbit(d4, d3, 16) & m.m3};
  return __builtin_bit_cast(bf16x8, v);
}

// Stage input rows [hi0, hi0 + rows) of image img into LDS rows of `pitch` elements: kLead zeros,
// 3*Wi values, zeros to the pitch; rows outside the image are zero.  16-byte chunks (Wi % 8 == 0).
__device__ __forceinline__ void stage_rows(uint16_t* lds, const uint16_t* __restrict__ X, int img, int hi0, int rows,
                                           int Hi, int Wi, int pitch, int t, int nthr) {
  const int cpr = pitch / 8, data = 3 * Wi;
  for (int i = t; i < rows * cpr; i += nthr) {
    const int r = i / cpr, c = i - r * cpr;
    const int e = c * 8 - kLead, hi = hi0 + r;
    u32x4 v{0u, 0u, 0u, 0u};
    if (hi >= 0 && hi < Hi && e >= 0 && e < data)
      v = *reinterpret_cast<const u32x4*>(X + ((int64_t)img * Hi + hi) * data + e);
    *reinterpret_cast<u32x4*>(lds + r * pitch + c * 8) = v;
  }
}

// ------------------------------------------------------------------------------------------
// forward: persistent blocks (one resident wave of them) loop over row groups = (image, kSRG
// output rows); the 4 waves of a block share the 7*kSRG pixel fragments of a group.  The weight
// fragments are loaded once per block; the statistics are one partial column per block.
//
// Staged rows hold 4 channels per pixel (c = 3 is zero), pixel slot s = input column s - 3: the
// window of output pixel wo starts at slot 2*wo, i.e. 16-byte aligned, and k = 4*kx + c of one ky
// is 8 consecutive slots -- every B fragment (k = 8q .. 8q+7) is ONE ds_read_b128 (slots 2wo+2q,
// 2wo+2q+1).  q = 3's upper half (slot 2wo+7, kx = 7) is masked.  The 3-channel layout needed five
// dword reads + funnel shifts per fragment and left the MFMAs waiting on LDS (242 us).
constexpr int kFwdTask = 8;  // input pixels per staging task (3 x 16-byte loads -> 8 x 8-byte writes)
constexpr int kFwdRT = 3;    // staging tasks per thread per group (prefetched in registers)

__device__ __forceinline__ uint32_t elem16(const uint32_t (&d)[12], int k) {  // k: compile-time
  return (d[k >> 1] >> ((k & 1) * 16)) & 0xffffu;
}

__global__ __launch_bounds__(256) void k_stem_fwd(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                  uint16_t* __restrict__ Y, float* __restrict__ pa,
                                                  float* __restrict__ pb, int Hi, int Wi, int Ho, int Wo, int pitch,
                                                  int rgs, int ngroups) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int b = blockIdx.x, nblk = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, q = lane >> 4, il = lane & 15;
  const int stage_elems = kSRows * pitch, slots = pitch / 4;

  // lead / tail slots (outside the image columns) are zero in both buffers and never rewritten
  for (int i = t; i < 2 * kSRows * slots; i += 256) {
    const int sl = i % slots;
    if (sl < 3 || sl >= 3 + Wi) *reinterpret_cast<uint2*>(lds + (size_t)i * 4) = uint2{0u, 0u};
  }

  // wave w: cout tiles {2 hc, 2 hc + 1} (hc = w & 1) of the pixel fragments of wave pair w >> 1;
  // weight fragments A[cout = 16 f + il][k = 8 q + j], k = 4 kx + c, in registers (zero for c = 3
  // and kx = 7)
  const int hc = w & 1, wp = w >> 1;
  bf16x8 wf[kTaps][2];
#pragma unroll
  for (int ky = 0; ky < kTaps; ++ky)
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const uint16_t* src = W + (32 * hc + 16 * f + il) * kK + ky * kKS;
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kx = 2 * q + (j >> 2), c = j & 3;
        const bool ok = c < 3 && kx < kTaps;
        const short x = (short)src[ok ? 3 * kx + c : 0];  // clamped, in-bounds read
        v[j] = ok ? x : (short)0;
      }
      wf[ky][f] = v;
    }
  const uint32_t m23 = q < 3 ? ~0u : 0u;  // q = 3: k 28..31 (kx = 7) -> zero

  const int fpr = (Wo + 15) >> 4;  // 16-pixel fragments per output row
  const int nfr = kSRG * fpr;
  float s[2][4], sq[2][4];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[f][r] = sq[f][r] = 0.f;

  // staging tasks: (row r, 8 input pixels from column 8 g); register prefetch of the next group
  const int gpr = Wi / kFwdTask, ntask = kSRows * gpr, data = 3 * Wi;
  u32x4 rx[kFwdRT][3];
#define HIPPS_STEMF_GLOAD(g_)                                                                      \
  {                                                                                                \
    const int img_ = (g_) / rgs, hi0_ = 2 * ((g_) - img_ * rgs) * kSRG - 3;                         \
    _Pragma("unroll") for (int u = 0; u < kFwdRT; ++u) {                                           \
      const int i_ = t + 256 * u;                                                                  \
      const int r_ = i_ / gpr, g8_ = i_ - r_ * gpr, hi_ = hi0_ + r_;                               \
      const bool ok_ = i_ < ntask && hi_ >= 0 && hi_ < Hi;                                         \
      const int64_t o_ = ok_ ? ((int64_t)img_ * Hi + hi_) * data + 3 * kFwdTask * g8_ : 0;          \
      _Pragma("unroll") for (int v = 0; v < 3; ++v) {                                              \
        const u32x4 x_ = *reinterpret_cast<const u32x4*>(X + o_ + 8 * v);                          \
        rx[u][v] = ok_ ? x_ : u32x4{0u, 0u, 0u, 0u};                                               \
      }                                                                                            \
    }                                                                                              \
  }
#define HIPPS_STEMF_SSTORE(s_)                                                                     \
  {                                                                                                \
    _Pragma("unroll") for (int u = 0; u < kFwdRT; ++u) {                                           \
      const int i_ = t + 256 * u;                                                                  \
      if (i_ < ntask) {                                                                            \
        const int r_ = i_ / gpr, g8_ = i_ - r_ * gpr;                                              \
        const uint32_t d_[12] = {rx[u][0].x, rx[u][0].y, rx[u][0].z, rx[u][0].w,                    \
                                 rx[u][1].x, rx[u][1].y, rx[u][1].z, rx[u][1].w,                    \
                                 rx[u][2].x, rx[u][2].y, rx[u][2].z, rx[u][2].w};                   \
        uint16_t* dst_ = lds + (s_) * stage_elems + r_ * pitch + 4 * (3 + kFwdTask * g8_);         \
        _Pragma("unroll") for (int px = 0; px < kFwdTask; ++px)                                    \
          *reinterpret_cast<uint2*>(dst_ + 4 * px) =                                               \
              uint2{elem16(d_, 3 * px) | (elem16(d_, 3 * px + 1) << 16), elem16(d_, 3 * px + 2)};  \
      }                                                                                            \
    }                                                                                              \
  }
  if (b < ngroups) {
    HIPPS_STEMF_GLOAD(b);
    HIPPS_STEMF_SSTORE(0);
  }
  __syncthreads();
  for (int g = b, it = 0; g < ngroups; g += nblk, ++it) {
    const int img = g / rgs, ho0 = (g - img * rgs) * kSRG;
    const int cur = it & 1;
    const bool more = g + nblk < ngroups;
    if (more) HIPPS_STEMF_GLOAD(g + nblk);
    const uint16_t* xs = lds + cur * stage_elems;
    for (int p0 = 2 * wp; p0 < nfr; p0 += 4) {  // two pixel fragments per pass
      int rl[2], wo[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int fr = min(p0 + p, nfr - 1);
        rl[p] = fr / fpr;
        wo[p] = (fr - rl[p] * fpr) * 16 + il;
      }
      // all 14 B fragments of the pass first (one b128 each), then the 28 MFMAs
      bf16x8 xb[kTaps][2];
#pragma unroll
      for (int ky = 0; ky < kTaps; ++ky)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          u32x4 v = *reinterpret_cast<const u32x4*>(xs + (2 * rl[p] + ky) * pitch + 8 * wo[p] + 8 * q);
          v.z &= m23;
          v.w &= m23;
          xb[ky][p] = __builtin_bit_cast(bf16x8, v);
        }
      f32x4 acc[2][2];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int f = 0; f < 2; ++f) acc[p][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ky = 0; ky < kTaps; ++ky)
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int f = 0; f < 2; ++f)
            acc[p][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ky][f], xb[ky][p], acc[p][f], 0, 0, 0);
      // D map: column (pixel) = il, row (cout within the 16-tile) = 4 q + r
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int ho = ho0 + rl[p];
        const bool ok = p0 + p < nfr && ho < Ho && wo[p] < Wo;
        if (!ok) continue;
        uint16_t* dst = Y + (((int64_t)img * Ho + ho) * Wo + wo[p]) * kCout + 32 * hc + 4 * q;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          uint16_t h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            h[r] = f32_to_bf16(acc[p][f][r]);
            const float v = bf16_to_f32(h[r]);
            s[f][r] += v;
            sq[f][r] = fmaf(v, v, sq[f][r]);
          }
          *reinterpret_cast<uint2*>(dst + 16 * f) =
              uint2{(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
        }
      }
    }
    // the other buffer's last readers finished before the barrier that ended the previous group
    if (more) HIPPS_STEMF_SSTORE(cur ^ 1);
    __syncthreads();
  }  // row groups
#undef HIPPS_STEMF_GLOAD
#undef HIPPS_STEMF_SSTORE
  if (pa == nullptr) return;
  // statistics: sum over the 16 pixel lanes of each q group, then over the 2 wave pairs (fixed order)
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        s[f][r] += __shfl_xor(s[f][r], m, 64);
        sq[f][r] += __shfl_xor(sq[f][r], m, 64);
      }
    }
  float* red = reinterpret_cast<float*>(lds);  // [2 wave pairs][64 couts][2]
  if (il == 0) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 32 * hc + 16 * f + 4 * q + r;
        red[(wp * kCout + c) * 2] = s[f][r];
        red[(wp * kCout + c) * 2 + 1] = sq[f][r];
      }
  }
  __syncthreads();
  if (t < kCout) {
    pa[(int64_t)t * nblk + b] = red[t * 2] + red[(kCout + t) * 2];
    pb[(int64_t)t * nblk + b] = red[t * 2 + 1] + red[(kCout + t) * 2 + 1];
  }
}

// ------------------------------------------------------------------------------------------
// weight gradient: block = (image, range of output rows), one output row per stage:
//   dy row  -> LDS [Wpad px][64 ch] (swizzled 16-byte chunks, read transposed)
//   7 input rows -> LDS rows of `pitch` elements (as the forward)
// wave w owns k fragments {w, w+4, w+8} (k = 16 kf + il < 147) of all 4 cout tiles.
constexpr int kWPx = 128;  // staged dy row: up to 128 output pixels (Wo <= 128)

__device__ __forceinline__ int dy_off(int row, int ch) {  // byte offset in a [rows][64 x bf16] tile
  return 128 * row + 16 * (ch ^ (((row & 3) << 1) | ((row >> 2) & 1)));
}

__device__ __forceinline__ bf16x8 dy_frag(const uint8_t* tile, int row0, int col0, int lane) {
  // rows row0 + 8*(lane>>4) + {0..7}, columns col0..col0+15: the A map (row = lane&15, k = 8q + j)
  const int il = lane & 15, qq = il >> 2, p = il & 3;
  const int r = row0 + 8 * (lane >> 4) + qq;
  const int ch = (col0 >> 3) + (p >> 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + dy_off(r, ch) + 8 * (p & 1)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + dy_off(r + 4, ch) + 8 * (p & 1)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Fused stem backward: the gradient reaching the stem conv output y (= the BatchNorm input) is
//   dy = a * dz * [y*scale + shift > 0] + k1 * y + k0,   dz = max-pool gather of dp (4-bit tap codes)
// (BN backward with the ReLU mask recomputed from y; a, k1, k0 from k_bn_finalize_bwd).  Neither dz
// nor dy is materialised: k_stem_pool_bwd_reduce computes dz on the fly for the BN reductions and
// the weight gradient's dy staging recomputes it (bf16-rounded exactly where the unfused pool
// backward / BN backward store it, so the staged dy equals the unfused kernels' output).
struct StemBnPoolBwd {
  const uint16_t* dp;     // pooled gradient [imgs, 64, Hp, Wp] channels-last bf16
  const uint32_t* code;   // tap codes, one uint32 per (pooled pixel, 8 channels)
  const uint16_t* y;      // stem conv output = BN input [imgs, 64, Ho, Wo]
  const float *scale, *shift, *ca, *ck1, *ck0;
  int Hp, Wp;
};

__device__ __forceinline__ void ld8f(const uint16_t* p, float v[8]) {
  const u32x4 u = *reinterpret_cast<const u32x4*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  v[4] = __uint_as_float(u.z << 16); v[5] = __uint_as_float(u.z & 0xffff0000u);
  v[6] = __uint_as_float(u.w << 16); v[7] = __uint_as_float(u.w & 0xffff0000u);
}

// dz (bf16-rounded, before the ReLU mask) of pixel (img, h, w), channels 8g .. 8g+7: the pool
// backward's gather, same window order as k_maxpool3s2_bwd
__device__ __forceinline__ void pool_dz8(const StemBnPoolBwd& f, int img, int h, int w, int g, float dz[8]) {
  // candidate windows (h>>1 | (h>>1)+1) x (w>>1 | (w>>1)+1); the +1 ones exist for odd h / w inside
  // the pooled map.  Static 2x2 with predicates: the 4 code / dp loads are independent and issue
  // together (a data-dependent loop serialised them)
  const int oh0 = h >> 1, ow0 = w >> 1;
  const bool h1 = (h & 1) && oh0 + 1 < f.Hp, w1 = (w & 1) && ow0 + 1 < f.Wp;
  uint32_t c[4];
  u32x4 d[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int oh = oh0 + (k >> 1), ow = ow0 + (k & 1);
    const bool ok = (!(k >> 1) || h1) && (!(k & 1) || w1);
    const int64_t o = ok ? ((int64_t)(img * f.Hp + oh) * f.Wp + ow) * (kCout / 8) + g : 0;
    const uint32_t cv = f.code[o];
    const u32x4 dv = *reinterpret_cast<const u32x4*>(f.dp + o * 8);
    c[k] = ok ? cv : 0xffffffffu;  // tap 15 never matches
    d[k] = dv;
  }
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // same (oh, ow) order as k_maxpool3s2_bwd
    const uint32_t tap = (uint32_t)((h - 2 * (oh0 + (k >> 1)) + 1) * 3 + (w - 2 * (ow0 + (k & 1)) + 1));
    const uint32_t dw[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = __uint_as_float(j & 1 ? dw[j >> 1] & 0xffff0000u : dw[j >> 1] << 16);
      acc[j] += ((c[k] >> (4 * j)) & 15u) == tap ? v : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) dz[j] = bf16_to_f32(f32_to_bf16(acc[j]));
}

// dz (bf16-rounded) of the 2x2 block of input pixels (2kb + a, 2jb + b), a, b in {0, 1}, channels
// 8g .. 8g+7 (pixel p = 2a + b).  All four lie in the same four windows (kb | kb+1) x (jb | jb+1) --
// the odd-odd pixel's candidates -- so the block loads 4 codes + 4 dp vectors instead of up to 16.
// Each pixel sums its windows in pool_dz8's order, adding +0 for the others (a window of the
// next row / column covers only the block's odd rows / columns): bit-identical dz.
__device__ __forceinline__ void pool_dz8_quad(const StemBnPoolBwd& f, int img, int kb, int jb, int g,
                                              float dz[4][8]) {
  uint32_t c[4];
  u32x4 d[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int oh = kb + (r >> 1), ow = jb + (r & 1);
    const bool ok = oh < f.Hp && ow < f.Wp;
    const int64_t o = ok ? ((int64_t)(img * f.Hp + oh) * f.Wp + ow) * (kCout / 8) + g : 0;
    const uint32_t cv = f.code[o];
    const u32x4 dv = *reinterpret_cast<const u32x4*>(f.dp + o * 8);
    c[r] = ok ? cv : 0xffffffffu;
    d[r] = dv;
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int a = p >> 1, b = p & 1;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // a window of the next row (column) holds only odd-row (odd-column) pixels of the block
      const bool in = (r >> 1) <= a && (r & 1) <= b;
      const uint32_t tap = in ? (uint32_t)((a - 2 * (r >> 1) + 1) * 3 + (b - 2 * (r & 1) + 1)) : 0xffffffffu;
      const uint32_t dw[4] = {d[r].x, d[r].y, d[r].z, d[r].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = __uint_as_float(j & 1 ? dw[j >> 1] & 0xffff0000u : dw[j >> 1] << 16);
        acc[j] += ((c[r] >> (4 * j)) & 15u) == tap ? v : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) dz[p][j] = bf16_to_f32(f32_to_bf16(acc[j]));
  }
}

// BN backward reductions over dz * relu'(y): a[c] = sum dz', b[c] = sum dz' * (y - mean) * invstd,
// per block partials pa/pb[c][block] (the format k_bn_finalize_bwd combines).  Lane = 8 channels of
// one pixel; the grid stride is a multiple of the 8 channel groups, so each lane keeps its group.
__global__ __launch_bounds__(256) void k_stem_pool_bwd_reduce(StemBnPoolBwd f, const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, int Ho, int Wo,
                                                              int64_t total, float* __restrict__ pa,
                                                              float* __restrict__ pb) {
  __shared__ float red[2][256][9];  // +1 pad
  constexpr int G = kCout / 8;
  const int t = threadIdx.x, g = t % G;
  float sc[8], sh[8], mu[8], is[8], sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = f.scale[8 * g + j];
    sh[j] = f.shift[8 * g + j];
    mu[j] = mean[8 * g + j];
    is[j] = invstd[8 * g + j];
    sa[j] = sb[j] = 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * 256;
  // kU items per trip, every item's gathers and y loads issued before any is reduced (one item per
  // trip left the loop latency-bound: 368 us per batch-256 stem, 1.5 TB/s; two: 274 us; four: 311)
  constexpr int kU = 2;
  for (int64_t v0 = (int64_t)blockIdx.x * 256 + t; v0 < total; v0 += kU * stride) {
    float dz[kU][8], yv[kU][8];
    bool ok[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t v = v0 + u * stride;
      ok[u] = v < total;
      const int64_t vc = ok[u] ? v : v0;  // (a clamped, valid item; its values are not used)
      // 32-bit index decomposition (the host checks total < 2^32); int64 div/mod dominated
      const uint32_t px = (uint32_t)vc / G;
      const uint32_t r = px / (uint32_t)Wo;
      const int w = (int)(px - r * (uint32_t)Wo);
      const int img = (int)(r / (uint32_t)Ho), h = (int)(r - (uint32_t)img * (uint32_t)Ho);
      pool_dz8(f, img, h, w, g, dz[u]);
      ld8f(f.y + vc * 8, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (!ok[u]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = fmaf(yv[u][j], sc[j], sh[j]) > 0.f ? dz[u][j] : 0.f;
        sa[j] += d;
        sb[j] = fmaf(d, (yv[u][j] - mu[j]) * is[j], sb[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][t][j] = sa[j];
    red[1][t][j] = sb[j];
  }
  __syncthreads();
  if (t < kCout) {  // channel t: group t / 8, element t % 8, summed over the 256 / G lanes in order
    const int gg = t >> 3, j = t & 7;
    float a = 0.f, c = 0.f;
    for (int l = gg; l < 256; l += G) {
      a += red[0][l][j];
      c += red[1][l][j];
    }
    pa[(int64_t)t * gridDim.x + blockIdx.x] = a;
    pb[(int64_t)t * gridDim.x + blockIdx.x] = c;
  }
}

// k_stem_pool_bwd_reduce over 2x2 pixel blocks (pool_dz8_quad): item = (block, channel group),
// total = imgs * Hb * Wb * 8 with Hb = ceil(Ho / 2); the four pixels accumulate in row-major order.
// One block per trip (178 us per batch-256 stem; two per trip measured 204 us)
__global__ __launch_bounds__(256) void k_stem_pool_bwd_reduce_q(StemBnPoolBwd f, const float* __restrict__ mean,
                                                                const float* __restrict__ invstd, int Ho, int Wo,
                                                                int64_t total, float* __restrict__ pa,
                                                                float* __restrict__ pb) {
  __shared__ float red[2][256][9];  // +1 pad
  constexpr int G = kCout / 8;
  const int t = threadIdx.x, g = t % G;
  const int Hb = (Ho + 1) >> 1, Wb = (Wo + 1) >> 1;
  float sc[8], sh[8], mu[8], is[8], sa[8], sb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = f.scale[8 * g + j];
    sh[j] = f.shift[8 * g + j];
    mu[j] = mean[8 * g + j];
    is[j] = invstd[8 * g + j];
    sa[j] = sb[j] = 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t v = (int64_t)blockIdx.x * 256 + t; v < total; v += stride) {
    const uint32_t q = (uint32_t)v / G;  // (the host checks total < 2^32)
    const uint32_t r = q / (uint32_t)Wb;
    const int jb = (int)(q - r * (uint32_t)Wb);
    const int img = (int)(r / (uint32_t)Hb), kb = (int)(r - (uint32_t)img * (uint32_t)Hb);
    float dz[4][8], yv[4][8];
    bool ok[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int h = 2 * kb + (p >> 1), w = 2 * jb + (p & 1);
      ok[p] = h < Ho && w < Wo;
      const int hc = ok[p] ? h : 2 * kb, wc = ok[p] ? w : 2 * jb;  // (a valid pixel; values unused)
      ld8f(f.y + (((int64_t)img * Ho + hc) * Wo + wc) * kCout + 8 * g, yv[p]);
    }
    pool_dz8_quad(f, img, kb, jb, g, dz);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (!ok[p]) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = fmaf(yv[p][j], sc[j], sh[j]) > 0.f ? dz[p][j] : 0.f;
        sa[j] += d;
        sb[j] = fmaf(d, (yv[p][j] - mu[j]) * is[j], sb[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][t][j] = sa[j];
    red[1][t][j] = sb[j];
  }
  __syncthreads();
  if (t < kCout) {
    const int gg = t >> 3, j = t & 7;
    float a = 0.f, c = 0.f;
    for (int l = gg; l < 256; l += G) {
      a += red[0][l][j];
      c += red[1][l][j];
    }
    pa[(int64_t)t * gridDim.x + blockIdx.x] = a;
    pb[(int64_t)t * gridDim.x + blockIdx.x] = c;
  }
}

// staged dy chunk (bf16 x 8) of pixel (img, h, w), channel group g: the BN backward apply on the
// recomputed dz, bit-for-bit the expression of k_bn_apply_bwd<MASK_X>
__device__ __forceinline__ u32x4 bnpool_dy8(const StemBnPoolBwd& f, int img, int h, int w, int g, int Ho, int Wo) {
  float dz[8], yv[8], o[8];
  pool_dz8(f, img, h, w, g, dz);
  ld8f(f.y + (((int64_t)img * Ho + h) * Wo + w) * kCout + 8 * g, yv);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = 8 * g + j;
    const float d = fmaf(yv[j], f.scale[c], f.shift[c]) > 0.f ? dz[j] : 0.f;
    o[j] = fmaf(f.ca[c], d, fmaf(f.ck1[c], yv[j], f.ck0[c]));
  }
  return u32x4{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]), pack_bf16x2(o[6], o[7])};
}

// dy = BN-backward(pool-backward(dp)) written out (mode 2 of stem_bnpool_backward): one lane = 8
// channels of one stem-output pixel, the same bits the weight gradient's fused staging computes
__global__ __launch_bounds__(256) void k_stem_bnpool_dy(StemBnPoolBwd f, int Ho, int Wo, int64_t total,
                                                        uint16_t* __restrict__ dy) {
  constexpr int G = kCout / 8;
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= total) return;
  const uint32_t px = (uint32_t)v / G, g = (uint32_t)v - px * G;  // (the host checks total < 2^32)
  const uint32_t r = px / (uint32_t)Wo;
  const int w = (int)(px - r * (uint32_t)Wo);
  const int img = (int)(r / (uint32_t)Ho), h = (int)(r - (uint32_t)img * (uint32_t)Ho);
  *reinterpret_cast<u32x4*>(dy + v * 8) = bnpool_dy8(f, img, h, w, (int)g, Ho, Wo);
}

// k_stem_bnpool_dy over 2x2 pixel blocks (pool_dz8_quad): the same bits per pixel
__global__ __launch_bounds__(256) void k_stem_bnpool_dy_q(StemBnPoolBwd f, int Ho, int Wo, int64_t total,
                                                          uint16_t* __restrict__ dy) {
  constexpr int G = kCout / 8;
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= total) return;
  const int Hb = (Ho + 1) >> 1, Wb = (Wo + 1) >> 1;
  const uint32_t q = (uint32_t)v / G, g = (uint32_t)v - q * G;
  const uint32_t r = q / (uint32_t)Wb;
  const int jb = (int)(q - r * (uint32_t)Wb);
  const int img = (int)(r / (uint32_t)Hb), kb = (int)(r - (uint32_t)img * (uint32_t)Hb);
  float dz[4][8], yv[4][8];
  bool ok[4];
  int64_t off[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int h = 2 * kb + (p >> 1), w = 2 * jb + (p & 1);
    ok[p] = h < Ho && w < Wo;
    off[p] = (((int64_t)img * Ho + (ok[p] ? h : 2 * kb)) * Wo + (ok[p] ? w : 2 * jb)) * kCout + 8 * g;
    ld8f(f.y + off[p], yv[p]);
  }
  pool_dz8_quad(f, img, kb, jb, (int)g, dz);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (!ok[p]) continue;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * g + j;
      const float d = fmaf(yv[p][j], f.scale[c], f.shift[c]) > 0.f ? dz[p][j] : 0.f;
      o[j] = fmaf(f.ca[c], d, fmaf(f.ck1[c], yv[p][j], f.ck0[c]));
    }
    *reinterpret_cast<u32x4*>(dy + off[p]) =
        u32x4{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]), pack_bf16x2(o[6], o[7])};
  }
}

template <bool PRO>
__global__ __launch_bounds__(256) void k_stem_wgrad(const uint16_t* __restrict__ dY, const uint16_t* __restrict__ X,
                                                    float* __restrict__ part, int Hi, int Wi, int Ho, int Wo,
                                                    int pitch, int rows_per_blk, int splits, StemBnPoolBwd fb) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  // [2 stages][dy tile kWPx x 64 | 7 input rows x pitch]
  const int stage_elems = kWPx * kCout + kTaps * pitch;
  const int b = blockIdx.x;
  const int img = b / splits, hb = (b - img * splits) * rows_per_blk, he = min(Ho, hb + rows_per_blk);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, q = lane >> 4, il = lane & 15;

  // dy tile rows past Wo stay zero (their B values are zero too, but 0 * garbage may be NaN)
  for (int i = t; i < 2 * (kWPx - Wo) * 8; i += 256) {
    const int s = i / ((kWPx - Wo) * 8), rem = i - s * (kWPx - Wo) * 8;
    const int row = Wo + rem / 8, ch = rem % 8;
    *reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(lds + s * stage_elems) + dy_off(row, ch)) =
        u32x4{0u, 0u, 0u, 0u};
  }

  // this lane's k column of each owned fragment: LDS offset (row ky, + 3 kx + c) or -1 (k >= 147)
  int koff[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int k = 16 * (w + 4 * i) + il;
    const int ky = k / kKS, rem = k - ky * kKS;
    koff[i] = (w + 4 * i < 10 && k < kK) ? ky * pitch + rem : -1;
  }
  const int nkf = w < 2 ? 3 : 2;

  f32x4 acc[4][3];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[f][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // staging with register prefetch: the next row's global loads are in flight during this row's
  // MFMAs (<= 4 dy chunks + <= 4 input-row chunks per thread; checked on the host)
  const int dch = Wo * 8;  // 16-byte chunks in a dy row
  const int cpr = pitch / 8, xch = kTaps * cpr, data = 3 * Wi;
  u32x4 rdy[4], rx[4];
#define HIPPS_STEM_GLOAD(ho_)                                                                      \
  {                                                                                                \
    const uint16_t* src_ = dY + ((int64_t)img * Ho + (ho_)) * Wo * kCout;                          \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                                \
      const int i_ = t + 256 * u;                                                                  \
      const int j_ = i_ < dch ? i_ : 0;                                                            \
      if constexpr (PRO) {                                                                         \
        rdy[u] = u32x4{0u, 0u, 0u, 0u};                                                            \
        if (i_ < dch) rdy[u] = bnpool_dy8(fb, img, (ho_), j_ >> 3, j_ & 7, Ho, Wo);                \
      } else {                                                                                     \
        const u32x4 v_ = *reinterpret_cast<const u32x4*>(src_ + (int64_t)(j_ >> 3) * kCout + (j_ & 7) * 8); \
        rdy[u] = i_ < dch ? v_ : u32x4{0u, 0u, 0u, 0u};                                            \
      }                                                                                            \
    }                                                                                              \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                                \
      const int i_ = t + 256 * u;                                                                  \
      const int r_ = i_ / cpr, e_ = (i_ - r_ * cpr) * 8 - kLead, hi_ = 2 * (ho_) - 3 + r_;          \
      const bool ok_ = i_ < xch && hi_ >= 0 && hi_ < Hi && e_ >= 0 && e_ < data;                   \
      const int64_t o_ = ok_ ? ((int64_t)img * Hi + hi_) * data + e_ : 0;                         \
      const u32x4 v_ = *reinterpret_cast<const u32x4*>(X + o_);                                    \
      rx[u] = ok_ ? v_ : u32x4{0u, 0u, 0u, 0u};                                                    \
    }                                                                                              \
  }
#define HIPPS_STEM_SSTORE(s_)                                                                      \
  {                                                                                                \
    uint16_t* base_ = lds + (s_) * stage_elems;                                                    \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                                \
      const int i_ = t + 256 * u;                                                                  \
      if (i_ < dch) *reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(base_) + dy_off(i_ >> 3, i_ & 7)) = rdy[u]; \
    }                                                                                              \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                                \
      const int i_ = t + 256 * u;                                                                  \
      if (i_ < xch) *reinterpret_cast<u32x4*>(base_ + kWPx * kCout + i_ * 8) = rx[u];              \
    }                                                                                              \
  }

  if (hb < he) {
    HIPPS_STEM_GLOAD(hb);
    HIPPS_STEM_SSTORE(0);
  }
  __syncthreads();
  const int nch = (Wo + 31) >> 5;  // 32-pixel reduction steps per row
  for (int ho = hb; ho < he; ++ho) {
    const int cur = (ho - hb) & 1;
    if (ho + 1 < he) HIPPS_STEM_GLOAD(ho + 1);
    const uint16_t* base = lds + cur * stage_elems;
    const uint8_t* dyt = reinterpret_cast<const uint8_t*>(base);
    const uint16_t* xr = base + kWPx * kCout;
    for (int c = 0; c < nch; ++c) {
      bf16x8 a[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) a[f] = dy_frag(dyt, 32 * c, 16 * f, lane);
      const int px0 = 32 * c + 8 * q;  // this lane's 8 pixels px0 .. px0 + 7
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (i >= nkf) break;
        // (a branch-free clamped gather measured slower: 311 vs 221 us at batch 256)
        bf16x8 bv;
        if (koff[i] < 0) {
          bv = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        } else {
          const uint16_t* src = xr + koff[i] + win0(px0);
#pragma unroll
          for (int j = 0; j < 8; ++j) bv[j] = (px0 + j < Wo) ? (short)src[6 * j] : (short)0;
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) acc[f][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f], bv, acc[f][i], 0, 0, 0);
      }
    }
    // the other buffer's last readers finished before the barrier that ended the previous row
    if (ho + 1 < he) HIPPS_STEM_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef HIPPS_STEM_GLOAD
#undef HIPPS_STEM_SSTORE
  // D map: column (k) = il, row (cout) = 16 f + 4 q + r
  float* out = part + (int64_t)b * kCout * kK;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (koff[i] < 0) continue;
    const int k = 16 * (w + 4 * i) + il;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(16 * f + 4 * q + r) * kK + k] = acc[f][i][r];
  }
}

// fixed-order slab sum: level 1 sums slabs [g*S/G, (g+1)*S/G) into tmp[g], level 2 sums the G rows
__global__ __launch_bounds__(kBlock) void k_stem_reduce1(const float* __restrict__ part, int S, int G, int n,
                                                         float* __restrict__ tmp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
  if (i >= n) return;
  const int s0 = (int)((int64_t)g * S / G), s1 = (int)((int64_t)(g + 1) * S / G);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = s0;
  for (; s + 3 < s1; s += 4) {
    a0 += part[(int64_t)s * n + i];
    a1 += part[(int64_t)(s + 1) * n + i];
    a2 += part[(int64_t)(s + 2) * n + i];
    a3 += part[(int64_t)(s + 3) * n + i];
  }
  for (; s < s1; ++s) a0 += part[(int64_t)s * n + i];
  tmp[(int64_t)g * n + i] = (a0 + a1) + (a2 + a3);
}

__global__ __launch_bounds__(kBlock) void k_stem_reduce2(const float* __restrict__ tmp, int G, int n,
                                                         float* __restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a[4] = {0.f, 0.f, 0.f, 0.f};  // independent chains: the G loads are in flight together
  int g = 0;
  for (; g + 3 < G; g += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += tmp[(int64_t)(g + u) * n + i];
  for (; g < G; ++g) a[0] += tmp[(int64_t)g * n + i];
  dw[i] = (a[0] + a[1]) + (a[2] + a[3]);
}

int64_t stem_pitch(int64_t Wi, int64_t Wo) {
  // window reads reach element win0(16*ceil(Wo/16) - 1) + 8*2 + 8 (five dwords of the q = 2 group)
  const int64_t need = std::max<int64_t>(kLead + 3 * Wi + 8, 6 * (16 * ((Wo + 15) / 16)) + kLead + 32);
  return (need + 7) / 8 * 8;
}

void check_geom(const at::Tensor& x, int64_t& Hi, int64_t& Wi, int64_t& Ho, int64_t& Wo) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) == 3 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: x must be a channels-last bf16 [imgs, 3, H, W] tensor");
  Hi = x.size(2);
  Wi = x.size(3);
  TORCH_CHECK(Wi % 8 == 0 && Hi >= 7 && Wi >= 7, "stem: needs W % 8 == 0");
  Ho = (Hi + 6 - 7) / 2 + 1;
  Wo = (Wi + 6 - 7) / 2 + 1;
  TORCH_CHECK(Wo <= kWPx, "stem: output width <= 128");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "stem: 16-byte aligned x");
}

}  // namespace

// forward grid: at most one resident wave of blocks (2 per CU at ~180 VGPRs), every block the same
// number of row groups
static int64_t stem_fwd_grid(int64_t groups) {
  const int64_t per = (groups + 256 * 2 - 1) / (256 * 2);
  return (groups + per - 1) / per;
}

int64_t stem_mtiles(int64_t imgs, int64_t Ho) { return stem_fwd_grid(imgs * ((Ho + kSRG - 1) / kSRG)); }

// x [imgs, 3, H, W], w [64, 3, 7, 7], y [imgs, 64, Ho, Wo]: channels-last bf16.
// part (optional): f32 [2, 64, stem_mtiles] per-block BatchNorm partial sums of the bf16 outputs.
void stem_forward(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part) {
  int64_t Hi, Wi, Ho, Wo;
  check_geom(x, Hi, Wi, Ho, Wo);
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(0) == kCout &&
                  w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem: w must be a channels-last bf16 [64, 3, 7, 7] tensor");
  const int64_t imgs = x.size(0);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.dim() == 4 && y.size(0) == imgs &&
                  y.size(1) == kCout && y.size(2) == Ho && y.size(3) == Wo &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast) && reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0,
              "stem: y must be a channels-last bf16 [imgs, 64, Ho, Wo] tensor");
  const int64_t rgs = (Ho + kSRG - 1) / kSRG, groups = imgs * rgs, nblk = stem_fwd_grid(groups);
  TORCH_CHECK(groups < (int64_t(1) << 31) && y.numel() < (int64_t(1) << 40), "stem: size");
  float *pa = nullptr, *pb = nullptr;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() == 2 * kCout * nblk, "stem: part must be f32 [2, 64, stem_mtiles]");
    pa = part->data_ptr<float>();
    pb = pa + kCout * nblk;
  }
  // slots: 3 lead + Wi image columns, and the last fragment's window reaches slot 2*(16*ceil(Wo/16)-1)+7
  const int64_t slots = (std::max<int64_t>(3 + Wi, 2 * 16 * ((Wo + 15) / 16) + 6) + 1) / 2 * 2;
  const int64_t pitch = 4 * slots;
  const size_t lds = (size_t)std::max<int64_t>(2 * kSRows * pitch * 2, 4 * kCout * 2 * 4);
  TORCH_CHECK(lds <= 160 * 1024 && kSRows * (Wi / kFwdTask) <= kFwdRT * 256, "stem: image too wide for the staged rows");
  if (lds > 64 * 1024)  // 2 blocks per CU still fit the 160 KB
    TORCH_CHECK(hipFuncSetAttribute((const void*)k_stem_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
                    hipSuccess, "stem: LDS attribute");
  hipLaunchKernelGGL(k_stem_fwd, (int)nblk, 256, lds, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)x.data_ptr(), (const uint16_t*)w.data_ptr(), (uint16_t*)y.data_ptr(), pa, pb,
                     (int)Hi, (int)Wi, (int)Ho, (int)Wo, (int)pitch, (int)rgs, (int)groups);
}

void bn_finalize_bwd_partials(at::Tensor part, int64_t nrb, int64_t M, at::Tensor weight, at::Tensor mean,
                              at::Tensor invstd, at::Tensor dweight, at::Tensor dbias, at::Tensor coef);  // norm.hip

static void launch_stem_wgrad(const at::Tensor& dy, const at::Tensor& x, at::Tensor& dw, const StemBnPoolBwd* fb) {
  int64_t Hi, Wi, Ho, Wo;
  check_geom(x, Hi, Wi, Ho, Wo);
  const int64_t imgs = x.size(0);
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == at::kFloat && dw.numel() == kCout * kK &&
                  dw.is_contiguous(at::MemoryFormat::ChannelsLast), "stem_wgrad: dw must be f32 [64, 3, 7, 7] channels-last");
  const int64_t pitch = stem_pitch(Wi, Wo);
  const size_t lds = (size_t)2 * (kWPx * kCout + kTaps * pitch) * 2;
  TORCH_CHECK(lds <= 64 * 1024 && kTaps * (pitch / 8) <= 4 * 256, "stem_wgrad: image too wide for the staged rows");
  // one resident wave of blocks (3 per CU: 52 KB of LDS each); each block sums >= 8 output rows
  const int64_t want = std::max<int64_t>(1, 256 * 3 / imgs);
  const int64_t rows = std::max<int64_t>(8, (Ho + want - 1) / want);
  const int64_t splits = (Ho + rows - 1) / rows, S = imgs * splits;
  TORCH_CHECK(S < (int64_t(1) << 31), "stem_wgrad: grid");
  auto stream = c10::hip::getCurrentHIPStream();
  auto part = at::empty({S, kCout * kK}, dw.options().memory_format(at::MemoryFormat::Contiguous));
  const uint16_t* dyp = fb ? nullptr : (const uint16_t*)dy.data_ptr();
  if (fb)
    hipLaunchKernelGGL(k_stem_wgrad<true>, (int)S, 256, lds, stream, dyp, (const uint16_t*)x.data_ptr(),
                       part.data_ptr<float>(), (int)Hi, (int)Wi, (int)Ho, (int)Wo, (int)pitch, (int)rows, (int)splits,
                       *fb);
  else
    hipLaunchKernelGGL(k_stem_wgrad<false>, (int)S, 256, lds, stream, dyp, (const uint16_t*)x.data_ptr(),
                       part.data_ptr<float>(), (int)Hi, (int)Wi, (int)Ho, (int)Wo, (int)pitch, (int)rows, (int)splits,
                       StemBnPoolBwd{});
  const int n = kCout * kK;
  const int G = (int)std::min<int64_t>(S, 32);
  const unsigned gx = (unsigned)((n + kBlock - 1) / kBlock);
  auto tmp = at::empty({(int64_t)G, (int64_t)n}, part.options());
  hipLaunchKernelGGL(k_stem_reduce1, dim3(gx, G), kBlock, 0, stream, part.data_ptr<float>(), (int)S, G, n,
                     tmp.data_ptr<float>());
  hipLaunchKernelGGL(k_stem_reduce2, gx, kBlock, 0, stream, tmp.data_ptr<float>(), G, n, dw.data_ptr<float>());
}

// dy [imgs, 64, Ho, Wo], x [imgs, 3, H, W] channels-last bf16; dw f32 [64, 3, 7, 7] channels-last
// (written, not accumulated).
void stem_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw) {
  int64_t Hi, Wi, Ho, Wo;
  check_geom(x, Hi, Wi, Ho, Wo);
  const int64_t imgs = x.size(0);
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == imgs &&
                  dy.size(1) == kCout && dy.size(2) == Ho && dy.size(3) == Wo &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0,
              "stem_wgrad: dy must be a 16-byte aligned channels-last bf16 [imgs, 64, Ho, Wo] tensor");
  launch_stem_wgrad(dy, x, dw, nullptr);
}

// Backward of pool(relu(bn(stem(x)))) without materialising the pool gradient (nor, with
// materialize_dy = false, the BN input gradient):
// dp [imgs, 64, Hp, Wp] bf16 + code (max pool tap codes) + y (stem output, BN input); BN vectors
// f32 [64] (weight, mean, invstd, scale, shift).  Writes dbn_w, dbn_b (BN parameter gradients) and
// dw (stem weight gradient, f32 channels-last [64, 3, 7, 7]).  materialize_dy: the BN input
// gradient is written by one elementwise pass and the plain weight gradient reads it (the gather
// inside the weight gradient's staging is latency-bound); otherwise the staging recomputes it.
void stem_bnpool_backward(at::Tensor dp, at::Tensor code, at::Tensor y, at::Tensor x, at::Tensor bn_weight,
                          at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift, at::Tensor dbn_w,
                          at::Tensor dbn_b, at::Tensor dw, bool materialize_dy, bool quad) {
  int64_t Hi, Wi, Ho, Wo;
  check_geom(x, Hi, Wi, Ho, Wo);
  const int64_t imgs = x.size(0), Hp = (Ho - 1) / 2 + 1, Wp = (Wo - 1) / 2 + 1;
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.dim() == 4 && y.size(0) == imgs &&
                  y.size(1) == kCout && y.size(2) == Ho && y.size(3) == Wo &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast) && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
              "stem_bnpool_backward: y must be the channels-last bf16 stem output");
  TORCH_CHECK(dp.is_cuda() && dp.scalar_type() == at::kBFloat16 && dp.dim() == 4 && dp.size(0) == imgs &&
                  dp.size(1) == kCout && dp.size(2) == Hp && dp.size(3) == Wp &&
                  dp.is_contiguous(at::MemoryFormat::ChannelsLast) && reinterpret_cast<uintptr_t>(dp.data_ptr()) % 16 == 0,
              "stem_bnpool_backward: dp must be the channels-last bf16 pooled gradient");
  TORCH_CHECK(code.is_cuda() && code.scalar_type() == at::kInt && code.is_contiguous() &&
                  code.numel() == imgs * Hp * Wp * (kCout / 8), "stem_bnpool_backward: code size");
  for (const at::Tensor* v : {&bn_weight, &mean, &invstd, &scale, &shift, &dbn_w, &dbn_b})
    TORCH_CHECK(v->is_cuda() && v->scalar_type() == at::kFloat && v->is_contiguous() && v->numel() == kCout,
                "stem_bnpool_backward: BN vectors must be f32 [64]");
  auto stream = c10::hip::getCurrentHIPStream();
  StemBnPoolBwd fb{(const uint16_t*)dp.data_ptr(), (const uint32_t*)code.data_ptr(), (const uint16_t*)y.data_ptr(),
                   scale.data_ptr<float>(), shift.data_ptr<float>(), nullptr, nullptr, nullptr, (int)Hp, (int)Wp};
  const int64_t total = imgs * Ho * Wo * (kCout / 8);
  TORCH_CHECK(total < (int64_t(1) << 32), "stem_bnpool_backward: size");
  // 8 resident blocks per CU (18 KB of LDS each): twice the loads in flight of 4
  const int nrb = (int)std::max<int64_t>(1, std::min<int64_t>(256 * 8, (total + 255) / 256));
  auto part = at::empty({2, kCout, (int64_t)nrb}, scale.options());
  // quad: 2x2 pixel blocks per item (one window gather shared by four pixels); else per pixel
  const int64_t qtotal = imgs * ((Ho + 1) / 2) * ((Wo + 1) / 2) * (kCout / 8);
  if (quad)
    hipLaunchKernelGGL(k_stem_pool_bwd_reduce_q, nrb, 256, 0, stream, fb, mean.data_ptr<float>(),
                       invstd.data_ptr<float>(), (int)Ho, (int)Wo, qtotal, part[0].data_ptr<float>(),
                       part[1].data_ptr<float>());
  else
    hipLaunchKernelGGL(k_stem_pool_bwd_reduce, nrb, 256, 0, stream, fb, mean.data_ptr<float>(),
                       invstd.data_ptr<float>(), (int)Ho, (int)Wo, total, part[0].data_ptr<float>(),
                       part[1].data_ptr<float>());
  auto coef = at::empty({3, kCout}, scale.options());
  bn_finalize_bwd_partials(part, nrb, imgs * Ho * Wo, bn_weight, mean, invstd, dbn_w, dbn_b, coef);
  fb.ca = coef[0].data_ptr<float>();
  fb.ck1 = coef[1].data_ptr<float>();
  fb.ck0 = coef[2].data_ptr<float>();
  if (materialize_dy) {
    auto dy = at::empty_like(y, y.options(), at::MemoryFormat::ChannelsLast);
    if (quad)
      hipLaunchKernelGGL(k_stem_bnpool_dy_q, (unsigned)((qtotal + 255) / 256), 256, 0, stream, fb, (int)Ho, (int)Wo,
                         qtotal, (uint16_t*)dy.data_ptr());
    else
      hipLaunchKernelGGL(k_stem_bnpool_dy, (unsigned)((total + 255) / 256), 256, 0, stream, fb, (int)Ho, (int)Wo,
                         total, (uint16_t*)dy.data_ptr());
    launch_stem_wgrad(dy, x, dw, nullptr);
  } else {
    launch_stem_wgrad(y, x, dw, &fb);
  }
}

}  // namespace hipps
