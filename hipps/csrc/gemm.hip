// hipps — MFMA 1x1-convolution GEMM for channels-last bf16 activations, with the next
// BatchNorm's batch statistics fused into the epilogue.
//
//   Y[M, N] = X[M, K] · W[N, K]^T      M = images*Ho*Wo rows, K = Cin, N = Cout
//
// A 1x1 convolution on NHWC memory is exactly this "NT" GEMM: both operands are K-contiguous,
// so every MFMA fragment (8 consecutive k of one row, v_mfma_f32_16x16x32_bf16) is ONE 16-byte
// LDS read.  The epilogue converts the fp32 accumulators to bf16, stages the tile through LDS
// for full-line 16-byte stores, and (STATS) reduces per-output-channel sum / sum-of-squares of
// the stored bf16 values into channel-major partials part[c][m_tile] -- the format the fused
// BatchNorm finalize (norm.hip) consumes.  That removes the BN forward's separate read pass
// over the convolution output (ResNet-50: 36 of 53 convolutions are 1x1).
//
// Tiling: 128 x BN x 64 (BN = 128 or 64), 4 waves (2x2 or 4x1), each wave a 64x64 / 32x64
// sub-tile of 16x16 MFMA accumulators; two LDS stages with register prefetch (the global loads
// of k-tile t+1 are in flight during the MFMAs of tile t; one barrier per k-tile).  LDS rows are
// 128 B with a 16-byte-chunk XOR swizzle (chunk ^= row & 7) so the 16 rows a fragment read
// touches spread over the banks.  Blocks are remapped so consecutive tiles (the N tiles of one
// M tile, which share the X rows) land on the same XCD and hit its L2.
// Strided 1x1 convolutions (ResNet downsample, stride 2) gather their rows in the A loader.
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // native vector: HIP uint4 is a struct

constexpr int kGBM = 128, kGBK = 64;

template <int BN> struct GemmCfg;
template <> struct GemmCfg<128> { static constexpr int WM = 2, WN = 2; };
template <> struct GemmCfg<64> { static constexpr int WM = 4, WN = 1; };

template <int BN>
constexpr int gemm_lds_elems() {
  // max(2 stages of A+B tiles, epilogue tile with 8-element row pad) + stats scratch (floats)
  constexpr int stage = 2 * (kGBM + BN) * kGBK;
  constexpr int epi = kGBM * (BN + 8);
  return (stage > epi ? stage : epi) + 2 * 2 * GemmCfg<BN>::WM * BN;
}

__device__ __forceinline__ uint32_t add_bf16x2(uint32_t a, uint32_t b) {
  return pack_bf16x2(__uint_as_float(a << 16) + __uint_as_float(b << 16),
                     __uint_as_float(a & 0xffff0000u) + __uint_as_float(b & 0xffff0000u));
}

// Backward BatchNorm statistics in the dgrad epilogue.  When the GEMM output Y is the COMPLETE
// gradient dy of a training BatchNorm's output (the conv is that BN output's only consumer, every
// other gradient path having been summed in through R), the BN backward's reduction pass
//   a[c] = sum_m dz,  b[c] = sum_m dz * (x - mean) * invstd,  dz = dy * relu'
// is done here on the tile still in registers (+ one read of the BN input x), instead of by a
// separate kernel that re-reads dy and x.  relu' = the BN's stored ReLU bits, or recomputed from
// x*scale + shift > 0 (bits == nullptr).  Per-M-tile partials go to pa/pb[c][mtile].
struct BnBwdTap {
  const uint16_t* x;
  const uint8_t* bits;
  const float *mean, *invstd, *scale, *shift;
};

__device__ const uint8_t kOnes[16] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                      0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};

// A-operand prologue: X is the INPUT of a training BatchNorm + ReLU whose output this conv
// consumes; each staged 16-byte chunk (8 channels) becomes bf16(max(x * scale[c] + shift[c], 0))
// -- the same rounding as the BN apply kernel -- so the BN output is never written to HBM.
__device__ __forceinline__ u32x4 bn_relu8(u32x4 v, const float (&sc)[8], const float (&sh)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lo = fmaxf(fmaf(__uint_as_float(w[j] << 16), sc[2 * j], sh[2 * j]), 0.f);
    const float hi = fmaxf(fmaf(__uint_as_float(w[j] & 0xffff0000u), sc[2 * j + 1], sh[2 * j + 1]), 0.f);
    o[j] = pack_bf16x2(lo, hi);
  }
  return u32x4{o[0], o[1], o[2], o[3]};
}

// KxK convolutions as implicit GEMM over K = KH*KW*Cin (k = (r*KW + s)*Cin + c, the physical order
// of a channels-last [Cout, Cin, KH, KW] weight); a 64-deep K tile stays inside one tap (Cin % 64
// == 0), so the A loader reads input pixel (ho*stride - pad + r, wo*stride - pad + s), zeros
// outside the image.  KH = KW = 1, pad = 0 is the plain 1x1 path.
struct ConvGeom {
  int KW, pad, Cin;
};

template <int BN, bool STATS, bool ADD, int BST = 0, bool PRO = false, bool TAPS = false>
__global__ __launch_bounds__(256) void k_conv1x1_nt(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                    uint16_t* __restrict__ Y, float* __restrict__ pa,
                                                    float* __restrict__ pb, const uint16_t* __restrict__ R,
                                                    const uint8_t* __restrict__ RM, int M, int N, int K, int Ho,
                                                    int Wo, int Hi, int Wi, int stride, int mtiles, int ntiles,
                                                    BnBwdTap bt, const float* __restrict__ psc,
                                                    const float* __restrict__ psh, ConvGeom cg) {
  constexpr int WM = GemmCfg<BN>::WM, WN = GemmCfg<BN>::WN;
  constexpr int TM = kGBM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_CH = kGBM * kGBK / 8 / 256;  // 16-byte chunks per thread per stage
  constexpr int B_CH = BN * kGBK / 8 / 256;
  constexpr int STAGE = (kGBM + BN) * kGBK;  // elements
  constexpr int EP = BN + 8;                 // epilogue row pitch (elements)
  __shared__ __attribute__((aligned(16))) uint16_t lds[gemm_lds_elems<BN>()];

  // XCD-aware tile order: hardware deals block ids round-robin to the 8 XCDs; give each XCD a
  // contiguous range of logical tiles so the N tiles of one M tile share an L2.
  int bid = blockIdx.x;
  const int nblk = gridDim.x;
  if ((nblk & 7) == 0) bid = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int m0 = mt * kGBM, n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w / WN, wn = w % WN;
  const int cchunk = t & 7;  // the 16-byte chunk (k/8) this thread stages, fixed

  // per-thread A source rows (fixed over the K loop); rows past M load zeros
  int64_t a_off[A_CH];
  bool a_ok[A_CH];
  int a_h[TAPS ? A_CH : 1], a_w[TAPS ? A_CH : 1];  // TAPS: top-left input pixel of the row's window
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int row = (t >> 3) + 32 * i;
    int m = m0 + row;
    a_ok[i] = m < M;
    m = a_ok[i] ? m : M - 1;
    int64_t src = m;
    if (TAPS || stride != 1) {
      const int hw = Ho * Wo;
      const int img = m / hw, rem = m - img * hw;
      const int ho = rem / Wo, wo = rem - ho * Wo;
      if constexpr (TAPS) {
        a_h[i] = ho * stride - cg.pad;
        a_w[i] = wo * stride - cg.pad;
        src = (int64_t)img * Hi * Wi;  // pixel index of the image's first pixel
      } else {
        src = ((int64_t)img * Hi + (int64_t)ho * stride) * Wi + (int64_t)wo * stride;
      }
    }
    a_off[i] = TAPS ? src : src * K + cchunk * 8;
  }
  int64_t b_off[B_CH];
#pragma unroll
  for (int i = 0; i < B_CH; ++i) b_off[i] = (int64_t)(n0 + (t >> 3) + 32 * i) * K + cchunk * 8;

  u32x4 ra[A_CH], rb[B_CH];
  float psr[PRO ? 8 : 1], phr[PRO ? 8 : 1];  // prologue scale / shift of this thread's 8 channels
  // (macros, not lambdas: a by-reference lambda capture of these arrays put them in scratch)
#define HIPPS_GLOAD(kt_)                                                        \
  {                                                                             \
    const int k0_ = (kt_) * kGBK;                                               \
    if constexpr (TAPS) {                                                       \
      const int tap_ = k0_ / cg.Cin, c0_ = k0_ - tap_ * cg.Cin;                 \
      const int r_ = tap_ / cg.KW, s_ = tap_ - r_ * cg.KW;                      \
      _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                        \
        const int hi_ = a_h[i] + r_, wi_ = a_w[i] + s_;                         \
        const bool ok_ = a_ok[i] && hi_ >= 0 && hi_ < Hi && wi_ >= 0 && wi_ < Wi; \
        const int64_t o_ = ok_ ? (a_off[i] + (int64_t)hi_ * Wi + wi_) * cg.Cin + c0_ + cchunk * 8 : 0; \
        u32x4 v_ = *reinterpret_cast<const u32x4*>(X + o_);                     \
        ra[i] = ok_ ? v_ : u32x4{0u, 0u, 0u, 0u};                               \
      }                                                                         \
    } else {                                                                    \
      _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                        \
        u32x4 v_ = *reinterpret_cast<const u32x4*>(X + a_off[i] + k0_);         \
        ra[i] = a_ok[i] ? v_ : u32x4{0u, 0u, 0u, 0u};                           \
      }                                                                         \
    }                                                                           \
    _Pragma("unroll") for (int i = 0; i < B_CH; ++i) rb[i] =                    \
        *reinterpret_cast<const u32x4*>(W + b_off[i] + k0_);                    \
    if constexpr (PRO) {                                                        \
      const int c_ = k0_ + cchunk * 8; /* 32-byte aligned: four 16-byte loads */ \
      const float4 s0_ = *reinterpret_cast<const float4*>(psc + c_);            \
      const float4 s1_ = *reinterpret_cast<const float4*>(psc + c_ + 4);        \
      const float4 h0_ = *reinterpret_cast<const float4*>(psh + c_);            \
      const float4 h1_ = *reinterpret_cast<const float4*>(psh + c_ + 4);        \
      psr[0] = s0_.x; psr[1] = s0_.y; psr[2] = s0_.z; psr[3] = s0_.w;           \
      psr[4] = s1_.x; psr[5] = s1_.y; psr[6] = s1_.z; psr[7] = s1_.w;           \
      phr[0] = h0_.x; phr[1] = h0_.y; phr[2] = h0_.z; phr[3] = h0_.w;           \
      phr[4] = h1_.x; phr[5] = h1_.y; phr[6] = h1_.z; phr[7] = h1_.w;           \
    }                                                                           \
  }
#define HIPPS_SSTORE(s_)                                                                           \
  {                                                                                                \
    uint16_t* base_ = lds + (s_) * STAGE;                                                          \
    _Pragma("unroll") for (int i = 0; i < A_CH; ++i) {                                             \
      const int row_ = (t >> 3) + 32 * i;                                                          \
      u32x4 v_ = ra[i];                                                                            \
      if constexpr (PRO) v_ = a_ok[i] ? bn_relu8(v_, psr, phr) : u32x4{0u, 0u, 0u, 0u};          \
      *reinterpret_cast<u32x4*>(base_ + row_ * kGBK + ((cchunk ^ (row_ & 7)) << 3)) = v_;         \
    }                                                                                              \
    _Pragma("unroll") for (int i = 0; i < B_CH; ++i) {                                             \
      const int row_ = (t >> 3) + 32 * i;                                                          \
      *reinterpret_cast<u32x4*>(base_ + kGBM * kGBK + row_ * kGBK + ((cchunk ^ (row_ & 7)) << 3)) = \
          rb[i];                                                                                   \
    }                                                                                              \
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = K / kGBK;
  constexpr int RCH = BN / 8;                // 16-byte chunks per output row
  constexpr int NOUT = kGBM * RCH / 256;     // output chunks per thread
  u32x4 rr[NOUT];                            // epilogue addend, prefetched during the last k-tile
  uint32_t rmb[NOUT];
  u32x4 bx[NOUT];                            // BST: the BN input x under the output tile
  uint32_t bmb[NOUT];
  // optional mask streams are read unconditionally (a missing one reads byte 0 of kOnes): a
  // select between "load" and "constant" makes hipcc branch around each load and drain vmcnt
  const uint8_t* rmp = RM != nullptr ? RM : kOnes;
  const int64_t rmk = RM != nullptr ? ~int64_t(0) : 0;
  const uint8_t* bmp = bt.bits;
  HIPPS_GLOAD(0);
  HIPPS_SSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) {
      HIPPS_GLOAD(kt + 1);
    } else if ((ADD || BST) && !(ADD && BST)) {  // last tile: load the epilogue operand now, under the MFMAs
#pragma unroll
      for (int i = 0; i < NOUT; ++i) {
        const int id = t + 256 * i;
        const int row = id / RCH, c = id - row * RCH;
        const bool ok = m0 + row < M;
        const int64_t o = (int64_t)(ok ? m0 + row : m0) * N + n0 + c * 8;
        if (ADD) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(R + o);
          rr[i] = ok ? v : u32x4{0u, 0u, 0u, 0u};
          rmb[i] = rmp[(o >> 3) & rmk];
        }
        if (BST && !ADD) {  // with ADD too, these wait for the epilogue (register budget: 2 waves/SIMD)
          bx[i] = *reinterpret_cast<const u32x4*>(bt.x + o);
          if (BST == 2) bmb[i] = bmp[o >> 3];
        }
      }
    }
    const uint16_t* As = lds + cur * STAGE;
    const uint16_t* Bs = As + kGBM * kGBK;
#pragma unroll
    for (int ks = 0; ks < kGBK / 32; ++ks) {
      const int c = ks * 4 + (lane >> 4);
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * TM + i * 16 + (lane & 15);
        a[i] = *reinterpret_cast<const bf16x8*>(As + row * kGBK + ((c ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * TN + j * 16 + (lane & 15);
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + row * kGBK + ((c ^ (row & 7)) << 3));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) HIPPS_SSTORE(cur ^ 1);
    __syncthreads();
  }

#undef HIPPS_GLOAD
#undef HIPPS_SSTORE
  // ---- epilogue: bf16 tile -> LDS (padded rows), per-channel stats, 16-byte row stores ----
  // C/D map (16x16x32): column = lane & 15, row = (lane >> 4) * 4 + r.
  float* st = reinterpret_cast<float*>(lds + (2 * STAGE > kGBM * EP ? 2 * STAGE : kGBM * EP));
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = wn * TN + j * 16 + (lane & 15);
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const uint16_t hb = f32_to_bf16(acc[i][j][r]);
        lds[row * EP + col] = hb;
        if (STATS) {
          const float v = bf16_to_f32(hb);
          s += v;
          q = fmaf(v, v, q);
        }
      }
    }
    if (STATS) {
      s += __shfl_xor(s, 16, 64);
      q += __shfl_xor(q, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) {
        st[(wm * BN + col) * 2] = s;
        st[(wm * BN + col) * 2 + 1] = q;
      }
    }
  }
  __syncthreads();
  if (BST && ADD) {  // both operands loaded only now, with the accumulators retired to LDS: held
#pragma unroll       // through the last k-tile they cost 2 -> 1 waves/SIMD (276 registers)
    for (int i = 0; i < NOUT; ++i) {
      const int id = t + 256 * i;
      const int row = id / RCH, c = id - row * RCH;
      const bool ok = m0 + row < M;
      const int64_t o = (int64_t)(ok ? m0 + row : m0) * N + n0 + c * 8;
      const u32x4 v = *reinterpret_cast<const u32x4*>(R + o);
      rr[i] = ok ? v : u32x4{0u, 0u, 0u, 0u};
      rmb[i] = rmp[(o >> 3) & rmk];
      bx[i] = *reinterpret_cast<const u32x4*>(bt.x + o);
      if (BST == 2) bmb[i] = bmp[o >> 3];
    }
  }
  // BST: this thread's 8 channels are fixed (256 % RCH == 0): per-channel BN constants in registers
  const int cc = (t % RCH) * 8;
  float bmu[8], bis[8], bsc[8], bsh[8], bsa[8], bsb[8];
  if (BST) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bmu[j] = bt.mean[n0 + cc + j];
      bis[j] = bt.invstd[n0 + cc + j];
      bsc[j] = BST == 1 ? bt.scale[n0 + cc + j] : 0.f;
      bsh[j] = BST == 1 ? bt.shift[n0 + cc + j] : 0.f;
      bsa[j] = 0.f;
      bsb[j] = 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < NOUT; ++i) {
    const int id = t + 256 * i;
    const int row = id / RCH, c = id - row * RCH;
    if (m0 + row < M) {
      const int64_t o = (int64_t)(m0 + row) * N + n0 + c * 8;
      uint4 v = *reinterpret_cast<const uint4*>(lds + row * EP + c * 8);
      if (ADD) {  // fused "+ R" (R * ReLU-mask bits): a second gradient path into Y
        u32x4 r = rr[i];
        const uint32_t mb = rmb[i];  // one mask byte per 8 channels = this 16-byte chunk
        r.x &= (mb & 1u ? 0xffffu : 0u) | (mb & 2u ? 0xffff0000u : 0u);
        r.y &= (mb & 4u ? 0xffffu : 0u) | (mb & 8u ? 0xffff0000u : 0u);
        r.z &= (mb & 16u ? 0xffffu : 0u) | (mb & 32u ? 0xffff0000u : 0u);
        r.w &= (mb & 64u ? 0xffffu : 0u) | (mb & 128u ? 0xffff0000u : 0u);
        v.x = add_bf16x2(v.x, r.x);
        v.y = add_bf16x2(v.y, r.y);
        v.z = add_bf16x2(v.z, r.z);
        v.w = add_bf16x2(v.w, r.w);
      }
      *reinterpret_cast<uint4*>(Y + o) = v;
      if (BST) {  // dz = dy * relu'(.) on the stored bf16 dy; x-hat from the BN input
        const uint32_t dv[4] = {v.x, v.y, v.z, v.w};
        const u32x4 xu = bx[i];
        const uint32_t xw[4] = {xu.x, xu.y, xu.z, xu.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = __uint_as_float(j & 1 ? dv[j >> 1] & 0xffff0000u : dv[j >> 1] << 16);
          const float xv = __uint_as_float(j & 1 ? xw[j >> 1] & 0xffff0000u : xw[j >> 1] << 16);
          const bool on = BST == 2 ? ((bmb[i] >> j) & 1u) != 0u : fmaf(xv, bsc[j], bsh[j]) > 0.f;
          const float dz = on ? d : 0.f;
          bsa[j] += dz;
          bsb[j] = fmaf(dz, (xv - bmu[j]) * bis[j], bsb[j]);
        }
      }
    }
  }
  if (BST) {  // combine the 256/RCH row lanes of each channel chunk through LDS, fixed order
    constexpr int RL = 256 / RCH;
    float* red = reinterpret_cast<float*>(lds);  // [2][RL][BN] floats = 16 KB; the staging area is free
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(t / RCH) * BN + cc + j] = bsa[j];
      red[RL * BN + (t / RCH) * BN + cc + j] = bsb[j];
    }
    __syncthreads();
    if (t < BN) {
      float s = 0.f, q = 0.f;
      for (int r = 0; r < RL; ++r) {
        s += red[r * BN + t];
        q += red[RL * BN + r * BN + t];
      }
      pa[(int64_t)(n0 + t) * mtiles + mt] = s;
      pb[(int64_t)(n0 + t) * mtiles + mt] = q;
    }
  }
  if (STATS && t < BN) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      s += st[(i * BN + t) * 2];
      q += st[(i * BN + t) * 2 + 1];
    }
    pa[(int64_t)(n0 + t) * mtiles + mt] = s;
    pb[(int64_t)(n0 + t) * mtiles + mt] = q;
  }
}


// ==========================================================================================
// Weight gradient:  dW[N][K] = sum_m dY[m][N] * X[src(m)][K]   (reduction over the M rows)
//
// Both operands arrive M-major (row m, channels contiguous), but an MFMA fragment wants 8
// consecutive REDUCTION indices (m) per lane.  The tiles are staged row-major in LDS and read
// back with gfx950's transposing ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses
// row q / columns 4p..4p+3 and lane i receives column i of the 4 rows -- exactly the 16x16x32
// A/B lane map (row = lane&15, k = 8*(lane>>4) + j) after two reads (rows +0..3, +4..7).
// LDS rows are 256 B (128 channels) with the XOR chunk swizzle
// ch ^ (((row&3)<<2) | ((row>>2)&3)) so the transposed reads spread over the banks.
// The M range is split into S chunks (S * tiles ~ 2048 blocks); each block writes an fp32
// partial tile and a second kernel sums the S partials in a fixed order (deterministic).
constexpr int kWT = 128, kWMS = 64;  // output tile kWT x kWT; m rows per LDS stage

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int wg_off(int row, int ch) {  // byte offset in a [rows][128 x bf16] tile
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ bf16x8 tr_frag(const uint8_t* tile, int row0, int col0, int lane) {
  // rows row0 + 8*(lane>>4) + {0..3, 4..7}, columns col0 .. col0+15 (col0 % 16 == 0)
  const int il = lane & 15, q = il >> 2, p = il & 3;
  const int r = row0 + 8 * (lane >> 4) + q;
  const int ch = (col0 >> 3) + (p >> 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + wg_off(r, ch) + 8 * (p & 1)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + wg_off(r + 4, ch) + 8 * (p & 1)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__global__ __launch_bounds__(256) void k_conv1x1_wgrad(const uint16_t* __restrict__ dY, const uint16_t* __restrict__ X,
                                                       float* __restrict__ part, int M, int N, int K, int Ho, int Wo,
                                                       int Hi, int Wi, int stride, int chunk, int tn, int tk) {
  constexpr int TILE = kWMS * kWT;  // elements of one operand tile
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * TILE];  // 2 stages x (dY, X)
  int bid = blockIdx.x;
  const int nblk = gridDim.x;
  if ((nblk & 7) == 0) bid = (bid & 7) * (nblk >> 3) + (bid >> 3);  // M chunk's tiles share an XCD
  const int tiles = tn * tk;
  const int sidx = bid / tiles, tile = bid - sidx * tiles;
  const int n0 = (tile / tk) * kWT, k0 = (tile % tk) * kWT;
  const int mbeg = sidx * chunk, mend = min(M, mbeg + chunk);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wn = w >> 1, wk = w & 1;  // 2x2 waves, 64x64 each
  const int ch = t & 15;              // staged 16-byte chunk (8 channels), fixed
  const bool n_ok = n0 + ch * 8 < N, k_ok = k0 + ch * 8 < K;

  u32x4 ry[4], rx[4];
#define HIPPS_WLOAD(mb_)                                                                           \
  {                                                                                                \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                \
      const int m_ = (mb_) + (t >> 4) + 16 * i;                                                   \
      const bool ok_ = m_ < mend;                                                                  \
      const int mc_ = ok_ ? m_ : mbeg;                                                             \
      int64_t src_ = mc_;                                                                          \
      if (stride != 1) {                                                                           \
        const int hw_ = Ho * Wo, img_ = mc_ / hw_, rem_ = mc_ - img_ * hw_;                        \
        const int ho_ = rem_ / Wo, wo_ = rem_ - ho_ * Wo;                                          \
        src_ = ((int64_t)img_ * Hi + (int64_t)ho_ * stride) * Wi + (int64_t)wo_ * stride;          \
      }                                                                                            \
      const u32x4 vy_ = *reinterpret_cast<const u32x4*>(dY + (int64_t)mc_ * N + (n_ok ? n0 + ch * 8 : 0)); \
      const u32x4 vx_ = *reinterpret_cast<const u32x4*>(X + src_ * K + (k_ok ? k0 + ch * 8 : 0));  \
      ry[i] = (ok_ && n_ok) ? vy_ : u32x4{0u, 0u, 0u, 0u};                                         \
      rx[i] = (ok_ && k_ok) ? vx_ : u32x4{0u, 0u, 0u, 0u};                                         \
    }                                                                                              \
  }
#define HIPPS_WSTORE(s_)                                                                           \
  {                                                                                                \
    uint8_t* ty_ = reinterpret_cast<uint8_t*>(lds + (s_) * 2 * TILE);                              \
    uint8_t* tx_ = ty_ + TILE * 2;                                                                 \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                \
      const int r_ = (t >> 4) + 16 * i;                                                            \
      *reinterpret_cast<u32x4*>(ty_ + wg_off(r_, ch)) = ry[i];                                     \
      *reinterpret_cast<u32x4*>(tx_ + wg_off(r_, ch)) = rx[i];                                     \
    }                                                                                              \
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = (mend - mbeg + kWMS - 1) / kWMS;
  HIPPS_WLOAD(mbeg);
  HIPPS_WSTORE(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) HIPPS_WLOAD(mbeg + (st + 1) * kWMS);
    const uint8_t* ty = reinterpret_cast<const uint8_t*>(lds + cur * 2 * TILE);
    const uint8_t* tx = ty + TILE * 2;
#pragma unroll
    for (int ks = 0; ks < kWMS / 32; ++ks) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = tr_frag(ty, ks * 32, wn * 64 + i * 16, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = tr_frag(tx, ks * 32, wk * 64 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nst) HIPPS_WSTORE(cur ^ 1);
    __syncthreads();
  }
#undef HIPPS_WLOAD
#undef HIPPS_WSTORE
  // D map: column (k) = lane & 15, row (n) = (lane >> 4) * 4 + r
  float* out = part + (int64_t)sidx * N * K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wk * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (n < N && k < K) out[(int64_t)n * K + k] = acc[i][j][r];
      }
    }
}

// dW = sum of the S partial slabs, deterministic two-level order: group g of G sums slabs
// [g*S/G, (g+1)*S/G) with 4 independent accumulators (a serial S-long chain per element was
// latency-bound: ~0.4 ms at S = 2048), then G group sums are added in order.
__global__ __launch_bounds__(kBlock) void k_wgrad_reduce1(const float* __restrict__ part, int S, int G, int64_t NK4,
                                                          float* __restrict__ tmp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (i >= NK4) return;
  const int s0 = (int)((int64_t)g * S / G), s1 = (int)((int64_t)(g + 1) * S / G);
  const float4* p = reinterpret_cast<const float4*>(part);
  float4 a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  int s = s0;
  for (; s + 3 < s1; s += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float4 b = p[(int64_t)(s + u) * NK4 + i];
      a[u].x += b.x; a[u].y += b.y; a[u].z += b.z; a[u].w += b.w;
    }
  }
  for (; s < s1; ++s) {
    const float4 b = p[(int64_t)s * NK4 + i];
    a[0].x += b.x; a[0].y += b.y; a[0].z += b.z; a[0].w += b.w;
  }
  float4 r;
  r.x = (a[0].x + a[1].x) + (a[2].x + a[3].x);
  r.y = (a[0].y + a[1].y) + (a[2].y + a[3].y);
  r.z = (a[0].z + a[1].z) + (a[2].z + a[3].z);
  r.w = (a[0].w + a[1].w) + (a[2].w + a[3].w);
  reinterpret_cast<float4*>(tmp)[(int64_t)g * NK4 + i] = r;
}

__global__ __launch_bounds__(kBlock) void k_wgrad_reduce2(const float* __restrict__ tmp, int G, int64_t NK4,
                                                          float* __restrict__ dw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NK4) return;
  const float4* p = reinterpret_cast<const float4*>(tmp);
  float4 a = p[i];
  for (int g = 1; g < G; ++g) {
    const float4 b = p[(int64_t)g * NK4 + i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  reinterpret_cast<float4*>(dw)[i] = a;
}

// ------------------------------------------------------------------------------------------
// Weight gradient v2 (channel counts multiples of 64, every ResNet 1x1 conv): the output tile
// is TN x TK with TN, TK in {64, 128} picked per shape, so Cin = 64 / Cout = 64 layers do no
// MFMA work on zero padding (v1 always used 128 x 128: 4x the work on the largest-M layer).
// The M split S targets ~2 blocks per CU while keeping the fp32 partial slabs (S * N * K * 4 B,
// written once, read once) small next to the operand bytes; v1's fixed ~2048 blocks wrote more
// partial bytes than it read operands on the deep layers (1024x512: 134 MB of slabs).
// n / d for 0 <= n < 2^31 with a host-precomputed multiplier (round-up method): the per-row
// pixel decomposition of the implicit-GEMM loaders was two runtime integer divisions per 16-byte
// load -- enough VALU work to make the 3x3 weight gradient slower than MIOpen's.
struct FastDiv {
  uint32_t d, mul, shift;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t mul = ((((1ull << l) - d) << 32) / d) + 1;
  return FastDiv{d, (uint32_t)mul, l};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.mul) + n) >> f.shift;
}

template <int TW>
__device__ __forceinline__ int wt_off(int row, int ch) {  // byte offset in a [rows][TW x bf16] tile
  if (TW == 128) return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  return 128 * row + 16 * (ch ^ (((row & 3) << 1) | ((row >> 2) & 1)));
}

template <int TW>
__device__ __forceinline__ bf16x8 tr_frag_w(const uint8_t* tile, int row0, int col0, int lane) {
  const int il = lane & 15, q = il >> 2, p = il & 3;
  const int r = row0 + 8 * (lane >> 4) + q;
  const int ch = (col0 >> 3) + (p >> 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + wt_off<TW>(r, ch) + 8 * (p & 1)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + wt_off<TW>(r + 4, ch) + 8 * (p & 1)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// KxK convolutions (implicit GEMM over K = KH*KW*Cin, k = (r*KW + s)*Cin + c: the physical
// order of a channels-last [Cout, Cin, KH, KW] weight): a K tile never straddles two taps
// (Cin % TK == 0), so each block has ONE tap (r, s) and its X loader reads the input pixel
// (ho*stride - pad + r, wo*stride - pad + s) of each output row m, zeros outside the image.
template <int TN, int TK, bool PRO = false>
__global__ __launch_bounds__(256) void k_conv1x1_wgrad2(const uint16_t* __restrict__ dY, const uint16_t* __restrict__ X,
                                                        float* __restrict__ part, int M, int N, int K, int Ho, int Wo,
                                                        int Hi, int Wi, int stride, int chunk, int tn, int tk, int Cin,
                                                        int KW, int pad, FastDiv fd_hw, FastDiv fd_w,
                                                        const float* __restrict__ psc, const float* __restrict__ psh) {
  constexpr int YCH = TN / 8, XCH = TK / 8;        // 16-byte chunks per staged row
  constexpr int YP = 64 * YCH / 256, XP = 64 * XCH / 256;  // chunks per thread per stage
  constexpr int YT = kWMS * TN * 2, XT = kWMS * TK * 2;  // bytes per staged tile
  constexpr int FN = TN / 32, FK = TK / 32;        // 16-wide fragments per wave (2x2 waves)
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * (YT + XT)];
  int bid = blockIdx.x;
  const int nblk = gridDim.x;
  if ((nblk & 7) == 0) bid = (bid & 7) * (nblk >> 3) + (bid >> 3);  // a split's tiles share an XCD
  const int tiles = tn * tk;
  const int sidx = bid / tiles, tile = bid - sidx * tiles;
  const int n0 = (tile / tk) * TN, k0 = (tile % tk) * TK;
  const int mbeg = sidx * chunk, mend = min(M, mbeg + chunk);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wn = w >> 1, wk = w & 1;
  const int ych = t % YCH, xch = t % XCH;  // this thread's fixed 16-byte column chunk

  const int tap = k0 / Cin, c0 = k0 - tap * Cin;
  const int kr = tap / KW, kc = tap - (tap / KW) * KW;
  float psr[PRO ? 8 : 1], phr[PRO ? 8 : 1];  // prologue (X = a BN input): this thread's 8 channels
  if (PRO) {
#pragma unroll
    for (int j = 0; j < (PRO ? 8 : 1); ++j) {
      psr[j] = psc[c0 + xch * 8 + j];
      phr[j] = psh[c0 + xch * 8 + j];
    }
  }
  const bool direct = KW == 1 && pad == 0 && stride == 1 && Cin == K;  // plain 1x1: row m is pixel m
  u32x4 ry[YP], rx[XP];
  // element offset of (input pixel of output row m under this block's tap, channel c0); -1 = padding
  auto src_off = [=](int m) -> int64_t {
    if (direct) return (int64_t)m * Cin + c0;
    const int img = (int)fdiv((uint32_t)m, fd_hw), rem = m - img * (int)fd_hw.d;
    const int ho = (int)fdiv((uint32_t)rem, fd_w), wo = rem - ho * Wo;
    const int hi = ho * stride - pad + kr, wi = wo * stride - pad + kc;
    if (hi < 0 || hi >= Hi || wi < 0 || wi >= Wi) return -1;
    return (((int64_t)img * Hi + hi) * Wi + wi) * Cin + c0;
  };
#define HIPPS_W2LOAD(mb_)                                                                          \
  {                                                                                                \
    _Pragma("unroll") for (int i = 0; i < YP; ++i) {                                               \
      const int m_ = (mb_) + t / YCH + (256 / YCH) * i;                                            \
      const u32x4 v_ = *reinterpret_cast<const u32x4*>(dY + (int64_t)(m_ < mend ? m_ : mbeg) * N + \
                                                       n0 + ych * 8);                              \
      ry[i] = m_ < mend ? v_ : u32x4{0u, 0u, 0u, 0u};                                              \
    }                                                                                              \
    _Pragma("unroll") for (int i = 0; i < XP; ++i) {                                               \
      const int m_ = (mb_) + t / XCH + (256 / XCH) * i;                                            \
      const int64_t so_ = m_ < mend ? src_off(m_) : -1;                                            \
      u32x4 v_ = *reinterpret_cast<const u32x4*>(X + (so_ < 0 ? 0 : so_) + xch * 8);               \
      if constexpr (PRO) v_ = bn_relu8(v_, psr, phr);                                              \
      rx[i] = so_ >= 0 ? v_ : u32x4{0u, 0u, 0u, 0u};                                               \
    }                                                                                              \
  }
#define HIPPS_W2STORE(s_)                                                                          \
  {                                                                                                \
    uint8_t* ty_ = lds + (s_) * (YT + XT);                                                         \
    uint8_t* tx_ = ty_ + YT;                                                                       \
    _Pragma("unroll") for (int i = 0; i < YP; ++i)                                                 \
        *reinterpret_cast<u32x4*>(ty_ + wt_off<TN>(t / YCH + (256 / YCH) * i, ych)) = ry[i];       \
    _Pragma("unroll") for (int i = 0; i < XP; ++i)                                                 \
        *reinterpret_cast<u32x4*>(tx_ + wt_off<TK>(t / XCH + (256 / XCH) * i, xch)) = rx[i];       \
  }

  f32x4 acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nst = (mend - mbeg + kWMS - 1) / kWMS;
  HIPPS_W2LOAD(mbeg);
  HIPPS_W2STORE(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) HIPPS_W2LOAD(mbeg + (st + 1) * kWMS);
    const uint8_t* ty = lds + cur * (YT + XT);
    const uint8_t* tx = ty + YT;
#pragma unroll
    for (int ks = 0; ks < kWMS / 32; ++ks) {
      bf16x8 a[FN], b[FK];
#pragma unroll
      for (int i = 0; i < FN; ++i) a[i] = tr_frag_w<TN>(ty, ks * 32, wn * (TN / 2) + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FK; ++j) b[j] = tr_frag_w<TK>(tx, ks * 32, wk * (TK / 2) + j * 16, lane);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nst) HIPPS_W2STORE(cur ^ 1);
    __syncthreads();
  }
#undef HIPPS_W2LOAD
#undef HIPPS_W2STORE
  // D map: column (k) = lane & 15, row (n) = (lane >> 4) * 4 + r
  float* out = part + (int64_t)sidx * N * K;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) {
      const int k = k0 + wk * (TK / 2) + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * (TN / 2) + i * 16 + (lane >> 4) * 4 + r;
        out[(int64_t)n * K + k] = acc[i][j][r];
      }
    }
}

// ==========================================================================================
int64_t conv1x1_mtiles(int64_t M) { return (M + kGBM - 1) / kGBM; }

// x: [img, Cin, Hi, Wi] channels-last bf16; w: [Cout, Cin(,1,1)] bf16 contiguous;
// y: [img, Cout, Ho, Wo] channels-last bf16.  part (optional): f32 [2, Cout, mtiles].
// add (optional): bf16 shaped like y, added in the epilogue (y = conv(x) + add); add_mask
// (optional, with add): uint8 [numel/8] ReLU bits, y = conv(x) + add * bit.
// bn_x (optional, dgrad only): y is the complete gradient of a BatchNorm output whose input was
// bn_x -- the epilogue then writes that BN backward's reduction partials into part (see BnBwdTap;
// bn_bits = its ReLU bits, or none to recompute the mask from bn_x with bn_scale / bn_shift).
// pro_scale / pro_shift (optional, forward with statistics): x is a BatchNorm INPUT, the conv
// reads relu(x * scale + shift) per input channel (bn_relu8) -- the BN apply pass is skipped.
void conv1x1_forward(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part, int64_t Hi,
                     int64_t Wi, int64_t stride, c10::optional<at::Tensor> add, c10::optional<at::Tensor> add_mask,
                     c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_bits,
                     c10::optional<at::Tensor> bn_mean, c10::optional<at::Tensor> bn_invstd,
                     c10::optional<at::Tensor> bn_scale, c10::optional<at::Tensor> bn_shift,
                     c10::optional<at::Tensor> pro_scale, c10::optional<at::Tensor> pro_shift) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && y.is_cuda(), "conv1x1: device tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  y.scalar_type() == at::kBFloat16, "conv1x1: bf16 tensors");
  const int64_t N = w.size(0), K = w.numel() / N;
  TORCH_CHECK(w.is_contiguous(), "conv1x1: weight must be contiguous [Cout, Cin]");
  TORCH_CHECK(K % kGBK == 0 && N % 64 == 0, "conv1x1: needs Cin % 64 == 0 and Cout % 64 == 0");
  const int64_t imgs = x.numel() / (K * Hi * Wi);
  TORCH_CHECK(imgs * K * Hi * Wi == x.numel(), "conv1x1: x size");
  const int64_t Ho = (Hi - 1) / stride + 1, Wo = (Wi - 1) / stride + 1;
  const int64_t M = imgs * Ho * Wo;
  TORCH_CHECK(y.numel() == M * N, "conv1x1: y size");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) || x.dim() != 4, "conv1x1: x must be channels-last");
  TORCH_CHECK(y.is_contiguous(at::MemoryFormat::ChannelsLast) || y.dim() != 4, "conv1x1: y must be channels-last");
  for (const at::Tensor* t : {&x, &w, &y})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "conv1x1: 16-byte aligned tensors");
  TORCH_CHECK(M < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 40), "conv1x1: size");
  const int64_t mtiles = conv1x1_mtiles(M);
  const bool bn128 = N % 128 == 0;
  const int64_t ntiles = N / (bn128 ? 128 : 64);
  const int64_t nblk = mtiles * ntiles;
  TORCH_CHECK(nblk < (int64_t(1) << 31), "conv1x1: grid");
  float *pa = nullptr, *pb = nullptr;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() == 2 * N * mtiles, "conv1x1: part must be f32 [2, Cout, mtiles]");
    pa = part->data_ptr<float>();
    pb = pa + N * mtiles;
  }
  const uint16_t* rp = nullptr;
  if (add.has_value() && add->defined()) {
    TORCH_CHECK(add->is_cuda() && add->scalar_type() == at::kBFloat16 && add->numel() == M * N &&
                    (add->is_contiguous(at::MemoryFormat::ChannelsLast) || add->dim() != 4) &&
                    reinterpret_cast<uintptr_t>(add->data_ptr()) % 16 == 0,
                "conv1x1: add must be a 16-byte aligned channels-last bf16 tensor shaped like y");
    rp = (const uint16_t*)add->data_ptr();
  }
  const uint8_t* mp = nullptr;
  if (add_mask.has_value() && add_mask->defined()) {
    TORCH_CHECK(rp != nullptr, "conv1x1: add_mask needs add");
    TORCH_CHECK(add_mask->is_cuda() && add_mask->scalar_type() == at::kByte && add_mask->is_contiguous() &&
                    add_mask->numel() == M * N / 8, "conv1x1: add_mask must be uint8[numel(y)/8]");
    mp = (const uint8_t*)add_mask->data_ptr();
  }
  BnBwdTap bt{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  const bool bst = bn_x.has_value() && bn_x->defined();
  if (bst) {
    TORCH_CHECK(pa != nullptr, "conv1x1: BN-backward statistics need part");
    TORCH_CHECK(bn_x->is_cuda() && bn_x->scalar_type() == at::kBFloat16 && bn_x->numel() == M * N &&
                    (bn_x->is_contiguous(at::MemoryFormat::ChannelsLast) || bn_x->dim() != 4) &&
                    reinterpret_cast<uintptr_t>(bn_x->data_ptr()) % 16 == 0,
                "conv1x1: bn_x must be a 16-byte aligned channels-last bf16 tensor shaped like y");
    for (const c10::optional<at::Tensor>* v : {&bn_mean, &bn_invstd, &bn_scale, &bn_shift})
      TORCH_CHECK(v->has_value() && (*v)->defined() && (*v)->is_cuda() && (*v)->scalar_type() == at::kFloat &&
                      (*v)->is_contiguous() && (*v)->numel() == N, "conv1x1: BN vectors must be f32 [C]");
    bt.x = (const uint16_t*)bn_x->data_ptr();
    bt.mean = bn_mean->data_ptr<float>();
    bt.invstd = bn_invstd->data_ptr<float>();
    bt.scale = bn_scale->data_ptr<float>();
    bt.shift = bn_shift->data_ptr<float>();
    if (bn_bits.has_value() && bn_bits->defined()) {
      TORCH_CHECK(bn_bits->is_cuda() && bn_bits->scalar_type() == at::kByte && bn_bits->is_contiguous() &&
                      bn_bits->numel() == M * N / 8, "conv1x1: bn_bits must be uint8[numel(y)/8]");
      bt.bits = (const uint8_t*)bn_bits->data_ptr();
    }
  }
  auto stream = c10::hip::getCurrentHIPStream();
  const uint16_t* xp = (const uint16_t*)x.data_ptr();
  const uint16_t* wp = (const uint16_t*)w.data_ptr();
  uint16_t* yp = (uint16_t*)y.data_ptr();
#define HIPPS_C1(BNv, ST, AD, BS)                                                                           \
  hipLaunchKernelGGL((k_conv1x1_nt<BNv, ST, AD, BS>), (int)nblk, 256, 0, stream, xp, wp, yp, pa, pb, rp, mp,     \
                     (int)M, (int)N, (int)K, (int)Ho, (int)Wo, (int)Hi, (int)Wi, (int)stride, (int)mtiles,        \
                     (int)ntiles, bt, (const float*)nullptr, (const float*)nullptr, ConvGeom{1, 0, (int)K})
#define HIPPS_C1_BN(BNv)                                                                                      \
  do {                                                                                                        \
    if (bst && bt.bits) {                                                                                     \
      if (rp) HIPPS_C1(BNv, false, true, 2); else HIPPS_C1(BNv, false, false, 2);                             \
    } else if (bst) {                                                                                         \
      if (rp) HIPPS_C1(BNv, false, true, 1); else HIPPS_C1(BNv, false, false, 1);                             \
    } else if (pa) {                                                                                          \
      HIPPS_C1(BNv, true, false, 0);                                                                          \
    } else if (rp) {                                                                                          \
      HIPPS_C1(BNv, false, true, 0);                                                                          \
    } else {                                                                                                  \
      HIPPS_C1(BNv, false, false, 0);                                                                         \
    }                                                                                                         \
  } while (0)
  TORCH_CHECK(bst || !(pa && rp), "conv1x1: the forward statistics epilogue and the add epilogue are exclusive");
  const bool pro = pro_scale.has_value() && pro_scale->defined();
  if (pro) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined(), "conv1x1: prologue needs scale and shift");
    for (const c10::optional<at::Tensor>* v : {&pro_scale, &pro_shift})
      TORCH_CHECK((*v)->is_cuda() && (*v)->scalar_type() == at::kFloat && (*v)->is_contiguous() && (*v)->numel() == K,
                  "conv1x1: prologue vectors must be f32 [Cin]");
    TORCH_CHECK(pa && !rp && !bst, "conv1x1: the BN-apply prologue runs with the statistics epilogue only");
    const float* ps = pro_scale->data_ptr<float>();
    const float* ph = pro_shift->data_ptr<float>();
#define HIPPS_C1P(BNv)                                                                                        \
  hipLaunchKernelGGL((k_conv1x1_nt<BNv, true, false, 0, true>), (int)nblk, 256, 0, stream, xp, wp, yp, pa, pb,  \
                     rp, mp, (int)M, (int)N, (int)K, (int)Ho, (int)Wo, (int)Hi, (int)Wi, (int)stride,             \
                     (int)mtiles, (int)ntiles, bt, ps, ph, ConvGeom{1, 0, (int)K})
    if (bn128) HIPPS_C1P(128); else HIPPS_C1P(64);
#undef HIPPS_C1P
    return;
  }
  if (bn128) HIPPS_C1_BN(128); else HIPPS_C1_BN(64);
#undef HIPPS_C1_BN
#undef HIPPS_C1
}


// KxK convolution forward (stride, symmetric zero padding) as the implicit-GEMM variant of the
// 1x1 MFMA kernel: x [img, Cin, Hi, Wi], w [Cout, Cin, KH, KW], y [img, Cout, Ho, Wo], all
// channels-last bf16; Cin % 64 == 0, Cout % 64 == 0.  part (optional): the following BatchNorm's
// per-channel partial statistics f32 [2, Cout, mtiles] from the epilogue.
void convkxk_forward(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part, int64_t stride,
                     int64_t pad) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && y.is_cuda(), "convkxk: device tensors");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  y.scalar_type() == at::kBFloat16, "convkxk: bf16 tensors");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && y.dim() == 4, "convkxk: 4-d tensors");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && w.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  y.is_contiguous(at::MemoryFormat::ChannelsLast), "convkxk: channels-last x, w, y");
  const int64_t imgs = x.size(0), Cin = x.size(1), Hi = x.size(2), Wi = x.size(3);
  const int64_t N = w.size(0), KH = w.size(2), KW = w.size(3);
  TORCH_CHECK(w.size(1) == Cin, "convkxk: weight Cin");
  TORCH_CHECK(Cin % kGBK == 0 && N % 64 == 0, "convkxk: needs Cin % 64 == 0 and Cout % 64 == 0");
  TORCH_CHECK(stride >= 1 && pad >= 0, "convkxk: geometry");
  const int64_t Ho = (Hi + 2 * pad - KH) / stride + 1, Wo = (Wi + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(y.size(0) == imgs && y.size(1) == N && y.size(2) == Ho && y.size(3) == Wo, "convkxk: y shape");
  for (const at::Tensor* t : {&x, &w, &y})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "convkxk: 16-byte aligned tensors");
  const int64_t M = imgs * Ho * Wo, K = KH * KW * Cin;
  TORCH_CHECK(M < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 40), "convkxk: size");
  const int64_t mtiles = conv1x1_mtiles(M);
  const bool bn128 = N % 128 == 0;
  const int64_t ntiles = N / (bn128 ? 128 : 64);
  const int64_t nblk = mtiles * ntiles;
  float *pa = nullptr, *pb = nullptr;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() == 2 * N * mtiles, "convkxk: part must be f32 [2, Cout, mtiles]");
    pa = part->data_ptr<float>();
    pb = pa + N * mtiles;
  }
  auto stream = c10::hip::getCurrentHIPStream();
  const uint16_t* xp = (const uint16_t*)x.data_ptr();
  const uint16_t* wp = (const uint16_t*)w.data_ptr();
  uint16_t* yp = (uint16_t*)y.data_ptr();
  const ConvGeom cg{(int)KW, (int)pad, (int)Cin};
  BnBwdTap bt{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
#define HIPPS_CK(BNv, ST)                                                                                        \
  hipLaunchKernelGGL((k_conv1x1_nt<BNv, ST, false, 0, false, true>), (int)nblk, 256, 0, stream, xp, wp, yp, pa, pb, \
                     (const uint16_t*)nullptr, (const uint8_t*)nullptr, (int)M, (int)N, (int)K, (int)Ho, (int)Wo,     \
                     (int)Hi, (int)Wi, (int)stride, (int)mtiles, (int)ntiles, bt, (const float*)nullptr,            \
                     (const float*)nullptr, cg)
  if (bn128) {
    if (pa) HIPPS_CK(128, true); else HIPPS_CK(128, false);
  } else {
    if (pa) HIPPS_CK(64, true); else HIPPS_CK(64, false);
  }
#undef HIPPS_CK
}

void wgrad_reduce_slabs(const at::Tensor& part, int64_t S, int64_t N, int64_t K, at::Tensor& dw,
                        hipStream_t stream0);

// v2 weight gradient launcher: dW[N][K] (K = KH*KW*Cin) as S split-M partial slabs + fixed-order sum.
static void launch_wgrad2(const at::Tensor& dy, const at::Tensor& x, at::Tensor& dw, int64_t M, int64_t N, int64_t K,
                          int64_t Cin, int64_t Ho, int64_t Wo, int64_t Hi, int64_t Wi, int64_t stride, int64_t KW,
                          int64_t pad, hipStream_t stream0, const float* psc = nullptr, const float* psh = nullptr) {
  const int TN = N % 128 == 0 ? 128 : 64, TK = Cin % 128 == 0 ? 128 : 64;  // a K tile stays in one tap
  const int64_t tn = N / TN, tk = K / TK, tiles = tn * tk;
  // one wave of resident blocks: 256 CUs x (2 | 3 | 5) blocks per CU at (186 | 124 | 92) VGPRs
  const int64_t resident = 256 * (TN * TK == 128 * 128 ? 2 : TN * TK == 128 * 64 ? 3 : 5);
  int64_t S = std::max<int64_t>(1, resident / tiles);
  S = std::min<int64_t>(S, std::max<int64_t>(1, M / (8 * kWMS)));           // >= 8 stages per block
  S = std::min<int64_t>(S, std::max<int64_t>(1, M * (N + K) / (4 * N * K)));  // slabs <= operand bytes
  const int64_t chunk = ((M + S - 1) / S + kWMS - 1) / kWMS * kWMS;
  S = (M + chunk - 1) / chunk;
  TORCH_CHECK(S * tiles < (int64_t(1) << 31), "conv wgrad: grid");
  at::Tensor part = S == 1 ? dw : at::empty({S, N, K}, dw.options());
  const FastDiv fd_hw = make_fastdiv((uint32_t)(Ho * Wo)), fd_w = make_fastdiv((uint32_t)Wo);
  const uint16_t* dyp = (const uint16_t*)dy.data_ptr();
  const uint16_t* xp = (const uint16_t*)x.data_ptr();
#define HIPPS_W2(TNv, TKv)                                                                                    \
  do {                                                                                                        \
    if (psc)                                                                                                  \
      hipLaunchKernelGGL((k_conv1x1_wgrad2<TNv, TKv, true>), (int)(S * tiles), 256, 0, stream0, dyp, xp,     \
                         part.data_ptr<float>(), (int)M, (int)N, (int)K, (int)Ho, (int)Wo, (int)Hi, (int)Wi,  \
                         (int)stride, (int)chunk, (int)tn, (int)tk, (int)Cin, (int)KW, (int)pad, fd_hw, fd_w, \
                         psc, psh);                                                                           \
    else                                                                                                      \
      hipLaunchKernelGGL((k_conv1x1_wgrad2<TNv, TKv>), (int)(S * tiles), 256, 0, stream0, dyp, xp,           \
                         part.data_ptr<float>(), (int)M, (int)N, (int)K, (int)Ho, (int)Wo, (int)Hi, (int)Wi,  \
                         (int)stride, (int)chunk, (int)tn, (int)tk, (int)Cin, (int)KW, (int)pad, fd_hw, fd_w, \
                         (const float*)nullptr, (const float*)nullptr);                                       \
  } while (0)
  if (TN == 128 && TK == 128) HIPPS_W2(128, 128);
  else if (TN == 128) HIPPS_W2(128, 64);
  else if (TK == 128) HIPPS_W2(64, 128);
  else HIPPS_W2(64, 64);
#undef HIPPS_W2
  if (S > 1) wgrad_reduce_slabs(part, S, N, K, dw, stream0);
}

// dw[N][K] = sum_s part[s][N][K] in a fixed order (deterministic); shared with gemm2.hip's
// weight-gradient core.  Split over G groups when N*K alone is too few threads to keep the
// loads in flight (64x64 outputs: 1024 float4 lanes x S serial loads was ~60 us).
int64_t wgrad_reduce_groups(int64_t S, int64_t N, int64_t K) {
  const int64_t NK4 = N * K / 4;
  return std::min<int64_t>(S, std::max<int64_t>(1, (65536 + NK4 - 1) / NK4));
}

void wgrad_reduce_slabs(const at::Tensor& part, int64_t S, int64_t N, int64_t K, at::Tensor& dw,
                        hipStream_t stream0) {
  const int64_t NK4 = N * K / 4;
  const int G = (int)wgrad_reduce_groups(S, N, K);
  const unsigned gx = (unsigned)((NK4 + kBlock - 1) / kBlock);
  if (G == 1) {
    hipLaunchKernelGGL(k_wgrad_reduce1, dim3(gx, 1), kBlock, 0, stream0, part.data_ptr<float>(), (int)S, 1, NK4,
                       dw.data_ptr<float>());
  } else {
    auto tmp = at::empty({(int64_t)G, N, K}, dw.options());
    hipLaunchKernelGGL(k_wgrad_reduce1, dim3(gx, G), kBlock, 0, stream0, part.data_ptr<float>(), (int)S, G, NK4,
                       tmp.data_ptr<float>());
    hipLaunchKernelGGL(k_wgrad_reduce2, gx, kBlock, 0, stream0, tmp.data_ptr<float>(), G, NK4, dw.data_ptr<float>());
  }
}

// dy: [img, Cout, Ho, Wo] channels-last bf16; x: [img, Cin, Hi, Wi] channels-last bf16;
// dw: f32 [Cout, Cin] (written, not accumulated).
// pro_scale / pro_shift (optional): x is a BatchNorm input; the GEMM reads relu(x * scale + shift).
void conv1x1_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw, int64_t Hi, int64_t Wi, int64_t stride,
                   c10::optional<at::Tensor> pro_scale, c10::optional<at::Tensor> pro_shift) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dw.is_cuda(), "conv1x1_wgrad: device tensors");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 && dw.scalar_type() == at::kFloat,
              "conv1x1_wgrad: bf16 dy/x, f32 dw");
  TORCH_CHECK(dw.is_contiguous(), "conv1x1_wgrad: dw contiguous [Cout, Cin]");
  const int64_t N = dw.size(0), K = dw.numel() / N;
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0, "conv1x1_wgrad: channels % 8");
  const int64_t imgs = x.numel() / (K * Hi * Wi);
  TORCH_CHECK(imgs * K * Hi * Wi == x.numel(), "conv1x1_wgrad: x size");
  const int64_t Ho = (Hi - 1) / stride + 1, Wo = (Wi - 1) / stride + 1;
  const int64_t M = imgs * Ho * Wo;
  TORCH_CHECK(dy.numel() == M * N, "conv1x1_wgrad: dy size");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) || x.dim() != 4, "conv1x1_wgrad: x channels-last");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) || dy.dim() != 4, "conv1x1_wgrad: dy channels-last");
  for (const at::Tensor* t : {&x, &dy, &dw})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "conv1x1_wgrad: 16-byte aligned tensors");
  TORCH_CHECK(M < (int64_t(1) << 31), "conv1x1_wgrad: size");
  auto stream0 = c10::hip::getCurrentHIPStream();
  const float *psc = nullptr, *psh = nullptr;
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(pro_shift.has_value() && pro_shift->defined(), "conv1x1_wgrad: prologue needs scale and shift");
    for (const c10::optional<at::Tensor>* v : {&pro_scale, &pro_shift})
      TORCH_CHECK((*v)->is_cuda() && (*v)->scalar_type() == at::kFloat && (*v)->is_contiguous() && (*v)->numel() == K,
                  "conv1x1_wgrad: prologue vectors must be f32 [Cin]");
    TORCH_CHECK(N % 64 == 0 && K % 64 == 0, "conv1x1_wgrad: the prologue needs Cin, Cout % 64 == 0");
    psc = pro_scale->data_ptr<float>();
    psh = pro_shift->data_ptr<float>();
  }
  if (N % 64 == 0 && K % 64 == 0) {  // v2: shape-fitted tiles, bounded split
    launch_wgrad2(dy, x, dw, M, N, K, K, Ho, Wo, Hi, Wi, stride, 1, 0, stream0, psc, psh);
    return;
  }
  const int64_t tn = (N + kWT - 1) / kWT, tk = (K + kWT - 1) / kWT, tiles = tn * tk;
  int64_t S = std::max<int64_t>(1, std::min<int64_t>(2048 / tiles, (M + kWMS - 1) / kWMS));
  int64_t chunk = ((M + S - 1) / S + kWMS - 1) / kWMS * kWMS;
  S = (M + chunk - 1) / chunk;
  auto part = at::empty({S, N, K}, dw.options());
  auto stream = c10::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(k_conv1x1_wgrad, (int)(S * tiles), 256, 0, stream, (const uint16_t*)dy.data_ptr(),
                     (const uint16_t*)x.data_ptr(), part.data_ptr<float>(), (int)M, (int)N, (int)K, (int)Ho, (int)Wo,
                     (int)Hi, (int)Wi, (int)stride, (int)chunk, (int)tn, (int)tk);
  const int64_t NK4 = N * K / 4;
  const int G = (int)std::min<int64_t>(S, 32);
  const int gx = (int)((NK4 + kBlock - 1) / kBlock);
  if (G == 1) {
    hipLaunchKernelGGL(k_wgrad_reduce2, gx, kBlock, 0, stream, part.data_ptr<float>(), (int)S, NK4,
                       dw.data_ptr<float>());
  } else {
    auto tmp = at::empty({G, N, K}, dw.options());
    hipLaunchKernelGGL(k_wgrad_reduce1, dim3(gx, G), kBlock, 0, stream, part.data_ptr<float>(), (int)S, G, NK4,
                       tmp.data_ptr<float>());
    hipLaunchKernelGGL(k_wgrad_reduce2, gx, kBlock, 0, stream, tmp.data_ptr<float>(), G, NK4, dw.data_ptr<float>());
  }
}

// KxK convolution weight gradient (stride, symmetric zero padding), channels-last bf16 dy/x;
// dw: f32 with the weight's channels-last layout, i.e. [Cout][KH][KW][Cin] in memory.
void conv_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw, int64_t KH, int64_t KW, int64_t stride, int64_t pad) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dw.is_cuda(), "conv_wgrad: device tensors");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 && dw.scalar_type() == at::kFloat,
              "conv_wgrad: bf16 dy/x, f32 dw");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4 && dw.dim() == 4, "conv_wgrad: 4-d tensors");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dw.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_wgrad: channels-last dy, x, dw");
  const int64_t imgs = x.size(0), Cin = x.size(1), Hi = x.size(2), Wi = x.size(3);
  const int64_t N = dw.size(0);
  TORCH_CHECK(dw.size(1) == Cin && dw.size(2) == KH && dw.size(3) == KW, "conv_wgrad: dw shape [Cout, Cin, KH, KW]");
  TORCH_CHECK(stride >= 1 && pad >= 0 && KH >= 1 && KW >= 1, "conv_wgrad: geometry");
  const int64_t Ho = (Hi + 2 * pad - KH) / stride + 1, Wo = (Wi + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(dy.size(0) == imgs && dy.size(1) == N && dy.size(2) == Ho && dy.size(3) == Wo, "conv_wgrad: dy shape");
  TORCH_CHECK(N % 64 == 0 && Cin % 64 == 0, "conv_wgrad: needs Cout % 64 == 0 and Cin % 64 == 0");
  for (const at::Tensor* t : {&x, &dy, &dw})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "conv_wgrad: 16-byte aligned tensors");
  const int64_t M = imgs * Ho * Wo;
  TORCH_CHECK(M < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 40), "conv_wgrad: size");
  launch_wgrad2(dy, x, dw, M, N, KH * KW * Cin, Cin, Ho, Wo, Hi, Wi, stride, KW, pad,
                c10::hip::getCurrentHIPStream());
}

}  // namespace hipps
