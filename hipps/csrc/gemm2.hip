// hipps — second-generation MFMA GEMM core for channels-last convolutions (gfx950).
//
//   Y[M, N] = X[M, K] · W[N, K]^T       1x1 conv: M = images*Ho*Wo, K = Cin, N = Cout
//                                       KxK conv: implicit GEMM, K = KH*KW*Cin (k = tap*Cin + c)
//
// What changes against the first core (gemm.hip k_conv1x1_nt, register-staged 128x128 tiles of
// 64x64-per-wave, 4 waves):
//   * staging by LDS DMA: every 16-byte chunk goes global -> LDS with global_load_lds_dwordx4,
//     no VGPR round trip and no ds_write pass (cdna_hip_programming.md §5 'Async global->LDS
//     copy'); the XOR swizzle (LDS slot = chunk ^ (row & 7)) is applied on the per-lane GLOBAL
//     address, so each wave-instruction's 1 KB LDS image stays lane-linear;
//   * rows outside M and zero-padding taps fetch a 16-byte zero page instead of branching;
//   * larger per-wave tiles (128x64 of 16x16x32 accumulators: 12 fragment reads per 32 MFMAs
//     instead of 8 per 16) -- the 64x64 core was LDS-read bound at the MFMA rate
//     (profiles/ab_r2/gemm_pf2_probe.json);
//   * block tiles 256x256 (8 waves), 256x128 / 128x128 (4 waves), picked per shape by the host
//     so the grid covers the 256 CUs; a bijective XCD-aware block order keeps the N tiles of one
//     M tile on one XCD (A rows re-read from that XCD's L2);
//   * one raw s_barrier per K-tile: the DMA of tile k+1 is issued right after it and lands
//     during the MFMAs of tile k; s_setprio(1) around the MFMA cluster.
// The epilogue (bf16 tile staged through LDS for 16-byte row stores, optional per-channel BN
// statistics, optional "+ R * mask" residual-gradient add) matches the first core's semantics.
#include "common.h"

#include <ATen/ATen.h>
#include <cstdlib>
#include <mutex>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {
namespace g2 {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

constexpr int BK = 64;  // k per stage = 8 chunks of 16 bytes per row

// 16-byte zero source for out-of-range rows and zero-padding taps (global memory, read-only)
__device__ __attribute__((aligned(64))) const uint16_t kZero16[32] = {0};
// the residual-mask byte of an unmasked add (kAdd without RM): every bit set
__device__ __attribute__((aligned(64))) const uint8_t kOnes8[64] = {
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
    0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};

// epilogue flags: kStats = forward BN statistics of Y; kAdd = Y += R (* mask bits); kBst =
// backward BN statistics of the BN whose output gradient Y is (relu' recomputed from x * scale +
// shift), kBstBits = the same with the BN's stored ReLU bits (gemm.hip BnBwdTap)
// kAddS2 (with kAdd, 1x1 only): R is the compact input gradient of a stride-2 1x1 conv reading the
// same tensor ([img, ceil(Ho/2), ceil(Wo/2), N]); it lands on the even (h, w) rows of Y only
// kPar (with TAPS): one output-parity class (ph, pw) of a stride-2 KxK input gradient -- the rows
// are the class's dx positions (2a+ph, 2b+pw), A is dy read at (a + tdr[t], b + tdc[t]) for the
// class's taps t, whose weights sit at K offset tko[t] * Cin of B (rot180(W)^T, all taps)
// kPro (2 LDS stages): the A operand is a BatchNorm input x; the GEMM reads relu(x * psc + psh)
// per K channel -- every thread transforms the 16-byte chunks it staged, in LDS, after its own
// DMA landed and before the tile's barrier (rows / taps that read the zero page stay zero), so
// the BN's output is never written (ResNet bn1 -> conv2, bn2 -> conv3)
// kBias (1x1 only; alone or with a plain kAdd): y = x w^T + bias[col] (+ R), the fp32 bias added
// to the fp32 accumulator before the bf16 rounding (a Linear layer's addmm; + R: the residual
// added by the same pass)
// kGelu (1x1, with kBias or alone): the Linear + GELU of a transformer MLP -- Y2 = bf16(acc + bias)
// (the pre-activation the backward needs) and Y = bf16(gelu(Y2)), exact erf form, as F.gelu on
// the bf16 pre-activation rounds it: one pass instead of the GEMM, a GELU read and its write
// kGeluB (1x1): the next Linear's input gradient with the GELU backward in its epilogue: Y =
// bf16(gelu'(x) * bf16(acc)), x the saved bf16 pre-activation (read like kBst's BN input)
// kGeluBS (with kGeluB): also the column sums of the bf16 Y written (the bias gradient of the
// Linear before the GELU), per m-tile into pa[mt][N] (a fixed-order fold sums the tiles)
enum Epi : int { kPlain = 0, kStats = 1, kAdd = 2, kBst = 4, kBstBits = 8, kAddS2 = 16, kPar = 32, kPro = 64,
                 kBias = 128, kGelu = 256, kGeluB = 512, kGeluBS = 1024 };

// Branch-free erf for the epilogues: erf(z) = 1 - poly(t) e^{-z^2}, t = 1 / (1 + p |z|)
// (Abramowitz & Stegun 7.1.26, |error| < 1.5e-7 -- far below the bf16 rounding of the result);
// ocml's erff branches on |z| and the divergent lanes of a 64-wide wave ran both of its paths (the
// GELU epilogue cost 48 us on BERT's 16384 x 3072 pre-activation with it).  e^{-z^2} is returned
// too: GELU's backward reuses it as its density term.
__device__ __forceinline__ float erf_fast(float z, float& ez2) {
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.f));
  ez2 = __expf(-az * az);
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = fmaf(-p * t, ez2, 1.f);
  return copysignf(e, z);
}
__device__ __forceinline__ float gelu_f(float x) {
  float ez2;
  return x * 0.5f * (1.f + erf_fast(x * 0.70710678118654752f, ez2));
}
__device__ __forceinline__ float gelu_bwd_f(float dy, float x) {
  float ez2;  // = e^{-x^2 / 2}
  const float cdf = 0.5f * (1.f + erf_fast(x * 0.70710678118654752f, ez2));
  return dy * fmaf(x, 0.3989422804014327f * ez2, cdf);
}

template <int BM, int BN> struct Cfg;
template <> struct Cfg<256, 256> { static constexpr int TM = 128, TN = 64; };
template <> struct Cfg<256, 128> { static constexpr int TM = 64, TN = 64; };  // 8 waves (3 stages fit: 144 KB)
template <> struct Cfg<128, 128> { static constexpr int TM = 64, TN = 64; };
template <> struct Cfg<256, 64> { static constexpr int TM = 64, TN = 64; };
template <> struct Cfg<128, 64> { static constexpr int TM = 64, TN = 32; };

template <int BM, int BN> constexpr int nthreads() { return 64 * (BM / Cfg<BM, BN>::TM) * (BN / Cfg<BM, BN>::TN); }

template <int BM, int BN, int NS = 2> constexpr int lds_bytes() {
  constexpr int stage = (NS >= 4 ? 2 : NS) * (BM + BN) * BK * 2;
  constexpr int epi = BM * (BN + 8) * 2;
  constexpr int wm = BM / Cfg<BM, BN>::TM;
  return (stage > epi ? stage : epi) + 2 * 2 * wm * BN * 4;
}

struct Args {
  const uint16_t* X;
  const uint16_t* W;
  uint16_t* Y;
  float* pa;
  float* pb;
  const uint16_t* R;
  const uint8_t* RM;
  const uint16_t* bx;  // kBst*: the BN input x under the output tile
  const uint8_t* bbits;
  const float *bmean, *binvstd, *bscale, *bshift;
  int M, N, K, Ho, Wo, Hi, Wi, stride, mtiles, ntiles;
  int KW, pad, Cin;  // implicit-GEMM geometry (TAPS)
  int ldb;           // B row stride (elements; K unless kPar)
  int pstride, pcol0;  // partials: row stride and first column (several launches share one array)
  int ph, pw, Hx, Wx;  // kPar: output parity class and the dx grid
  int tdr[4], tdc[4], tko[4];
  const float *psc, *psh;  // kPro: per-channel scale / shift of the A operand's BN
  const float* bias;       // kBias: f32 [N]
  uint16_t* Y2;            // kGelu: the bf16 pre-activation [M, N]
  int epf;                 // EPF allowed (HIPPS_G2_EPF, default 1)
};

__device__ __forceinline__ uint32_t add_bf16x2(uint32_t a, uint32_t b) {
  return pack_bf16x2(__uint_as_float(a << 16) + __uint_as_float(b << 16),
                     __uint_as_float(a & 0xffff0000u) + __uint_as_float(b & 0xffff0000u));
}

__device__ __forceinline__ void glds16(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)dst, 16, 0, 0);
}

// vmcnt-only s_waitcnt immediate (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at bits 15:14; expcnt and
// lgkmcnt at their maxima, i.e. not waited for)
constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
// lgkmcnt-only s_waitcnt immediate (vmcnt / expcnt at their maxima)
constexpr int waitcnt_lgkm(int n) { return 15 | (3 << 14) | (7 << 4) | ((n & 15) << 8); }

// NS: LDS stages.  2: the DMA of tile k+1 is issued after the barrier of tile k and drained
// (vmcnt(0)) before the next barrier.  3: tile k+2 is issued after the barrier of tile k and the
// wait before each barrier is counted (vmcnt(glds per tile)), so one tile's DMA stays in flight
// across every barrier (cdna_hip_programming.md §5 'Pipelining across barriers').
// 4 (k-halves): the two stages' LDS split into four 32-deep units (rows of 64 bytes); one barrier
// per unit, unit u+3 is issued right after the barrier of unit u into the slot unit u-1 just
// freed, and each wait leaves the two younger units in flight (3 half-tiles of lead instead of 2,
// with no drain before any barrier) -- same LDS bytes as 2 stages.
__host__ __device__ constexpr int khalf_swz(int row) {  // conflict-free ds_read_b128 on 64-byte rows
  return ((0x1320 >> (4 * ((row >> 2) & 3))) & 3);     // [0, 2, 3, 1][(row >> 2) & 3]
}

template <int BM, int BN, int EPI, bool TAPS, int NS>
__global__ __launch_bounds__((nthreads<BM, BN>())) void k_gemm(Args g) {
  constexpr int TM = Cfg<BM, BN>::TM, TN = Cfg<BM, BN>::TN;
  constexpr int WM = BM / TM, WN = BN / TN, NW = WM * WN, NT = 64 * NW;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr bool KH = NS == 4;
  // NS == 5: ping-pong (2 LDS stages, 256x256 on 8 waves).  The two row halves of the tile are two
  // wave groups, one wave of each on every SIMD, one phase apart: while group 0 runs the MFMAs of
  // tile k, group 1 issues the DMA of tile k+2 and waits on its landing, then they swap -- the
  // DMA issue and the drains before each barrier sit beside the partner's MFMAs instead of
  // stalling both waves of the SIMD at the same barrier.  Group 0 stages its own A half (freed
  // as soon as it finished tile k), group 1 the other A half and all of B (freed one phase later).
  constexpr bool PP = NS == 5;
  // NS == 6: the 2-stage loop with v_mfma_f32_32x32x16_bf16 (256x256, 8 waves of 128x64 as 4x2
  // 32x32 accumulators): half the MFMA instructions of the 16x16x32 form for the same work, so
  // three times the issue slack per MFMA (24 of 32 cycles vs 8 of 16) for the DMA, LDS reads and
  // address arithmetic (MI355X_MICROARCH.md cycle constants).  LDS chunk swizzle (row >> 1) & 7:
  // the 16 lanes of a ds_read_b128 group read 16 different rows of one 32-row fragment at the
  // same logical chunk, which row & 7 would pair 2-way on the 128-byte rows.
  constexpr bool M32 = NS == 6;
  constexpr int NSX = M32 ? 2 : NS;  // LDS stages of the generic loop
  constexpr bool PAR = (EPI & kPar) != 0;
  constexpr bool PRO = (EPI & kPro) != 0;
  static_assert(!PAR || TAPS, "kPar needs the implicit-GEMM loader");
  static_assert(!PRO || NS == 2, "kPro: 2 LDS stages");
  static_assert(!PP || (BM == 256 && BN == 256), "ping-pong: 256x256 on 8 waves");
  static_assert(!M32 || (BM == 256 && BN == 256 && !PRO), "32x32x16 MFMA: the 256x256 tile");
  // output row of GEMM row m (kPar: the class's dx position)
  auto orow = [&](int m) -> int64_t {
    if constexpr (PAR) {
      const int hw = g.Ho * g.Wo;
      const int img = m / hw, rem = m - img * hw;
      const int a = rem / g.Wo, b = rem - a * g.Wo;
      return ((int64_t)img * g.Hx + 2 * a + g.ph) * g.Wx + 2 * b + g.pw;
    } else {
      return m;
    }
  };
  constexpr int STAGE = (BM + BN) * BK;   // elements per stage (KH: two 32-deep units)
  constexpr int UNIT = (BM + BN) * 32;    // KH: elements per unit
  constexpr int RPI = KH ? 16 : 8;        // rows per wave-instruction (1 KB)
  constexpr int AI = BM / RPI / NW;       // A wave-instructions per stage (KH: per unit) per wave
  constexpr int BI = BN / RPI / NW;
  constexpr int EP = BN + 8;              // epilogue row pitch (elements)
  constexpr int NSB = (KH || PP || M32) ? 2 : NS;  // stage-sized LDS buffers
  constexpr int SCR = (NSB * STAGE * 2 > BM * EP * 2 ? NSB * STAGE * 2 : BM * EP * 2);  // bytes before the stats scratch
  static_assert(AI >= 1 && BI >= 1, "tile too small for the wave count");
  static_assert(NS >= 2 && NS <= 6, "stages");
  constexpr int NG = AI + BI;  // glds per tile (KH: per unit) per wave
  constexpr int BIP = PP ? 2 * BI : BI;  // PP: group 1 stages all of B (group 0 none)
  __shared__ __attribute__((aligned(16))) uint16_t lds[lds_bytes<BM, BN, NS>() / 2];

  // bijective XCD-aware block order (cdna_hip_programming.md §5 'XCD swizzle must be bijective'):
  // the hardware deals blocks round-robin to 8 XCDs; give each XCD a contiguous run of tiles
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int mt = bid / g.ntiles, nt = bid - mt * g.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w / WN, wn = w - (w / WN) * WN;
  // first row of this wave's i-th A / B wave-instruction (PP: A rows of the wave's own group)
  auto arb = [&](int i) { return PP ? (BM / 2) * wm + RPI * (i * (NW / 2) + wn) : RPI * (i * NW + w); };
  auto brb = [&](int i) { return PP ? RPI * (i * (NW / 2) + wn) : RPI * (i * NW + w); };
  // row in the wave-instruction's row group, logical chunk this lane fetches (the LDS slot is
  // lane-linear; the swizzle is applied on the source)
  const int lr = KH ? lane >> 2 : lane >> 3;
  // (M32: the swizzle (row >> 1) & 7 of row 8m + lr is (lr >> 1) | (m & 1) << 2, and m = i*NW + w
  // has the parity of w for every wave-instruction i of this wave)
  const int lc = KH ? (lane & 3) ^ khalf_swz(lr)
                    : M32 ? (lane & 7) ^ (((lr >> 1) | ((w & 1) << 2)) & 7) : (lane & 7) ^ lr;

  // ---- per-lane sources (fixed over the K loop) ----
  const uint16_t* a_src[AI];  // 1x1: row base + chunk; TAPS: image base
  int a_h[TAPS ? AI : 1], a_w[TAPS ? AI : 1];
  bool a_ok[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = arb(i) + lr;
    int m = m0 + row;
    a_ok[i] = m < g.M;
    m = a_ok[i] ? m : g.M - 1;
    if constexpr (TAPS) {
      const int hw = g.Ho * g.Wo;
      const int img = m / hw, rem = m - img * hw;
      const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
      a_h[i] = PAR ? ho : ho * g.stride - g.pad;
      a_w[i] = PAR ? wo : wo * g.stride - g.pad;
      a_src[i] = g.X + (int64_t)img * g.Hi * g.Wi * g.Cin + lc * 8;
    } else {
      int64_t src = m;
      if (g.stride != 1) {
        const int hw = g.Ho * g.Wo;
        const int img = m / hw, rem = m - img * hw;
        const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
        src = ((int64_t)img * g.Hi + (int64_t)ho * g.stride) * g.Wi + (int64_t)wo * g.stride;
      }
      a_src[i] = g.X + src * g.K + lc * 8;
    }
  }
  // B rows of consecutive wave-instructions are a fixed (wave-uniform) distance apart: one per-lane
  // base pointer, the rest scalar offsets (no per-instruction VGPR pair)
  const uint16_t* b_src0 = g.W + (int64_t)(n0 + brb(0) + lr) * g.ldb + lc * 8;
  auto b_src = [&](int i) { return b_src0 + (int64_t)(brb(i) - brb(0)) * g.ldb; };

  // kPro: which of this thread's A chunks of the staged tile hold data (not the zero page), and
  // the BN scale / shift of its 8 channels -- loaded with the tile's DMA, used at the next barrier
  uint32_t pro_ok = 0;
  float pro_sc[PRO ? 8 : 1], pro_sh[PRO ? 8 : 1];
  // stage kt (KH: unit 2*kt + h, k0 = 64*kt + 32*h, rows of 32 elements) into LDS at ``base``
  auto issue_at = [&](int k0, uint16_t* base, int rowlen, bool do_b = true) {
    int bk = k0;  // B column of this K tile
    if constexpr (PRO) {
      const int ch = (TAPS ? k0 - (k0 / g.Cin) * g.Cin : k0) + lc * 8;
      const float4 s0 = *reinterpret_cast<const float4*>(g.psc + ch);
      const float4 s1 = *reinterpret_cast<const float4*>(g.psc + ch + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(g.psh + ch);
      const float4 h1 = *reinterpret_cast<const float4*>(g.psh + ch + 4);
      pro_sc[PRO ? 0 : 0] = s0.x; pro_sc[PRO ? 1 : 0] = s0.y; pro_sc[PRO ? 2 : 0] = s0.z; pro_sc[PRO ? 3 : 0] = s0.w;
      pro_sc[PRO ? 4 : 0] = s1.x; pro_sc[PRO ? 5 : 0] = s1.y; pro_sc[PRO ? 6 : 0] = s1.z; pro_sc[PRO ? 7 : 0] = s1.w;
      pro_sh[PRO ? 0 : 0] = h0.x; pro_sh[PRO ? 1 : 0] = h0.y; pro_sh[PRO ? 2 : 0] = h0.z; pro_sh[PRO ? 3 : 0] = h0.w;
      pro_sh[PRO ? 4 : 0] = h1.x; pro_sh[PRO ? 5 : 0] = h1.y; pro_sh[PRO ? 6 : 0] = h1.z; pro_sh[PRO ? 7 : 0] = h1.w;
      pro_ok = 0;
    }
    if constexpr (TAPS) {
      const int tap = k0 / g.Cin, c0 = k0 - tap * g.Cin;
      int kr, kc;
      if constexpr (PAR) {
        kr = g.tdr[tap];
        kc = g.tdc[tap];
        bk = g.tko[tap] * g.Cin + c0;
      } else {
        kr = tap / g.KW;
        kc = tap - kr * g.KW;
      }
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        const int hi = a_h[i] + kr, wi = a_w[i] + kc;
        const bool ok = a_ok[i] && hi >= 0 && hi < g.Hi && wi >= 0 && wi < g.Wi;
        const uint16_t* p = ok ? a_src[i] + ((int64_t)hi * g.Wi + wi) * g.Cin + c0 : kZero16;
        glds16(p, base + arb(i) * rowlen);
        if constexpr (PRO) pro_ok |= (ok ? 1u : 0u) << i;
      }
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        glds16(a_ok[i] ? a_src[i] + k0 : kZero16, base + arb(i) * rowlen);
        if constexpr (PRO) pro_ok |= (a_ok[i] ? 1u : 0u) << i;
      }
    }
    if (do_b) {
#pragma unroll
      for (int i = 0; i < BIP; ++i) glds16(b_src(i) + bk, base + BM * rowlen + brb(i) * rowlen);
    }
  };
  auto issue = [&](int kt, int s) { issue_at(kt * BK, lds + s * STAGE, BK); };
  auto issue_unit = [&](int u) { issue_at(u * 32, lds + (u & 3) * UNIT, 32); };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int FM2 = M32 ? TM / 32 : 1, FN2 = M32 ? TN / 32 : 1;  // M32: 32x32 accumulators
  f32x16 acc32[FM2][FN2];
  if constexpr (M32) {
#pragma unroll
    for (int i = 0; i < FM2; ++i)
#pragma unroll
      for (int j = 0; j < FN2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc32[i][j][r] = 0.f;
  }

  // epilogue operands (residual-gradient addend, BN-backward x and bits) are loaded during the
  // MFMAs of the last K tile, when no DMA is in flight, if they fit the register budget
  constexpr bool ADDE = (EPI & kAdd) != 0;
  constexpr bool S2 = (EPI & kAddS2) != 0;
  constexpr int BSTE = (EPI & kBstBits) ? 2 : (EPI & kBst) ? 1 : 0;
  constexpr bool GELUB = (EPI & kGeluB) != 0;
  constexpr bool XS = BSTE || GELUB;  // the bx operand stream (BN input, or GELU pre-activation)
  // element offset in R of output row m's chunk (col), or -1 for a row that gets no addend (S2)
  auto r_off = [&](int m, int col) -> int64_t {
    if constexpr (S2) {
      const int hw = g.Ho * g.Wo;
      const int img = m / hw, rem = m - img * hw;
      const int h = rem / g.Wo, wv = rem - h * g.Wo;
      if ((h | wv) & 1) return -1;
      const int hs = (g.Ho + 1) >> 1, ws = (g.Wo + 1) >> 1;
      return (((int64_t)img * hs + (h >> 1)) * ws + (wv >> 1)) * g.N + col;
    } else {
      return (int64_t)m * g.N + col;
    }
  };
  constexpr int RCH = BN / 8;             // 16-byte chunks per output row
  constexpr int NOUT = BM * RCH / NT;     // output chunks per thread
  constexpr int NSTR = (ADDE ? 1 : 0) + (XS ? 1 : 0);       // epilogue operand streams
  // EPF: a 1x1 GEMM with a short K (<= 2 tiles: the memory-bound dgrad passes with a residual
  // add and a BN-backward reduction, K = 64..128) whose prefetched operands fit (PF) issues them
  // right after the first tile's DMA, so their HBM latency overlaps the DMA and the MFMAs
  // instead of following them.  (A larger PF budget for the 128x128 tile measured 138 -> 256
  // VGPRs: one wave per SIMD.)
  constexpr bool EPF_OK = !TAPS && !S2 && !PP && !KH && !M32 && !PRO && NSX == 2;
  constexpr bool PF = NSTR > 0 && NOUT * 5 * NSTR <= 40;  // <= 40 registers
  // vector-memory instructions of one prefetch (16-byte operand + mask byte per stream and chunk)
  constexpr int NPFL = PF ? NOUT * ((ADDE ? 2 : 0) + (BSTE == 2 ? 2 : XS ? 1 : 0)) : 0;
  static_assert(NPFL < 64, "vmcnt immediate");
  u32x4 pr[PF && ADDE ? NOUT : 1], px[PF && XS ? NOUT : 1];
  uint32_t prm[PF && ADDE ? NOUT : 1], pxm[PF && XS ? NOUT : 1];
  const uint8_t* rm_src = g.RM;  // (no mask: a byte of ones, so every prefetch issues the same loads)
  if constexpr (ADDE) {
    if (rm_src == nullptr) rm_src = kOnes8;
  }

  // epilogue operands loaded during the MFMAs of the last K step (no DMA in flight then)
  auto prefetch_epi = [&]() {
    if constexpr (PF) {
#pragma unroll
        for (int i = 0; i < NOUT; ++i) {
          const int id = t + NT * i;
          const int row = id / RCH, c = id - row * RCH;
          const int64_t o = orow(m0 + row < g.M ? m0 + row : m0) * g.N + n0 + c * 8;
          if constexpr (ADDE) {
            const int64_t ro = r_off(m0 + row < g.M ? m0 + row : m0, n0 + c * 8);
            pr[i] = ro >= 0 ? *reinterpret_cast<const u32x4*>(g.R + ro) : u32x4{0u, 0u, 0u, 0u};
            prm[i] = rm_src[rm_src == kOnes8 ? 0 : (o >> 3)];
          }
          if constexpr (XS) {
            px[i] = *reinterpret_cast<const u32x4*>(g.bx + o);
            pxm[i] = BSTE == 2 ? g.bbits[o >> 3] : 0u;
          }
        }
    }
  };
  if constexpr (PP) {
    const int KT = g.K / BK;
    const bool g1 = wm != 0;
    // MFMAs of tile kt (both k-steps' fragments read up front, the second set in flight while the
    // first step's MFMAs run)
    auto compute = [&](int kt) {
      const uint16_t* As = lds + (kt & 1) * STAGE;
      const uint16_t* Bs = As + BM * BK;
      // (TAPS: one fragment set -- the implicit-GEMM loader's per-row state leaves no room for two)
      constexpr int FS2 = TAPS ? 1 : 2;
      bf16x8 a[FS2][FM], b[FS2][FN];
      auto frag = [&](int ks, int slot) {
        const int c = ks * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * TN + j * 16 + (lane & 15);
          b[slot][j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((c ^ (row & 7)) << 3));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * TM + i * 16 + (lane & 15);
          a[slot][i] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((c ^ (row & 7)) << 3));
        }
      };
      if constexpr (FS2 == 2) {
        frag(0, 0);
        frag(1, 1);
        __builtin_amdgcn_s_waitcnt(waitcnt_lgkm(FM + FN));  // step 0's reads; step 1's in flight
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int slot = FS2 == 2 ? ks : 0;
        if constexpr (FS2 == 1) frag(ks, 0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[slot][i], b[slot][j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    };
    // prologue: tiles 0 and 1 (each group its part), drained; group 1 then waits out phase 0
    issue_at(0, lds, BK, g1);
    if (KT > 1) issue_at(BK, lds + STAGE, BK, g1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (g1) __builtin_amdgcn_s_barrier();
    // phase p ends at a barrier; group 0 computes tile kt in phase 2kt, group 1 in phase 2kt+1.
    // Every wave passes 2 + 2*KT barriers.
    for (int kt = 0; kt < KT; ++kt) {
      compute(kt);
      if (!g1) {
        __builtin_amdgcn_s_barrier();  // end of phase 2kt: this group's A half of stage kt&1 is free
        asm volatile("" ::: "memory");
        if (kt + 2 < KT) {
          issue_at((kt + 2) * BK, lds + (kt & 1) * STAGE, BK, false);
          __builtin_amdgcn_s_waitcnt(waitcnt_vm(AI));  // A half of tile kt+1 landed; kt+2's in flight
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();  // end of phase 2kt+1
        asm volatile("" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this group's part of tile kt+1 landed
        __builtin_amdgcn_s_barrier();  // end of phase 2kt+1: stage kt&1 fully read
        asm volatile("" ::: "memory");
        if (kt + 2 < KT) issue_at((kt + 2) * BK, lds + (kt & 1) * STAGE, BK, true);
        __builtin_amdgcn_s_barrier();  // end of phase 2kt+2
        asm volatile("" ::: "memory");
      }
    }
    if (!g1) __builtin_amdgcn_s_barrier();  // pairs group 1's end of phase 2KT
  } else if constexpr (KH) {
    // k-half units: unit u = K rows [32u, 32u + 32) in LDS slot u & 3
    const int NU = g.K / 32;
    issue_unit(0);
    if (NU > 1) issue_unit(1);
    if (NU > 2) issue_unit(2);
    for (int u = 0; u < NU; ++u) {
      // unit u landed (this wave's DMAs; up to two younger units stay in flight), this wave's
      // reads of unit u-1 retired; after the barrier the same holds for every wave
      const int younger = (NU - 1 - u) < 2 ? (NU - 1 - u) : 2;
      if (younger == 2) __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * NG));
      else if (younger == 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(NG));
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (u + 3 < NU) issue_unit(u + 3);  // into slot (u + 3) & 3 == (u - 1) & 3, just freed
      else if (u + 1 == NU) prefetch_epi();
      const uint16_t* As = lds + (u & 3) * UNIT;
      const uint16_t* Bs = As + BM * 32;
      bf16x8 a[FM], b[FN];
      const int c = lane >> 4;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * TN + j * 16 + (lane & 15);
        b[j] = *reinterpret_cast<const bf16x8*>(Bs + row * 32 + ((c ^ khalf_swz(row)) << 3));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * TM + i * 16 + (lane & 15);
        a[i] = *reinterpret_cast<const bf16x8*>(As + row * 32 + ((c ^ khalf_swz(row)) << 3));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
    const int KT = g.K / BK;
    issue(0, 0);
    if (NSX == 3 && KT > 1) issue(1, 1);
    const bool early = EPF_OK && PF && KT <= 2 && g.epf;
    if (early) {
      asm volatile("" ::: "memory");  // (the prefetch's loads issue after tile 0's DMA)
      prefetch_epi();
      asm volatile("" ::: "memory");
    }
    int cur = 0;
    for (int kt = 0; kt < KT; ++kt) {
      // this wave's DMA of tile kt has landed and its reads of tile kt-1 are retired; after the
      // barrier every wave's have, so tile kt is readable and tile kt-1's buffer is free to refill
      if (NSX == 3 && kt + 1 < KT) {
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(NG));  // tile kt+1 stays in flight
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      } else if (early && kt == 0) {
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(NPFL));  // tile 0 landed; the epilogue loads stay in flight
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      }
      if constexpr (PRO) {  // relu(x * scale + shift) on this thread's landed chunks of tile kt
        uint16_t* tb = lds + cur * STAGE;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
          if ((pro_ok >> i) & 1u) {
            uint4* q = reinterpret_cast<uint4*>(tb + RPI * (i * NW + w) * BK + lane * 8);
            const uint4 v = *q;
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float lo = fmaxf(fmaf(__uint_as_float(u[j] << 16), pro_sc[PRO ? 2 * j : 0], pro_sh[PRO ? 2 * j : 0]), 0.f);
              const float hi = fmaxf(fmaf(__uint_as_float(u[j] & 0xffff0000u), pro_sc[PRO ? 2 * j + 1 : 0],
                                          pro_sh[PRO ? 2 * j + 1 : 0]), 0.f);
              o[j] = pack_bf16x2(lo, hi);
            }
            *q = make_uint4(o[0], o[1], o[2], o[3]);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + NSX - 1 < KT) {
        int nxt = cur + NSX - 1;
        nxt = nxt >= NSX ? nxt - NSX : nxt;
        issue(kt + NSX - 1, nxt);
      } else if (kt + 1 < KT) {
        // NS == 3, second-to-last tile: nothing left to issue
      } else if (!early) {
        prefetch_epi();
      }
      const uint16_t* As = lds + cur * STAGE;
      cur = cur + 1 == NSX ? 0 : cur + 1;
      const uint16_t* Bs = As + BM * BK;
      if constexpr (M32) {
        // four 16-deep k-steps per 64-deep tile; step s+1's fragments are read while step s's
        // MFMAs run (counted lgkmcnt)
        bf16x8 a2[2][FM2], b2[2][FN2];
        auto frag32 = [&](int ks, int slot) {
          const int c = 2 * ks + (lane >> 5);
#pragma unroll
          for (int j = 0; j < FN2; ++j) {
            const int row = wn * TN + j * 32 + (lane & 31);
            b2[slot][j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((c ^ ((row >> 1) & 7)) << 3));
          }
#pragma unroll
          for (int i = 0; i < FM2; ++i) {
            const int row = wm * TM + i * 32 + (lane & 31);
            a2[slot][i] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((c ^ ((row >> 1) & 7)) << 3));
          }
        };
        frag32(0, 0);
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
          if (ks + 1 < BK / 16) {
            frag32(ks + 1, (ks + 1) & 1);
            __builtin_amdgcn_s_waitcnt(waitcnt_lgkm(FM2 + FN2));
          } else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < FM2; ++i)
#pragma unroll
            for (int j = 0; j < FN2; ++j)
              acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2[ks & 1][i], b2[ks & 1][j], acc32[i][j], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        }
        continue;
      }
      // FPF (one wave per SIMD): both k-steps' fragments are read up front, so the second step's
      // reads are in flight while the first step's MFMAs run (counted lgkmcnt) instead of a
      // read-wait-MFMA round per step; at two waves per SIMD (256x256) the other wave covers the
      // read latency and the registers are not there for two fragment sets
      constexpr bool FPF = NW <= 4;
      constexpr int KS = BK / 32, FS = FPF ? KS : 1;
      bf16x8 a[FS][FM], b[FS][FN];
      auto frag = [&](int ks, int slot) {
        const int c = ks * 4 + (lane >> 4);
  #pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * TN + j * 16 + (lane & 15);
          b[slot][j] = *reinterpret_cast<const bf16x8*>(Bs + row * BK + ((c ^ (row & 7)) << 3));
        }
  #pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * TM + i * 16 + (lane & 15);
          a[slot][i] = *reinterpret_cast<const bf16x8*>(As + row * BK + ((c ^ (row & 7)) << 3));
        }
      };
      if constexpr (FPF) {
  #pragma unroll
        for (int ks = 0; ks < KS; ++ks) frag(ks, ks);
      }
  #pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int slot = FPF ? ks : 0;
        if constexpr (FPF) {
          // step 0 needs its own FM + FN reads; the other step's stay in flight
          if (ks == 0 && FM + FN <= 15) __builtin_amdgcn_s_waitcnt(waitcnt_lgkm(FM + FN));
        } else {
          frag(ks, 0);
        }
        __builtin_amdgcn_s_setprio(1);
  #pragma unroll
        for (int i = 0; i < FM; ++i)
  #pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[slot][i], b[slot][j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: bf16 tile -> LDS (padded rows), per-channel stats, 16-byte row stores ----
  // C/D map (16x16x32): column = lane & 15, row = (lane >> 4) * 4 + r.
  float* st = reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(lds) + SCR);
  constexpr bool STATS = (EPI & kStats) != 0, ADD = (EPI & kAdd) != 0;
  constexpr int BST = (EPI & kBstBits) ? 2 : (EPI & kBst) ? 1 : 0;
  constexpr bool BIAS = (EPI & kBias) != 0;
  constexpr bool GBS = (EPI & kGeluBS) != 0;
  if constexpr (M32) {  // C/D map (32x32x16): column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int j = 0; j < FN2; ++j) {
      const int col = wn * TN + j * 32 + (lane & 31);
      const float bcol = BIAS ? g.bias[n0 + col] : 0.f;
      float s = 0.f, qq = 0.f;
#pragma unroll
      for (int i = 0; i < FM2; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const uint16_t hb = f32_to_bf16(BIAS ? acc32[i][j][r] + bcol : acc32[i][j][r]);
          lds[row * EP + col] = hb;
          if (STATS) {
            const float v = bf16_to_f32(hb);
            s += v;
            qq = fmaf(v, v, qq);
          }
        }
      }
      if (STATS) {
        s += __shfl_xor(s, 32, 64);
        qq += __shfl_xor(qq, 32, 64);
        if (lane < 32) {
          st[(wm * BN + col) * 2] = s;
          st[(wm * BN + col) * 2 + 1] = qq;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < (M32 ? 0 : FN); ++j) {
    const int col = wn * TN + j * 16 + (lane & 15);
    const float bcol = BIAS ? g.bias[n0 + col] : 0.f;
    float s = 0.f, qq = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const uint16_t hb = f32_to_bf16(BIAS ? acc[i][j][r] + bcol : acc[i][j][r]);
        lds[row * EP + col] = hb;
        if (STATS) {  // rows past M hold zeros (zero-page operands)
          const float v = bf16_to_f32(hb);
          s += v;
          qq = fmaf(v, v, qq);
        }
      }
    }
    if (STATS) {
      s += __shfl_xor(s, 16, 64);
      qq += __shfl_xor(qq, 16, 64);
      s += __shfl_xor(s, 32, 64);
      qq += __shfl_xor(qq, 32, 64);
      if (lane < 16) {
        st[(wm * BN + col) * 2] = s;
        st[(wm * BN + col) * 2 + 1] = qq;
      }
    }
  }
  __syncthreads();
  static_assert(BM * RCH % NT == 0 && NT % RCH == 0, "epilogue split");
  // BST: this thread's 8 channels are fixed (NT % RCH == 0): per-channel BN constants in registers
  const int cc = (t % RCH) * 8;
  float bmu[8], bis[8], bsc[8], bsh[8], bsa[8], bsb[8];
  if (GBS) {
#pragma unroll
    for (int j = 0; j < 8; ++j) bsa[j] = bsb[j] = 0.f;
  }
  if (BST) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bmu[j] = g.bmean[n0 + cc + j];
      bis[j] = g.binvstd[n0 + cc + j];
      bsc[j] = BST == 1 ? g.bscale[n0 + cc + j] : 0.f;
      bsh[j] = BST == 1 ? g.bshift[n0 + cc + j] : 0.f;
      bsa[j] = 0.f;
      bsb[j] = 0.f;
    }
  }
  // Without the MFMA-time prefetch (PF), the epilogue operands of NB chunks are loaded together
  // before any of them is used: loads and the Y stores interleaved chunk by chunk serialised every
  // chunk on two HBM round trips (the compiler cannot hoist a load of R / bx over a store to Y).
  constexpr int NB = PF ? 1 : (NOUT < 8 ? NOUT : 8);
  static_assert(NOUT % NB == 0, "epilogue batches");
#pragma unroll
  for (int i0 = 0; i0 < NOUT; i0 += NB) {
    u32x4 lr[NB], lx[NB];
    uint32_t lrm[NB], lxm[NB];
    if constexpr (!PF && NSTR > 0) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int id = t + NT * (i0 + b);
        const int row = id / RCH, c = id - row * RCH;
        const int mr = m0 + row < g.M ? m0 + row : m0;
        const int64_t o = orow(mr) * g.N + n0 + c * 8;
        if constexpr (ADDE) {
          if constexpr (S2) {
            const int64_t ro = r_off(mr, n0 + c * 8);
            const int64_t rc = ro >= 0 ? ro : 0;
            const u32x4 rv = *reinterpret_cast<const u32x4*>(g.R + rc);
            lr[b] = ro >= 0 ? rv : u32x4{0u, 0u, 0u, 0u};
          } else {
            lr[b] = *reinterpret_cast<const u32x4*>(g.R + o);
          }
          lrm[b] = g.RM != nullptr ? g.RM[o >> 3] : 0xffu;
        }
        if constexpr (XS) {
          lx[b] = *reinterpret_cast<const u32x4*>(g.bx + o);
          lxm[b] = BSTE == 2 ? g.bbits[o >> 3] : 0u;
        }
      }
    }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int i = i0 + b;
    const int id = t + NT * i;
    const int row = id / RCH, c = id - row * RCH;
    if (m0 + row < g.M) {
      const int64_t o = orow(m0 + row) * g.N + n0 + c * 8;
      uint4 v = *reinterpret_cast<const uint4*>(lds + row * EP + c * 8);
      if (ADD) {  // + R (* ReLU-mask bits): a second gradient path into Y
        u32x4 r;
        uint32_t mb;
        if constexpr (PF) {
          r = pr[i];
          mb = prm[i];
        } else {
          r = lr[b];
          mb = lrm[b];
        }
        {
          r.x &= (mb & 1u ? 0xffffu : 0u) | (mb & 2u ? 0xffff0000u : 0u);
          r.y &= (mb & 4u ? 0xffffu : 0u) | (mb & 8u ? 0xffff0000u : 0u);
          r.z &= (mb & 16u ? 0xffffu : 0u) | (mb & 32u ? 0xffff0000u : 0u);
          r.w &= (mb & 64u ? 0xffffu : 0u) | (mb & 128u ? 0xffff0000u : 0u);
        }
        v.x = add_bf16x2(v.x, r.x);
        v.y = add_bf16x2(v.y, r.y);
        v.z = add_bf16x2(v.z, r.z);
        v.w = add_bf16x2(v.w, r.w);
      }
      if constexpr ((EPI & kGelu) != 0) {  // v = pre-activation: kept for the backward, GELU stored
        *reinterpret_cast<uint4*>(g.Y2 + o) = v;
        uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          vw[j] = pack_bf16x2(gelu_f(__uint_as_float(vw[j] << 16)), gelu_f(__uint_as_float(vw[j] & 0xffff0000u)));
        v = uint4{vw[0], vw[1], vw[2], vw[3]};
      }
      if constexpr (GELUB) {  // v = bf16 input gradient of the GELU output -> of its input
        u32x4 xu;
        if constexpr (PF) xu = px[i];
        else xu = lx[b];
        const uint32_t xw[4] = {xu.x, xu.y, xu.z, xu.w};
        uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          vw[j] = pack_bf16x2(gelu_bwd_f(__uint_as_float(vw[j] << 16), __uint_as_float(xw[j] << 16)),
                              gelu_bwd_f(__uint_as_float(vw[j] & 0xffff0000u), __uint_as_float(xw[j] & 0xffff0000u)));
        v = uint4{vw[0], vw[1], vw[2], vw[3]};
        if constexpr (GBS) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            bsa[2 * j] += __uint_as_float(vw[j] << 16);
            bsa[2 * j + 1] += __uint_as_float(vw[j] & 0xffff0000u);
          }
        }
      }
      *reinterpret_cast<uint4*>(g.Y + o) = v;
      if (BST) {  // dz = dy * relu'(.) on the stored bf16 dy; x-hat from the BN input
        u32x4 xu;
        uint32_t mbits;
        if constexpr (PF) {
          xu = px[i];
          mbits = pxm[i];
        } else {
          xu = lx[b];
          mbits = lxm[b];
        }
        const uint32_t dv[4] = {v.x, v.y, v.z, v.w};
        const uint32_t xw[4] = {xu.x, xu.y, xu.z, xu.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = __uint_as_float(j & 1 ? dv[j >> 1] & 0xffff0000u : dv[j >> 1] << 16);
          const float xv = __uint_as_float(j & 1 ? xw[j >> 1] & 0xffff0000u : xw[j >> 1] << 16);
          const bool on = BST == 2 ? ((mbits >> j) & 1u) != 0u : fmaf(xv, bsc[j], bsh[j]) > 0.f;
          const float dz = on ? d : 0.f;
          bsa[j] += dz;
          bsb[j] = fmaf(dz, (xv - bmu[j]) * bis[j], bsb[j]);
        }
      }
    }
  }
  }
  if (BST || GBS) {  // combine the NT/RCH row lanes of each channel chunk through LDS, fixed order
    constexpr int RL = NT / RCH;
    static_assert(2 * RL * BN * 4 <= lds_bytes<BM, BN, NS>(), "BST scratch");
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(t / RCH) * BN + cc + j] = bsa[j];
      red[RL * BN + (t / RCH) * BN + cc + j] = bsb[j];
    }
    __syncthreads();
    if (t < BN) {
      float sa = 0.f, sb = 0.f;
      for (int r = 0; r < RL; ++r) {
        sa += red[r * BN + t];
        sb += red[RL * BN + r * BN + t];
      }
      if constexpr (GBS) {
        g.pa[(int64_t)mt * g.N + n0 + t] = sa;  // [mtiles][N]: rows of column partial sums
      } else {
        g.pa[(int64_t)(n0 + t) * g.pstride + g.pcol0 + mt] = sa;
        g.pb[(int64_t)(n0 + t) * g.pstride + g.pcol0 + mt] = sb;
      }
    }
  }
  if (STATS && t < BN) {
    float sa = 0.f, qa = 0.f;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      sa += st[(i * BN + t) * 2];
      qa += st[(i * BN + t) * 2 + 1];
    }
    g.pa[(int64_t)(n0 + t) * g.pstride + g.pcol0 + mt] = sa;
    g.pb[(int64_t)(n0 + t) * g.pstride + g.pcol0 + mt] = qa;
  }
}

// ==========================================================================================
// Weight gradient:  dW[N][Kt] = sum_m dY[m][n] * X[src(m, tap)][c]     (Kt = KH*KW*Cin, k = tap*Cin + c)
//
// The first core's split-M kernel (gemm.hip k_conv1x1_wgrad2) with the operand path of this file:
// each 64-row M stage of dY [64][TN] and X [64][TK] goes global -> LDS by DMA (16-byte chunks, the
// XOR swizzle ch ^ f(row) applied on the per-lane global address), two stages, one barrier per
// stage; fragments are read with the transposing ds_read_b64_tr_b16 (8 consecutive m per lane).
// Rows past the block's M chunk and padding taps read the zero page.  Each block writes an fp32
// partial slab; gemm.hip wgrad_reduce_slabs sums the S slabs in a fixed order.
struct FastDiv2 {
  uint32_t d, mul, shift;
};
inline FastDiv2 make_fastdiv2(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t mul = ((((1ull << l) - d) << 32) / d) + 1;
  return FastDiv2{d, (uint32_t)mul, l};
}
__device__ __forceinline__ uint32_t fdiv2(uint32_t n, const FastDiv2& f) { return (__umulhi(n, f.mul) + n) >> f.shift; }

struct WArgs {
  const uint16_t* dY;
  const uint16_t* X;
  float* part;
  int M, N, K, Cin, Ho, Wo, Hi, Wi, stride, KW, pad, chunk, tn, tk;
  FastDiv2 fd_hw, fd_w;
  const float *psc, *psh;  // PRO: the X operand is a BN input; the GEMM reads relu(x * psc + psh)
  // in-launch split-M reduction (S > 1): per-tile arrival tickets (zero on entry, re-armed by the
  // reducer), the number of slabs S, the reduce1 group count G (same order as gemm.hip
  // wgrad_reduce_slabs, so the result is bit-identical to the separate reduce kernels) and dW
  int* cnt;
  int S, G;
  float* dw;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));

template <int TW>
__device__ __forceinline__ int wswz(int row) {  // chunk XOR of a [rows][TW x bf16] tile row
  // (a 256-wide row spans two 256-byte bank rows: the XOR acts on the chunk within a bank row)
  return TW >= 128 ? (((row & 3) << 2) | ((row >> 2) & 3)) : (((row & 3) << 1) | ((row >> 2) & 1));
}

template <int TW>
__device__ __forceinline__ bf16x8 tr_frag2(const uint8_t* tile, int row0, int col0, int lane) {
  // rows row0 + 8*(lane>>4) + {0..3, 4..7}, columns col0 .. col0+15 (col0 % 16 == 0)
  const int il = lane & 15, q = il >> 2, p = il & 3;
  const int r = row0 + 8 * (lane >> 4) + q;
  const int ch = (col0 >> 3) + (p >> 1);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + 2 * TW * r + 16 * (ch ^ wswz<TW>(r)) + 8 * (p & 1)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s16x4*)(tile + 2 * TW * (r + 4) + 16 * (ch ^ wswz<TW>(r + 4)) + 8 * (p & 1)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

constexpr int kWM = 64;  // m rows per stage

// TN x TK output tile on WN x WK waves (each (TN/WN) x (TK/WK) of 16x16 accumulators)
// NS LDS stages as in k_gemm (3: one stage's DMA in flight across every barrier)
// MT (multi-tap): TK > Cin, each 16-byte X chunk takes its own tap (k = tap*Cin + c); K may be
// padded up to a multiple of TK (columns past K read the zero page and are not stored) -- the
// 64-channel 3x3 layers, whose 64-wide tiles are LDS-read bound
// PRO (2 stages): BN + ReLU on the X operand, transformed in LDS by the thread that staged each
// chunk after its own DMA landed (as k_gemm kPro); the per-channel scale / shift of the tile's
// channels sit in a table at the end of the LDS array
template <int TN, int TK, int WN, int WK, int NS, bool MT = false, bool PRO = false>
__global__ __launch_bounds__(64 * WN * WK) void k_wgrad(WArgs g) {
  constexpr int NW = WN * WK;
  // NS == 4 (k-half units, as k_gemm): 32-row units in 4 slots, two in flight at each barrier
  constexpr bool KH = NS == 4;
  constexpr int UR = KH ? 32 : kWM;                    // M rows per staged unit
  constexpr int NSLOT = KH ? 4 : NS;
  constexpr int YT = UR * TN * 2, XT = UR * TK * 2;    // bytes per staged unit
  constexpr int CY = TN / 8, CX = TK / 8;             // 16-byte chunks per staged row
  constexpr int RY = 64 / CY > 0 ? 64 / CY : 1;       // rows per wave-instruction (1 KB)
  constexpr int RX = 64 / CX > 0 ? 64 / CX : 1;
  constexpr int IY = UR / RY / NW, IX = UR / RX / NW;  // wave-instructions per unit per wave
  constexpr int WTN = TN / WN, WTK = TK / WK;
  constexpr int FN = WTN / 16, FK = WTK / 16;
  static_assert(CY <= 64 && CX <= 64 && IY >= 1 && IX >= 1, "wgrad tile");
  static_assert(NS >= 2 && NS <= 4, "stages");
  constexpr int NG = IY + IX;  // glds per unit per wave
  static_assert(!PRO || NS == 2, "PRO: 2 stages");
  constexpr int TT = PRO ? (MT ? 64 : TK) : 0;  // channels in the BN table
  __shared__ __attribute__((aligned(16))) uint8_t lds[NSLOT * (YT + XT) + 2 * TT * 4];
  float* ptab = reinterpret_cast<float*>(lds + NSLOT * (YT + XT));  // [2][TT]: scale, shift
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tiles = g.tn * g.tk;
  const int sidx = bid / tiles, tile = bid - sidx * tiles;
  const int n0 = (tile / g.tk) * TN, k0 = (tile % g.tk) * TK;
  const int mbeg = sidx * g.chunk, mend = min(g.M, mbeg + g.chunk);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wn = w / WK, wk = w - (w / WK) * WK;
  const int tap = k0 / g.Cin, c0 = k0 - tap * g.Cin;
  const int kr = tap / g.KW, kc = tap - kr * g.KW;
  const bool direct = !MT && g.KW == 1 && g.pad == 0 && g.stride == 1 && g.Cin == g.K;
  // lane -> (row within the wave-instruction, logical chunk); the LDS slot is lane % C
  const int ry = lane / CY, sy = lane % CY, rx = lane / CX, sx = lane % CX;
  // MT: per X wave-instruction, this lane's chunk column -> (tap row, tap col, channel, in K)
  int xkr[MT ? IX : 1], xkc[MT ? IX : 1], xch[MT ? IX : 1];
  bool xin[MT ? IX : 1];
  if constexpr (MT) {
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int row = (i * NW + w) * RX + rx;
      const int kk = k0 + (sx ^ wswz<TK>(row)) * 8;
      const int tp = kk / g.Cin;
      xin[i] = kk < g.K;
      xkr[i] = tp / g.KW;
      xkc[i] = tp - xkr[i] * g.KW;
      xch[i] = kk - tp * g.Cin;
    }
  }

  const int tc0 = MT ? 0 : c0;  // PRO: first channel of the table
  if constexpr (PRO) {  // before any DMA is in flight (the barrier would drain it)
    for (int c = t; c < TT; c += 64 * NW) {
      ptab[c] = g.psc[tc0 + c];
      ptab[TT + c] = g.psh[tc0 + c];
    }
    __syncthreads();
  }
  uint32_t xok = 0;  // PRO: this thread's X chunks of the staged stage that hold data
  // implicit-GEMM X rows: (image, ho, wo) of this lane's row i in the next stage to issue, advanced
  // by UR rows per stage with adds and compares instead of two divisions per chunk per stage
  // (stages are issued strictly in order)
  // (8-wave tiles keep the divisions: the 256x256 kernel is at the 256-register cap)
  constexpr bool INC = NW <= 4;
  int xs_img[INC ? IX : 1], xs_ho[INC ? IX : 1], xs_wo[INC ? IX : 1];
  const int dq = UR / g.Wo, dr = UR - dq * g.Wo;
  if (INC && !direct) {
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int m = mbeg + (i * NW + w) * RX + rx;
      const int img = (int)fdiv2((uint32_t)m, g.fd_hw), rem = m - img * (int)g.fd_hw.d;
      const int ho = (int)fdiv2((uint32_t)rem, g.fd_w);
      xs_img[INC ? i : 0] = img;
      xs_ho[INC ? i : 0] = ho;
      xs_wo[INC ? i : 0] = rem - ho * g.Wo;
    }
  }
  auto issue = [&](int st, int s) {
    uint8_t* ty = lds + s * (YT + XT);
    uint8_t* tx = ty + YT;
    const int mb = mbeg + st * UR;
    if constexpr (PRO) xok = 0;
#pragma unroll
    for (int i = 0; i < IY; ++i) {
      const int row = (i * NW + w) * RY + ry;
      const int m = mb + row;
      const int ch = sy ^ wswz<TN>(row);
      const uint16_t* p = m < mend ? g.dY + (int64_t)m * g.N + n0 + ch * 8 : kZero16;
      glds16(p, ty + (i * NW + w) * 1024);
    }
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int row = (i * NW + w) * RX + rx;
      const int m = mb + row;
      const int ch = sx ^ wswz<TK>(row);
      const uint16_t* p = kZero16;
      if (m < mend) {
        if (direct) {
          p = g.X + (int64_t)m * g.Cin + c0 + ch * 8;
        } else {
          int img, ho, wo;
          if constexpr (INC) {
            img = xs_img[INC ? i : 0];
            ho = xs_ho[INC ? i : 0];
            wo = xs_wo[INC ? i : 0];
          } else {
            img = (int)fdiv2((uint32_t)m, g.fd_hw);
            const int rem = m - img * (int)g.fd_hw.d;
            ho = (int)fdiv2((uint32_t)rem, g.fd_w);
            wo = rem - ho * g.Wo;
          }
          const int hi = ho * g.stride - g.pad + (MT ? xkr[MT ? i : 0] : kr);
          const int wi = wo * g.stride - g.pad + (MT ? xkc[MT ? i : 0] : kc);
          const bool inx = MT ? xin[MT ? i : 0] : true;
          if (inx && hi >= 0 && hi < g.Hi && wi >= 0 && wi < g.Wi)
            p = g.X + (((int64_t)img * g.Hi + hi) * g.Wi + wi) * g.Cin + (MT ? xch[MT ? i : 0] : c0 + ch * 8);
        }
      }
      glds16(p, tx + (i * NW + w) * 1024);
      if constexpr (PRO) xok |= (p != kZero16 ? 1u : 0u) << i;
      if (INC && !direct) {  // this row in the next stage: m + UR
        int wo = xs_wo[INC ? i : 0] + dr, ho = xs_ho[INC ? i : 0] + dq, img = xs_img[INC ? i : 0];
        if (wo >= g.Wo) { wo -= g.Wo; ++ho; }
        while (ho >= g.Ho) { ho -= g.Ho; ++img; }
        xs_wo[INC ? i : 0] = wo;
        xs_ho[INC ? i : 0] = ho;
        xs_img[INC ? i : 0] = img;
      }
    }
  };

  f32x4 acc[FN][FK];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (KH) {
    const int nu = (mend - mbeg + UR - 1) / UR;
    issue(0, 0);
    if (nu > 1) issue(1, 1);
    if (nu > 2) issue(2, 2);
    for (int u = 0; u < nu; ++u) {
      const int younger = (nu - 1 - u) < 2 ? (nu - 1 - u) : 2;
      if (younger == 2) __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * NG));
      else if (younger == 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(NG));
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (u + 3 < nu) issue(u + 3, (u + 3) & 3);  // the slot unit u-1 just freed
      const uint8_t* ty = lds + (u & 3) * (YT + XT);
      const uint8_t* tx = ty + YT;
      bf16x8 a[FN], b[FK];
#pragma unroll
      for (int i = 0; i < FN; ++i) a[i] = tr_frag2<TN>(ty, 0, wn * WTN + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FK; ++j) b[j] = tr_frag2<TK>(tx, 0, wk * WTK + j * 16, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  } else {
  const int nst = (mend - mbeg + kWM - 1) / kWM;
  issue(0, 0);
  if (NS == 3 && nst > 1) issue(1, 1);
  int cur = 0;
  for (int st = 0; st < nst; ++st) {
    if (NS == 3 && st + 1 < nst) {
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(NG));  // stage st+1 stays in flight
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    if constexpr (PRO) {  // relu(x * scale + shift) on this thread's landed X chunks of stage st
      uint8_t* txs = lds + cur * (YT + XT) + YT;
#pragma unroll
      for (int i = 0; i < IX; ++i) {
        if ((xok >> i) & 1u) {
          const int row = (i * NW + w) * RX + rx;
          const int chan = (MT ? xch[MT ? i : 0] : c0 + (sx ^ wswz<TK>(row)) * 8) - tc0;
          uint4* q = reinterpret_cast<uint4*>(txs + (i * NW + w) * 1024 + lane * 16);
          const uint4 v = *q;
          const uint32_t u[4] = {v.x, v.y, v.z, v.w};
          uint32_t o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float lo = fmaxf(fmaf(__uint_as_float(u[j] << 16), ptab[chan + 2 * j], ptab[TT + chan + 2 * j]), 0.f);
            const float hi = fmaxf(fmaf(__uint_as_float(u[j] & 0xffff0000u), ptab[chan + 2 * j + 1],
                                        ptab[TT + chan + 2 * j + 1]), 0.f);
            o[j] = pack_bf16x2(lo, hi);
          }
          *q = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (st + NS - 1 < nst) {
      int nxt = cur + NS - 1;
      nxt = nxt >= NS ? nxt - NS : nxt;
      issue(st + NS - 1, nxt);
    }
    const uint8_t* ty = lds + cur * (YT + XT);
    cur = cur + 1 == NS ? 0 : cur + 1;
    const uint8_t* tx = ty + YT;
    // one wave per SIMD (NW <= 4): both 32-row steps' fragments are read up front and the
    // second step's transposing reads overlap the first step's MFMAs (counted lgkmcnt)
    constexpr bool FPF = NW <= 4;
    constexpr int KS = kWM / 32, FS = FPF ? KS : 1;
    bf16x8 a[FS][FN], b[FS][FK];
    auto frag = [&](int ks, int slot) {
#pragma unroll
      for (int i = 0; i < FN; ++i) a[slot][i] = tr_frag2<TN>(ty, ks * 32, wn * WTN + i * 16, lane);
#pragma unroll
      for (int j = 0; j < FK; ++j) b[slot][j] = tr_frag2<TK>(tx, ks * 32, wk * WTK + j * 16, lane);
    };
    if constexpr (FPF) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) frag(ks, ks);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int slot = FPF ? ks : 0;
      if constexpr (FPF) {
        constexpr int later = 2 * (FN + FK);  // ds_read_b64_tr per step
        if (ks == 0) __builtin_amdgcn_s_waitcnt(waitcnt_lgkm(later < 15 ? later : 15));
      } else {
        frag(ks, 0);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FK; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[slot][i], b[slot][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  }
  // D map: column (k) = lane & 15, row (n) = (lane >> 4) * 4 + r
  float* out = g.part + (int64_t)sidx * g.N * g.K;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FK; ++j) {
      const int k = k0 + wk * WTK + j * 16 + (lane & 15);
      if (MT && k >= g.K) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * WTN + i * 16 + (lane >> 4) * 4 + r;
        out[(int64_t)n * g.K + k] = acc[i][j][r];
      }
    }
  if (g.cnt == nullptr) return;  // S == 1 wrote dW directly, or the separate reduce kernels run
  // In-launch split-M reduction: the block that completes a tile's S slabs sums them
  // (cdna_hip_programming.md, "In-launch split-K reduction": plain slab stores, every wave drains,
  // one agent-scope release before the ticket, one agent-scope acquire in the reducer; correct for
  // any placement of a tile's slabs over XCDs).  Replaces one or two reduce launches per layer.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's slab stores have completed; LDS is free (main loop done)
  int* flag = reinterpret_cast<int*>(lds);  // the one LDS array (no second __shared__ object)
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(g.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == g.S - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(g.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
    }
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  // dW[n][k..k+3] = sum over slabs in wgrad_reduce_slabs' order: G groups of consecutive slabs,
  // each summed with 4 interleaved accumulators, then the group sums in order
  const int64_t NK = (int64_t)g.N * g.K;
  constexpr int TK4 = TK / 4;
  for (int e = t; e < TN * TK4; e += 64 * NW) {
    const int n = n0 + e / TK4, k = k0 + (e - (e / TK4) * TK4) * 4;
    if (MT && k >= g.K) continue;
    const float* base = g.part + (int64_t)n * g.K + k;
    float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int gi = 0; gi < g.G; ++gi) {
      const int s0 = (int)((int64_t)gi * g.S / g.G), s1 = (int)((int64_t)(gi + 1) * g.S / g.G);
      float4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      int s = s0;
      for (; s + 3 < s1; s += 4) {
        float4 b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = *reinterpret_cast<const float4*>(base + (int64_t)(s + u) * NK);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u].x += b[u].x; a[u].y += b[u].y; a[u].z += b[u].z; a[u].w += b[u].w;
        }
      }
      for (; s < s1; ++s) {
        const float4 b = *reinterpret_cast<const float4*>(base + (int64_t)s * NK);
        a[0].x += b.x; a[0].y += b.y; a[0].z += b.z; a[0].w += b.w;
      }
      float4 r;
      r.x = (a[0].x + a[1].x) + (a[2].x + a[3].x);
      r.y = (a[0].y + a[1].y) + (a[2].y + a[3].y);
      r.z = (a[0].z + a[1].z) + (a[2].z + a[3].z);
      r.w = (a[0].w + a[1].w) + (a[2].w + a[3].w);
      if (gi == 0) {
        tot = r;
      } else {
        tot.x += r.x; tot.y += r.y; tot.z += r.z; tot.w += r.w;
      }
    }
    *reinterpret_cast<float4*>(g.dw + (int64_t)n * g.K + k) = tot;
  }
}

// default block tile for a problem (the Python side autotunes per shape and passes bm / bn)
inline void pick_tile(int64_t M, int64_t N, int64_t K, int& bm, int& bn) {
  auto blocks = [&](int a, int b) { return ((M + a - 1) / a) * (N / b); };
  if (N % 256 == 0 && ((K >= 1024 && blocks(256, 256) >= 192 && blocks(128, 128) < 1536) ||
                       (K >= 2048 && blocks(256, 256) >= 512))) {
    bm = 256; bn = 256; return;
  }
  if (N % 128 == 0) { bm = 128; bn = 128; return; }
  bm = 128; bn = 64;
}

}  // namespace g2

int64_t gemm2_mtiles(int64_t M, int64_t N, int64_t K, int64_t bm) {
  int b = (int)bm, n = 0;
  if (b <= 0) g2::pick_tile(M, N, K, b, n);
  return (M + b - 1) / b;
}

// x: [img, Cin, Hi, Wi] channels-last bf16; w: [Cout, Cin, KH, KW] channels-last bf16 (1x1: [Cout, Cin]);
// y: [img, Cout, Ho, Wo] channels-last bf16.
//   part (optional): f32 [2, Cout, mtiles] (mtiles = gemm2_mtiles(M, N, K, bm)): the forward BN
//     statistics of y, or -- with bn_x -- the backward BN reduction of the BN whose output
//     gradient y is (bn_x its input, bn_bits its ReLU bits or none to recompute relu' from
//     bn_x * bn_scale + bn_shift)
//   add (+ add_mask, 1x1 only): y = conv(x) + add (* mask bits); with add_s2 add is the compact
//     [img, ceil(Ho/2), ceil(Wo/2), Cout] input gradient of a stride-2 1x1 conv over the same
//     tensor, added on the even (h, w) rows only (ResNet downsample branch)
//   bm / bn: block tile (0 = default per shape); stages: LDS stages (2, or 3 below 256x256)
//   gelu_pre + gelu (1x1, no other epilogue): gelu=1 -> y = gelu(x w^T + bias), gelu_pre = the
//     bf16 pre-activation; gelu=2 -> y = gelu'(gelu_pre) * (x w^T), the GELU backward folded
//     into an input-gradient GEMM (x = the output gradient, w = the next layer's weight^T)
void gemm2_conv(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part,
                c10::optional<at::Tensor> add, c10::optional<at::Tensor> add_mask, int64_t Hi, int64_t Wi,
                int64_t stride, int64_t KH, int64_t KW, int64_t pad, int64_t bm, int64_t bn,
                c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_bits, c10::optional<at::Tensor> bn_mean,
                c10::optional<at::Tensor> bn_invstd, c10::optional<at::Tensor> bn_scale,
                c10::optional<at::Tensor> bn_shift, int64_t stages, bool add_s2,
                c10::optional<at::Tensor> pro_scale, c10::optional<at::Tensor> pro_shift,
                c10::optional<at::Tensor> bias, c10::optional<at::Tensor> gelu_pre, int64_t gelu) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && y.is_cuda(), "gemm2: device tensors");
  TORCH_CHECK(stages >= 2 && stages <= 6,
              "gemm2: stages must be 2, 3, 4 (k-half units), 5 (ping-pong) or 6 (32x32x16 MFMA)");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  y.scalar_type() == at::kBFloat16, "gemm2: bf16 tensors");
  const int64_t N = w.size(0), K = w.numel() / N, Cin = K / (KH * KW);
  TORCH_CHECK(Cin * KH * KW == K && Cin % g2::BK == 0 && N % 64 == 0, "gemm2: needs Cin % 64 == 0, Cout % 64 == 0");
  const int64_t imgs = x.numel() / (Cin * Hi * Wi);
  TORCH_CHECK(imgs * Cin * Hi * Wi == x.numel(), "gemm2: x size");
  const int64_t Ho = (Hi + 2 * pad - KH) / stride + 1, Wo = (Wi + 2 * pad - KW) / stride + 1;
  const int64_t M = imgs * Ho * Wo;
  TORCH_CHECK(y.numel() == M * N, "gemm2: y size");
  TORCH_CHECK(w.is_contiguous() || w.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2: dense w");
  for (const at::Tensor* t : {&x, &w, &y})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm2: 16-byte aligned tensors");
  TORCH_CHECK(x.dim() != 4 || x.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2: channels-last x");
  TORCH_CHECK(y.dim() != 4 || y.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2: channels-last y");
  TORCH_CHECK(w.dim() != 4 || KH * KW == 1 || w.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2: channels-last w");
  TORCH_CHECK(M < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 40), "gemm2: size");
  int BMv = (int)bm, BNv = (int)bn;
  if (BMv <= 0 || BNv <= 0) g2::pick_tile(M, N, K, BMv, BNv);
  TORCH_CHECK(N % BNv == 0, "gemm2: Cout must be a multiple of the block tile");
  const int64_t mtiles = (M + BMv - 1) / BMv, ntiles = N / BNv;
  TORCH_CHECK(mtiles * ntiles < (int64_t(1) << 31), "gemm2: grid");
  g2::Args a{};
  a.X = (const uint16_t*)x.data_ptr();
  a.W = (const uint16_t*)w.data_ptr();
  a.Y = (uint16_t*)y.data_ptr();
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.Ho = (int)Ho; a.Wo = (int)Wo; a.Hi = (int)Hi; a.Wi = (int)Wi;
  a.stride = (int)stride; a.mtiles = (int)mtiles; a.ntiles = (int)ntiles;
  a.KW = (int)KW; a.pad = (int)pad; a.Cin = (int)Cin;
  a.ldb = (int)K; a.pstride = (int)mtiles; a.pcol0 = 0;
  int epi = g2::kPlain;
  if (part.has_value() && part->defined()) {
    TORCH_CHECK(part->is_cuda() && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->numel() == (gelu == 2 ? 1 : 2) * N * mtiles,
                "gemm2: part must be f32 [2, Cout, mtiles] ([mtiles, Cout] with the GELU backward)");
    a.pa = part->data_ptr<float>();
    a.pb = a.pa + N * mtiles;
  }
  const bool taps = !(KH == 1 && KW == 1 && pad == 0);
  if (add.has_value() && add->defined()) {
    TORCH_CHECK(!taps, "gemm2: the add epilogue is for 1x1 convolutions");
    // add shaped like y, or (a stride-1 conv over [img, Ho, Wo]) the compact [img, ceil(Ho/2),
    // ceil(Wo/2), N] input gradient of a stride-2 1x1 conv over the same tensor (add_s2)
    const int64_t Ms2 = imgs * ((Ho + 1) / 2) * ((Wo + 1) / 2);
    const bool s2 = add_s2;
    TORCH_CHECK(!s2 || (stride == 1 && !(add_mask.has_value() && add_mask->defined())),
                "gemm2: add_s2 needs a stride-1 conv and no add mask");
    TORCH_CHECK(add->is_cuda() && add->scalar_type() == at::kBFloat16 && add->numel() == (s2 ? Ms2 : M) * N &&
                    (add->dim() != 4 || add->is_contiguous(at::MemoryFormat::ChannelsLast)) &&
                    reinterpret_cast<uintptr_t>(add->data_ptr()) % 16 == 0, "gemm2: add shaped like y (or compact)");
    if (s2) epi |= g2::kAddS2;
    a.R = (const uint16_t*)add->data_ptr();
    if (add_mask.has_value() && add_mask->defined()) {
      TORCH_CHECK(add_mask->is_cuda() && add_mask->scalar_type() == at::kByte && add_mask->is_contiguous() &&
                      add_mask->numel() == M * N / 8, "gemm2: add_mask must be uint8[numel(y)/8]");
      a.RM = (const uint8_t*)add_mask->data_ptr();
    }
    epi |= g2::kAdd;
  }
  if (bn_x.has_value() && bn_x->defined()) {
    TORCH_CHECK(a.pa != nullptr, "gemm2: BN-backward statistics need part");
    TORCH_CHECK(bn_x->is_cuda() && bn_x->scalar_type() == at::kBFloat16 && bn_x->numel() == M * N &&
                    (bn_x->dim() != 4 || bn_x->is_contiguous(at::MemoryFormat::ChannelsLast)) &&
                    reinterpret_cast<uintptr_t>(bn_x->data_ptr()) % 16 == 0, "gemm2: bn_x shaped like y");
    for (const c10::optional<at::Tensor>* v : {&bn_mean, &bn_invstd, &bn_scale, &bn_shift})
      TORCH_CHECK(v->has_value() && (*v)->defined() && (*v)->is_cuda() && (*v)->scalar_type() == at::kFloat &&
                      (*v)->is_contiguous() && (*v)->numel() == N, "gemm2: BN vectors must be f32 [C]");
    a.bx = (const uint16_t*)bn_x->data_ptr();
    a.bmean = bn_mean->data_ptr<float>();
    a.binvstd = bn_invstd->data_ptr<float>();
    a.bscale = bn_scale->data_ptr<float>();
    a.bshift = bn_shift->data_ptr<float>();
    if (bn_bits.has_value() && bn_bits->defined()) {
      TORCH_CHECK(bn_bits->is_cuda() && bn_bits->scalar_type() == at::kByte && bn_bits->is_contiguous() &&
                      bn_bits->numel() == M * N / 8, "gemm2: bn_bits must be uint8[numel(y)/8]");
      a.bbits = (const uint8_t*)bn_bits->data_ptr();
      epi |= g2::kBstBits;
    } else {
      epi |= g2::kBst;
    }
  } else if (a.pa != nullptr && gelu != 2) {
    TORCH_CHECK(!(epi & g2::kAdd), "gemm2: forward statistics and the add epilogue are exclusive");
    epi |= g2::kStats;
  }
  if (pro_scale.has_value() && pro_scale->defined()) {
    TORCH_CHECK(stages == 2 && epi == g2::kStats, "gemm2: the BN prologue runs with 2 stages and forward statistics");
    for (const c10::optional<at::Tensor>* v : {&pro_scale, &pro_shift})
      TORCH_CHECK(v->has_value() && (*v)->defined() && (*v)->is_cuda() && (*v)->scalar_type() == at::kFloat &&
                      (*v)->is_contiguous() && (*v)->numel() == Cin &&
                      reinterpret_cast<uintptr_t>((*v)->data_ptr()) % 16 == 0,
                  "gemm2: prologue scale / shift must be 16-byte aligned f32 [Cin]");
    a.psc = pro_scale->data_ptr<float>();
    a.psh = pro_shift->data_ptr<float>();
    epi |= g2::kPro;
  }
  if (gelu_pre.has_value() && gelu_pre->defined()) {
    TORCH_CHECK(epi == g2::kPlain && !taps && (gelu == 1 || gelu == 2),
                "gemm2: the GELU epilogues run on a plain 1x1 GEMM (gelu=1 forward, 2 backward)");
    TORCH_CHECK(gelu_pre->is_cuda() && gelu_pre->scalar_type() == at::kBFloat16 && gelu_pre->numel() == M * N &&
                    gelu_pre->is_contiguous() && reinterpret_cast<uintptr_t>(gelu_pre->data_ptr()) % 16 == 0,
                "gemm2: gelu_pre must be a 16-byte aligned contiguous bf16 tensor shaped like y");
    if (gelu == 1) {
      a.Y2 = (uint16_t*)gelu_pre->data_ptr();
      epi |= g2::kGelu;
    } else {
      TORCH_CHECK(!(bias.has_value() && bias->defined()), "gemm2: the GELU backward epilogue takes no bias");
      a.bx = (const uint16_t*)gelu_pre->data_ptr();
      epi |= g2::kGeluB;
      if (a.pa != nullptr) epi |= g2::kGeluBS;  // + the column sums of y, per m-tile
    }
  } else {
    TORCH_CHECK(gelu == 0, "gemm2: gelu needs gelu_pre");
  }
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK((epi == g2::kPlain || epi == g2::kAdd || epi == g2::kGelu) && !taps,
                "gemm2: the bias epilogue runs on a 1x1 GEMM, alone or with a plain add (a residual)");
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() == N,
                "gemm2: bias must be f32 [Cout]");
    a.bias = bias->data_ptr<float>();
    epi |= g2::kBias;
  }
  static const int epf_env = [] {
    const char* e = std::getenv("HIPPS_G2_EPF");
    return e ? std::atoi(e) : 1;
  }();
  a.epf = epf_env;
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = (int)(mtiles * ntiles);
#define HIPPS_G2S(BMc, BNc, EPc, TPc, NSc) \
  hipLaunchKernelGGL((g2::k_gemm<BMc, BNc, EPc, TPc, NSc>), grid, (g2::nthreads<BMc, BNc>()), 0, stream, a)
#define HIPPS_G2(BMc, BNc, EPc, TPc) \
  do {                                                      \
    if (NS3) HIPPS_G2S(BMc, BNc, EPc, TPc, NS3_OF(BMc, BNc)); \
    else if (NS4) HIPPS_G2S(BMc, BNc, EPc, TPc, 4);          \
    else if (NS5) HIPPS_G2S(BMc, BNc, EPc, TPc, NS5_OF(BMc, BNc)); \
    else if (NS6) HIPPS_G2S(BMc, BNc, EPc, TPc, NS6_OF(BMc, BNc)); \
    else HIPPS_G2S(BMc, BNc, EPc, TPc, 2);                   \
  } while (0)
#define HIPPS_G2_E(BMc, BNc)                                                                        \
  do {                                                                                              \
    if (taps) {                                                                                     \
      switch (epi) {                                                                                \
        case g2::kStats | g2::kPro: HIPPS_G2S(BMc, BNc, (g2::kStats | g2::kPro), true, 2); break;    \
        case g2::kStats: HIPPS_G2(BMc, BNc, g2::kStats, true); break;                               \
        case g2::kBst: HIPPS_G2(BMc, BNc, g2::kBst, true); break;                                   \
        case g2::kBstBits: HIPPS_G2(BMc, BNc, g2::kBstBits, true); break;                           \
        default: HIPPS_G2(BMc, BNc, g2::kPlain, true); break;                                       \
      }                                                                                             \
    } else {                                                                                        \
      switch (epi) {                                                                                \
        case g2::kStats | g2::kPro: HIPPS_G2S(BMc, BNc, (g2::kStats | g2::kPro), false, 2); break;   \
        case g2::kStats: HIPPS_G2(BMc, BNc, g2::kStats, false); break;                              \
        case g2::kAdd: HIPPS_G2(BMc, BNc, g2::kAdd, false); break;                                  \
        case g2::kBias: HIPPS_G2(BMc, BNc, g2::kBias, false); break;                                \
        case g2::kBias | g2::kAdd: HIPPS_G2(BMc, BNc, (g2::kBias | g2::kAdd), false); break;        \
        case g2::kGelu: HIPPS_G2(BMc, BNc, g2::kGelu, false); break;                                \
        case g2::kBias | g2::kGelu: HIPPS_G2(BMc, BNc, (g2::kBias | g2::kGelu), false); break;      \
        case g2::kGeluB: HIPPS_G2(BMc, BNc, g2::kGeluB, false); break;                              \
        case g2::kGeluB | g2::kGeluBS: HIPPS_G2(BMc, BNc, (g2::kGeluB | g2::kGeluBS), false); break;  \
        case g2::kBst: HIPPS_G2(BMc, BNc, g2::kBst, false); break;                                  \
        case g2::kBst | g2::kAdd: HIPPS_G2(BMc, BNc, (g2::kBst | g2::kAdd), false); break;          \
        case g2::kBstBits: HIPPS_G2(BMc, BNc, g2::kBstBits, false); break;                          \
        case g2::kBstBits | g2::kAdd: HIPPS_G2(BMc, BNc, (g2::kBstBits | g2::kAdd), false); break;  \
        case g2::kAdd | g2::kAddS2: HIPPS_G2(BMc, BNc, (g2::kAdd | g2::kAddS2), false); break;      \
        case g2::kBst | g2::kAdd | g2::kAddS2:                                                        \
          HIPPS_G2(BMc, BNc, (g2::kBst | g2::kAdd | g2::kAddS2), false); break;                      \
        case g2::kBstBits | g2::kAdd | g2::kAddS2:                                                    \
          HIPPS_G2(BMc, BNc, (g2::kBstBits | g2::kAdd | g2::kAddS2), false); break;                  \
        default: HIPPS_G2(BMc, BNc, g2::kPlain, false); break;                                      \
      }                                                                                             \
    }                                                                                               \
  } while (0)
  // 3 stages where they fit the LDS (not 256x256: 3 x 64 KB)
  const bool NS3 = stages == 3, NS4 = stages == 4;  // 4: k-half units (see k_gemm)
  const bool NS5 = stages == 5;                      // 5: ping-pong wave groups (256x256 only)
  const bool NS6 = stages == 6;                      // 6: 32x32x16 MFMA (256x256 only)
  TORCH_CHECK(!NS3 || !(BMv == 256 && BNv == 256), "gemm2: 3 stages do not fit a 256x256 tile");
  TORCH_CHECK(!NS5 || (BMv == 256 && BNv == 256), "gemm2: the ping-pong schedule (stages 5) is a 256x256 tile");
  TORCH_CHECK(!NS6 || (BMv == 256 && BNv == 256), "gemm2: the 32x32x16 MFMA loop (stages 6) is a 256x256 tile");
#define NS3_OF(BMc, BNc) ((BMc) == 256 && (BNc) == 256 ? 2 : 3)
#define NS5_OF(BMc, BNc) ((BMc) == 256 && (BNc) == 256 ? 5 : 2)
#define NS6_OF(BMc, BNc) ((BMc) == 256 && (BNc) == 256 ? 6 : 2)
  if (BMv == 256 && BNv == 256) HIPPS_G2_E(256, 256);
  else if (BMv == 256 && BNv == 128) HIPPS_G2_E(256, 128);
  else if (BMv == 128 && BNv == 128) HIPPS_G2_E(128, 128);
  else if (BMv == 256 && BNv == 64) HIPPS_G2_E(256, 64);
  else if (BMv == 128 && BNv == 64) HIPPS_G2_E(128, 64);
  else TORCH_CHECK(false, "gemm2: unsupported block tile ", BMv, "x", BNv);
#undef HIPPS_G2_E
#undef HIPPS_G2
#undef HIPPS_G2S
#undef NS3_OF
#undef NS5_OF
#undef NS6_OF
}

// Input gradient of a stride-2 3x3 / pad-1 convolution as four output-parity classes (kPar): dx
// positions (2a+ph, 2b+pw) take 1, 2, 2 and 4 taps of dy (the taps whose stride-2 footprint hits
// them), each class one implicit GEMM writing its rows of dx -- every dx element written exactly
// once, no zero fill, no scatter.  dy [img, Cout, Hd, Wd], wf = rot180(W)^T [Cin, Cout, 3, 3]
// (channels-last, i.e. [Cin][3][3][Cout]), dx [img, Cin, Hx, Wx].  With bn_x: the backward
// reduction of the BN whose output gradient dx is (epilogue kBst / kBstBits), all four classes'
// partials in one [2, Cin, sum of m tiles] array, returned.
at::Tensor gemm2_dgrad_s2(at::Tensor dy, at::Tensor wf, at::Tensor dx, int64_t bm, int64_t bn,
                          c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_bits,
                          c10::optional<at::Tensor> bn_mean, c10::optional<at::Tensor> bn_invstd,
                          c10::optional<at::Tensor> bn_scale, c10::optional<at::Tensor> bn_shift) {
  TORCH_CHECK(dy.is_cuda() && wf.is_cuda() && dx.is_cuda(), "gemm2_dgrad_s2: device tensors");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && wf.scalar_type() == at::kBFloat16 && dx.scalar_type() == at::kBFloat16,
              "gemm2_dgrad_s2: bf16 tensors");
  TORCH_CHECK(dy.dim() == 4 && dx.dim() == 4 && wf.dim() == 4 && wf.size(2) == 3 && wf.size(3) == 3,
              "gemm2_dgrad_s2: 4-d tensors, 3x3 weight");
  const int64_t imgs = dy.size(0), Cout = dy.size(1), Hd = dy.size(2), Wd = dy.size(3);
  const int64_t Cin = dx.size(1), Hx = dx.size(2), Wx = dx.size(3);
  TORCH_CHECK(dx.size(0) == imgs && wf.size(0) == Cin && wf.size(1) == Cout, "gemm2_dgrad_s2: shapes");
  TORCH_CHECK((Hx - 1) / 2 + 1 == Hd && (Wx - 1) / 2 + 1 == Wd, "gemm2_dgrad_s2: dy must be the stride-2 / pad-1 output");
  TORCH_CHECK(Cout % 64 == 0 && Cin % 64 == 0, "gemm2_dgrad_s2: Cin % 64 == 0, Cout % 64 == 0");
  TORCH_CHECK(dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dx.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  wf.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2_dgrad_s2: channels-last tensors");
  for (const at::Tensor* t : {&dy, &wf, &dx})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm2_dgrad_s2: 16-byte aligned tensors");
  TORCH_CHECK(dx.numel() < (int64_t(1) << 31) && dy.numel() < (int64_t(1) << 31), "gemm2_dgrad_s2: size");
  const int BMv = (int)bm, BNv = (int)bn;
  TORCH_CHECK(Cin % BNv == 0, "gemm2_dgrad_s2: Cin must be a multiple of the block tile");
  // classes: (ph, pw) -> rows Ma x Mb of dx positions, taps (dy offset, rot180 tap index)
  int64_t Mc[4], mt[4], tot = 0;
  for (int c = 0; c < 4; ++c) {
    const int ph = c >> 1, pw = c & 1;
    Mc[c] = imgs * ((Hx - ph + 1) / 2) * ((Wx - pw + 1) / 2);
    mt[c] = (Mc[c] + BMv - 1) / BMv;
    tot += mt[c];
  }
  const bool bst = bn_x.has_value() && bn_x->defined();
  at::Tensor part;
  int epi = g2::kPar;
  g2::Args a{};
  if (bst) {
    TORCH_CHECK(bn_x->is_cuda() && bn_x->scalar_type() == at::kBFloat16 && bn_x->numel() == dx.numel() &&
                    bn_x->is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2_dgrad_s2: bn_x shaped like dx");
    for (const c10::optional<at::Tensor>* v : {&bn_mean, &bn_invstd, &bn_scale, &bn_shift})
      TORCH_CHECK(v->has_value() && (*v)->defined() && (*v)->is_cuda() && (*v)->scalar_type() == at::kFloat &&
                      (*v)->is_contiguous() && (*v)->numel() == Cin, "gemm2_dgrad_s2: BN vectors must be f32 [Cin]");
    part = at::empty({2, Cin, tot}, dy.options().dtype(at::kFloat));
    a.pa = part.data_ptr<float>();
    a.pb = a.pa + Cin * tot;
    a.bx = (const uint16_t*)bn_x->data_ptr();
    a.bmean = bn_mean->data_ptr<float>();
    a.binvstd = bn_invstd->data_ptr<float>();
    a.bscale = bn_scale->data_ptr<float>();
    a.bshift = bn_shift->data_ptr<float>();
    if (bn_bits.has_value() && bn_bits->defined()) {
      TORCH_CHECK(bn_bits->is_cuda() && bn_bits->scalar_type() == at::kByte && bn_bits->numel() == dx.numel() / 8,
                  "gemm2_dgrad_s2: bn_bits uint8[numel(dx)/8]");
      a.bbits = (const uint8_t*)bn_bits->data_ptr();
      epi |= g2::kBstBits;
    } else {
      epi |= g2::kBst;
    }
  }
  a.X = (const uint16_t*)dy.data_ptr();
  a.W = (const uint16_t*)wf.data_ptr();
  a.Y = (uint16_t*)dx.data_ptr();
  a.N = (int)Cin;
  a.Hi = (int)Hd; a.Wi = (int)Wd; a.Cin = (int)Cout;
  a.stride = 1; a.KW = 3; a.pad = 0;
  a.ldb = (int)(9 * Cout);
  a.Hx = (int)Hx; a.Wx = (int)Wx;
  a.pstride = (int)tot;
  a.ntiles = (int)(Cin / BNv);
  auto stream = c10::hip::getCurrentHIPStream();
  int64_t col = 0;
  for (int c = 0; c < 4; ++c) {
    const int ph = c >> 1, pw = c & 1;
    // dx row 2a+ph takes dy row a + (ph + 1 - kr) / 2 for the kr of its parity
    const int nkr = ph ? 2 : 1, nkc = pw ? 2 : 1;
    int nt = 0;
    for (int i = 0; i < nkr; ++i)
      for (int j = 0; j < nkc; ++j) {
        const int kr = ph ? 2 * i : 1, kc = pw ? 2 * j : 1;
        a.tdr[nt] = (ph + 1 - kr) / 2;
        a.tdc[nt] = (pw + 1 - kc) / 2;
        a.tko[nt] = (2 - kr) * 3 + (2 - kc);  // rot180: wf tap (2-kr, 2-kc) holds W[.., kr, kc]
        ++nt;
      }
    a.ph = ph; a.pw = pw;
    a.Ho = (int)((Hx - ph + 1) / 2); a.Wo = (int)((Wx - pw + 1) / 2);
    a.M = (int)Mc[c];
    a.K = (int)(nt * Cout);
    a.mtiles = (int)mt[c];
    a.pcol0 = (int)col;
    col += mt[c];
    const int grid = (int)(mt[c] * a.ntiles);
    if (grid == 0) continue;
#define HIPPS_G2P(BMc, BNc)                                                                                          \
  do {                                                                                                             \
    if (epi == (g2::kPar | g2::kBst))                                                                              \
      hipLaunchKernelGGL((g2::k_gemm<BMc, BNc, g2::kPar | g2::kBst, true, 2>), grid, (g2::nthreads<BMc, BNc>()), 0, \
                         stream, a);                                                                               \
    else if (epi == (g2::kPar | g2::kBstBits))                                                                     \
      hipLaunchKernelGGL((g2::k_gemm<BMc, BNc, g2::kPar | g2::kBstBits, true, 2>), grid, (g2::nthreads<BMc, BNc>()), \
                         0, stream, a);                                                                            \
    else                                                                                                           \
      hipLaunchKernelGGL((g2::k_gemm<BMc, BNc, g2::kPar, true, 2>), grid, (g2::nthreads<BMc, BNc>()), 0, stream, a); \
  } while (0)
    if (BMv == 256 && BNv == 256) HIPPS_G2P(256, 256);
    else if (BMv == 128 && BNv == 128) HIPPS_G2P(128, 128);
    else if (BMv == 128 && BNv == 64) HIPPS_G2P(128, 64);
    else if (BMv == 256 && BNv == 64) HIPPS_G2P(256, 64);
    else TORCH_CHECK(false, "gemm2_dgrad_s2: unsupported block tile ", BMv, "x", BNv);
#undef HIPPS_G2P
  }
  return part;
}

void wgrad_reduce_slabs(const at::Tensor& part, int64_t S, int64_t N, int64_t K, at::Tensor& dw,
                        hipStream_t stream0);
int64_t wgrad_reduce_groups(int64_t S, int64_t N, int64_t K);

// Arrival tickets of the in-launch weight-gradient reduction: a zeroed per-device ring, handed out
// in consecutive ranges (one counter per output tile); the reducer of a tile re-arms its counter, so
// the ring is never cleared again.  Launches in flight at once never share counters unless 64K
// tiles' worth of launches are queued between them.
static int* wgrad_tickets(const at::Tensor& like, int64_t n) {
  constexpr int64_t kRing = 1 << 16;
  static std::mutex mu;
  static at::Tensor ring[64];
  static int64_t cur[64];
  const int dev = like.get_device();
  TORCH_CHECK(dev >= 0 && dev < 64 && n <= kRing / 4, "wgrad tickets");
  std::lock_guard<std::mutex> lock(mu);
  if (!ring[dev].defined()) ring[dev] = at::zeros({kRing}, like.options().dtype(at::kInt));
  if (cur[dev] + n > kRing) cur[dev] = 0;
  int* p = ring[dev].data_ptr<int>() + cur[dev];
  cur[dev] += n;
  return p;
}

// Opt-in (HIPPS_WGRAD_FUSED_REDUCE=1): bit-identical, 76 fewer launches per ResNet-50 step, but
// measured 1.5 % slower in the step (same-box A/B 11554 / 11544 on vs 11762 / 11705 img/s off,
// profiles/r4/ab_r4b.txt): the serial slab reads of each tile's last block lengthen the weight-
// gradient kernels on the side stream more than the separate, chip-wide reduce costs there.
static bool wgrad_fused_reduce() {
  static const bool on = [] {
    const char* e = std::getenv("HIPPS_WGRAD_FUSED_REDUCE");
    return e && e[0] == '1';
  }();
  return on;
}

// Weight gradient on the LDS-DMA core: dy [img, Cout, Ho, Wo] and x [img, Cin, Hi, Wi] channels-last
// bf16; dw f32 [Cout, KH, KW, Cin] in memory (the channels-last weight layout; 1x1: [Cout, Cin]).
// Cout % 64 == 0, Cin % 64 == 0.  S split-M partial slabs (~2 resident blocks per CU) + fixed-order sum.
void gemm2_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                 int64_t Hi, int64_t Wi, int64_t cfg, int64_t stages, c10::optional<at::Tensor> pro_scale,
                 c10::optional<at::Tensor> pro_shift, int64_t sdiv) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dw.is_cuda(), "gemm2_wgrad: device tensors");
  const bool pro = pro_scale.has_value() && pro_scale->defined();
  TORCH_CHECK(!pro || stages == 2, "gemm2_wgrad: the BN prologue runs with 2 stages");
  TORCH_CHECK(stages == 2 || stages == 4 || (stages == 3 && cfg != 2),
              "gemm2_wgrad: stages 2, 4 (k-half units), or 3 below the 256x256 tile");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16 && dw.scalar_type() == at::kFloat,
              "gemm2_wgrad: bf16 dy/x, f32 dw");
  TORCH_CHECK(dw.is_contiguous() || dw.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2_wgrad: dense dw");
  const int64_t N = dw.size(0), K = dw.numel() / N, Cin = K / (KH * KW);
  TORCH_CHECK(Cin * KH * KW == K && N % 64 == 0 && Cin % 64 == 0, "gemm2_wgrad: Cout % 64 == 0, Cin % 64 == 0");
  const int64_t imgs = x.numel() / (Cin * Hi * Wi);
  TORCH_CHECK(imgs * Cin * Hi * Wi == x.numel(), "gemm2_wgrad: x size");
  const int64_t Ho = (Hi + 2 * pad - KH) / stride + 1, Wo = (Wi + 2 * pad - KW) / stride + 1;
  const int64_t M = imgs * Ho * Wo;
  TORCH_CHECK(dy.numel() == M * N, "gemm2_wgrad: dy size");
  TORCH_CHECK(x.dim() != 4 || x.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2_wgrad: channels-last x");
  TORCH_CHECK(dy.dim() != 4 || dy.is_contiguous(at::MemoryFormat::ChannelsLast), "gemm2_wgrad: channels-last dy");
  for (const at::Tensor* t : {&x, &dy, &dw})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm2_wgrad: 16-byte aligned tensors");
  TORCH_CHECK(M < (int64_t(1) << 31) && x.numel() < (int64_t(1) << 40), "gemm2_wgrad: size");
  // cfg 0: 128|64 x 128|64 tile on 4 waves (64x64 each: the first core's tiling and slab split);
  // 1: 256 x 128 on 4 waves of 128x64; 2: 256 x 256 on 8 waves of 128x64 (a third of the LDS
  // bytes per MFMA of cfg 0: the transposing-read wgrad is LDS-bandwidth bound)
  // 3: 128 x 256 and 4: 256 x 128 on 8 waves of 64x64 (more MFMA work per staged byte than cfg 0
  // at two waves per SIMD; 3 stages fit)
  int TN = N % 128 == 0 ? 128 : 64, TK = Cin % 128 == 0 ? 128 : 64;
  if (cfg == 1) {
    TORCH_CHECK(N % 256 == 0 && Cin % 128 == 0, "gemm2_wgrad cfg 1 needs Cout % 256, Cin % 128");
    TN = 256; TK = 128;
  } else if (cfg == 2) {
    TORCH_CHECK(N % 256 == 0 && Cin % 256 == 0, "gemm2_wgrad cfg 2 needs Cout % 256, Cin % 256");
    TN = 256; TK = 256;
  } else if (cfg == 3) {
    TORCH_CHECK(N % 128 == 0 && Cin % 256 == 0, "gemm2_wgrad cfg 3 needs Cout % 128, Cin % 256");
    TN = 128; TK = 256;
  } else if (cfg == 4) {
    TORCH_CHECK(N % 256 == 0 && Cin % 128 == 0, "gemm2_wgrad cfg 4 needs Cout % 256, Cin % 128");
    TN = 256; TK = 128;
  }
  // 5 / 6: multi-tap TN x 128 tiles for Cin == 64 KxK layers (2 taps per tile, K padded to a
  // multiple of 128): 5 on 2 waves of TNx64, 6 on 4 waves of TNx32
  const bool mt = cfg == 5 || cfg == 6;
  if (mt) {
    TORCH_CHECK(Cin == 64 && KH * KW > 1, "gemm2_wgrad cfg 5/6: 64-channel KxK layers");
    TN = N % 128 == 0 && cfg == 6 ? 128 : 64;
    TK = 128;
  }
  TORCH_CHECK(cfg >= 0 && cfg <= 6, "gemm2_wgrad: cfg 0..6");
  const int64_t tn = N / TN, tk = (K + TK - 1) / TK, tiles = tn * tk;
  TORCH_CHECK(mt || tk * TK == K, "gemm2_wgrad: K tile");
  int64_t resident = 256 * (cfg ? 1 : TN * TK == 128 * 128 ? 2 : TN * TK == 128 * 64 ? 3 : 5);
  if (cfg >= 3) resident = 256;
  if (stages == 3 || mt)  // (stages 4 = the LDS bytes of 2)
    resident = 256 * std::max<int64_t>(1, 160 * 1024 / ((stages == 4 ? 2 : stages) * g2::kWM * (TN + TK) * 2));
  // sdiv > 1: fewer, longer M slabs (less fp32 slab traffic, fewer resident blocks)
  TORCH_CHECK(sdiv >= 1, "gemm2_wgrad: sdiv >= 1");
  int64_t S = std::max<int64_t>(1, resident / tiles / sdiv);
  S = std::min<int64_t>(S, std::max<int64_t>(1, M / (8 * g2::kWM)));           // >= 8 stages per block
  S = std::min<int64_t>(S, std::max<int64_t>(1, M * (N + K) / (4 * N * K)));  // slabs <= operand bytes
  const int64_t chunk = ((M + S - 1) / S + g2::kWM - 1) / g2::kWM * g2::kWM;
  S = (M + chunk - 1) / chunk;
  TORCH_CHECK(S * tiles < (int64_t(1) << 31), "gemm2_wgrad: grid");
  auto stream = c10::hip::getCurrentHIPStream();
  at::Tensor part = S == 1 ? dw : at::empty({S, N, K}, dw.options());
  g2::WArgs a{};
  a.dY = (const uint16_t*)dy.data_ptr();
  a.X = (const uint16_t*)x.data_ptr();
  a.part = part.data_ptr<float>();
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.Cin = (int)Cin; a.Ho = (int)Ho; a.Wo = (int)Wo; a.Hi = (int)Hi;
  a.Wi = (int)Wi; a.stride = (int)stride; a.KW = (int)KW; a.pad = (int)pad; a.chunk = (int)chunk;
  a.tn = (int)tn; a.tk = (int)tk;
  a.fd_hw = g2::make_fastdiv2((uint32_t)(Ho * Wo));
  a.fd_w = g2::make_fastdiv2((uint32_t)Wo);
  if (pro) {
    for (const c10::optional<at::Tensor>* v : {&pro_scale, &pro_shift})
      TORCH_CHECK(v->has_value() && (*v)->defined() && (*v)->is_cuda() && (*v)->scalar_type() == at::kFloat &&
                      (*v)->is_contiguous() && (*v)->numel() == Cin, "gemm2_wgrad: prologue scale / shift f32 [Cin]");
    a.psc = pro_scale->data_ptr<float>();
    a.psh = pro_shift->data_ptr<float>();
  }
  const bool fused = S > 1 && wgrad_fused_reduce();
  if (fused) {  // the last block of each tile sums its S slabs in the launch (no reduce kernels)
    a.cnt = wgrad_tickets(dw, tiles);
    a.S = (int)S;
    a.G = (int)wgrad_reduce_groups(S, N, K);
    a.dw = dw.data_ptr<float>();
  }
  const int grid = (int)(S * tiles);
#define HIPPS_W2M(TNc, TKc, WNc, WKc, MTc)                                                                         \
  do {                                                                                                            \
    if (pro) hipLaunchKernelGGL((g2::k_wgrad<TNc, TKc, WNc, WKc, 2, MTc, true>), grid, 64 * WNc * WKc, 0, stream, a); \
    else if (stages == 3) hipLaunchKernelGGL((g2::k_wgrad<TNc, TKc, WNc, WKc, 3, MTc>), grid, 64 * WNc * WKc, 0, stream, a); \
    else if (stages == 4) hipLaunchKernelGGL((g2::k_wgrad<TNc, TKc, WNc, WKc, 4, MTc>), grid, 64 * WNc * WKc, 0, stream, a); \
    else hipLaunchKernelGGL((g2::k_wgrad<TNc, TKc, WNc, WKc, 2, MTc>), grid, 64 * WNc * WKc, 0, stream, a);            \
  } while (0)
#define HIPPS_W2(TNc, TKc, WNc, WKc) HIPPS_W2M(TNc, TKc, WNc, WKc, false)
  if (cfg == 2 && pro) hipLaunchKernelGGL((g2::k_wgrad<256, 256, 2, 4, 2, false, true>), grid, 512, 0, stream, a);
  else if (cfg == 2 && stages == 4) hipLaunchKernelGGL((g2::k_wgrad<256, 256, 2, 4, 4>), grid, 512, 0, stream, a);
  else if (cfg == 2) hipLaunchKernelGGL((g2::k_wgrad<256, 256, 2, 4, 2>), grid, 512, 0, stream, a);
  else if (cfg == 5) HIPPS_W2M(64, 128, 1, 2, true);
  else if (cfg == 6 && TN == 128) HIPPS_W2M(128, 128, 2, 2, true);
  else if (cfg == 6) HIPPS_W2M(64, 128, 1, 4, true);
  else if (cfg == 3) HIPPS_W2(128, 256, 2, 4);
  else if (cfg == 4) HIPPS_W2(256, 128, 4, 2);
  else if (cfg == 1) HIPPS_W2(256, 128, 2, 2);
  else if (TN == 128 && TK == 128) HIPPS_W2(128, 128, 2, 2);
  else if (TN == 128) HIPPS_W2(128, 64, 2, 2);
  else if (TK == 128) HIPPS_W2(64, 128, 2, 2);
  else HIPPS_W2(64, 64, 2, 2);
#undef HIPPS_W2
#undef HIPPS_W2M
  if (S > 1 && !fused) {
    at::Tensor dwv = dw;
    wgrad_reduce_slabs(part, S, N, K, dwv, stream);
  }
}

}  // namespace hipps
