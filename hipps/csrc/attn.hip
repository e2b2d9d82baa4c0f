// hipps — flash attention on the CDNA4 matrix cores (gfx950): forward, and a deterministic
// backward (dQ and dK/dV in separate kernels, no float atomics), for the transformer configs
// (BASELINE.json configs 4/5: BERT-base head dim 64, Llama-3 head dim 128 with causal masking
// and grouped-query heads).  Replaces PyTorch SDPA, whose ROCm route runs aotriton's
// Triton-generated kernels on the hot path.
//
// Layout: q [B, Sq, Hq, D], k / v [B, Sk, Hkv, D] with any batch / sequence / head strides (d
// contiguous, 16-byte rows) -- the [B, S, H*D] projection outputs viewed per head, so no
// transpose pass runs before or after; o / dq / dk / dv come out contiguous in the same layout.
//
// MFMA: v_mfma_f32_32x32x16_bf16 throughout (cdna_hip_programming.md §3 operand maps: lane l holds
// A[row l&31][k 8(l>>5)+j] and B[k 8(l>>5)+j][col l&31]; C[row (r&3)+8(r>>2)+4(l>>5)][col l&31]).
//
//   forward / dQ (a workgroup = 4 waves x 32 query rows of one (batch, head); K/V tiles of 64
//   keys double-buffered in LDS by LDS-DMA):
//     S^T = K Q^T        key in the accumulator rows, the query on the lane: the softmax row
//                        max / sum is lane-local (+ one exchange with lane l^32), and the
//                        rescale of the output accumulator by exp(m_old - m_new) too;
//     O^T += V^T P^T     P^T's accumulator registers are the B operand as they stand (k order
//                        permuted: element j of lane half h at k-step s is key 16s + 8(j>>2) +
//                        4h + (j&3), §3 'An accumulator tile as the next MFMA's operand'), and
//                        V^T's A operand comes from ds_read_b64_tr_b16 (T10) on the row-major V
//                        tile at exactly those keys.
//   dQ:  dP^T = V dO^T (accumulator initialised to -delta),  dS^T = P^T (dP^T - delta),
//        dQ^T += K^T dS^T  (K^T by transposed reads of the same K tile the S^T product row-reads).
//   dK/dV (a workgroup = 4 waves x 32 keys of one (batch, kv head); the wave's K and V rows stay
//   in registers while Q / dO tiles of 64 queries stream through LDS, over every query head of
//   the GQA group -- dK / dV need no cross-workgroup sum unless the group is split for occupancy):
//     S = Q K^T (accumulator initialised to -lse per query row, so p = exp2(c * acc)),
//     dP = dO V^T (initialised to -delta), dV^T += dO^T P, dK^T += Q^T dS.
//
// LDS images: every tile is [rows][D] bf16 with the 16-byte chunk c of row r stored at chunk
// c ^ f(r) -- one image serves the ds_read_b128 row reads (operand rows on the lanes) and the
// ds_read_b64_tr_b16 transposed reads conflict-free (T10 'One image for row reads AND transposed
// reads'; f for 128-byte rows derived the same way for D = 64).  The DMA writes each
// wave-instruction's 1 KB lane-linearly; the swizzle is applied on the global source address.
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {
namespace attn {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef __attribute__((address_space(1))) void glb_void;

// 16-byte zero source for rows outside the sequence (global memory, read-only)
__device__ __attribute__((aligned(64))) const uint16_t kZero[32] = {0};

constexpr float kLog2e = 1.4426950408889634f;
constexpr int KT = 64;   // rows per streamed tile (keys in forward / dQ, queries in dK/dV)
constexpr int NW = 4;    // waves per workgroup
constexpr int QB = 128;  // query rows (forward / dQ) or keys (dK/dV) per workgroup

struct Args {
  const uint16_t *q, *k, *v, *o, *dout;
  uint16_t *out, *dq, *dk, *dv;
  float* lse;       // [B, Hq, Sq] natural-log row log-sum-exp (forward writes it, backward reads it)
  float* rowstat;   // backward: per (b, hq, 64-row tile) {-lse*log2e/c [64], -delta [64]}
  float* part;      // dK/dV with a split GQA group: fp32 [gsplit][2][B, Sk, Hkv, D]
  const int* kvlen; // [B] valid keys per batch row (key padding), or null
  int64_t qsb, ksb, vsb, osb, dosb;       // batch strides (elements)
  int64_t qss, qsh, kss, ksh, vss, vsh;   // sequence / head strides
  int64_t oss, osh, doss, dosh;
  int64_t gqb, gqs, gqh, gkb, gks, gkh;  // dq / (dk, dv) output strides (packed QKV gradients)
  int B, Hq, Hkv, Sq, Sk;
  float scale;
  int nblk;    // query blocks (forward / dQ) or key blocks (dK/dV) of QB rows
  int nqblk;   // query blocks (the rowstat tiles per (b, hq) are 2 * nqblk)
  int gsplit;  // dK/dV: slices of the GQA group (1 = write bf16 dK / dV directly)
};

template <int D> __device__ __forceinline__ int swz(int row) {
  return D == 128 ? (((row & 3) << 2) | ((row >> 2) & 3)) : ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
}
// byte offset of 16-byte chunk c of row r in a [rows][D] tile image
template <int D> __device__ __forceinline__ int toff(int row, int c) { return row * (2 * D) + ((c ^ swz<D>(row)) << 4); }

__device__ __forceinline__ void glds16(const void* src, void* dst) {
  __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)dst, 16, 0, 0);
}

// DMA rows [row0, row0 + KT) of a [rows, D] bf16 matrix (row stride rs elements; rows >= nrows
// read the zero page) into a tile image
template <int D>
__device__ __forceinline__ void stage_tile(char* tile, const uint16_t* base, int64_t rs, int row0, int nrows, int w,
                                           int lane) {
  constexpr int CPR = D / 8;                // 16-byte chunks per row
  constexpr int RPI = 64 / CPR;             // rows per wave-instruction (1 KB)
  constexpr int N = KT * CPR / (64 * NW);   // wave-instructions per wave
  const int lr = lane / CPR, slot = lane % CPR;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int r = (i * NW + w) * RPI + lr;
    const int g = row0 + r;
    const uint16_t* src = g < nrows ? base + (int64_t)g * rs + ((slot ^ swz<D>(r)) << 3) : kZero;
    glds16(src, tile + (i * NW + w) * RPI * 2 * D);
  }
}

// A / B operand of a 32x32x16 MFMA whose rows (on the lanes) are tile rows rb .. rb+31: chunk 2dk+h
template <int D> __device__ __forceinline__ bf16x8 row_frag(const char* tile, int rb, int dk, int lane) {
  return *reinterpret_cast<const bf16x8*>(tile + toff<D>(rb + (lane & 31), 2 * dk + (lane >> 5)));
}

// A operand whose rows are the tile's COLUMNS d = 32db + (l&31) and whose k index runs over tile
// rows in the permuted accumulator order: element j of lane half h = tile row rb + 8(j>>2) + 4h +
// (j&3) -- two ds_read_b64_tr_b16, each a 4-row x 16-column block per 16-lane group
template <int D> __device__ __forceinline__ bf16x8 tr_frag(const char* tile, int rb, int db, int lane) {
  const int h = lane >> 5, q = (lane >> 2) & 3, p = lane & 3, g1 = (lane >> 4) & 1;
  const int c = 4 * db + 2 * g1 + (p >> 1);
  const int r0 = rb + 4 * h + q;
  const char* a0 = tile + toff<D>(r0, c) + 8 * (p & 1);
  const char* a1 = tile + toff<D>(r0 + 8, c) + 8 * (p & 1);
  const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a1));
  return bf16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

__device__ __forceinline__ bf16x8 pack8(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t u = pack_bf16x2(a[8 * s + 2 * j], a[8 * s + 2 * j + 1]);
    r[2 * j] = (short)(u & 0xffff);
    r[2 * j + 1] = (short)(u >> 16);
  }
  return r;
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// lane l and lane l ^ 32 hold the two halves of one query row: combine them with
// v_permlane32_swap (a VALU lane swap) instead of a ds_bpermute round trip through the LDS unit
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

// vmcnt-only s_waitcnt immediate (gfx9 encoding; expcnt / lgkmcnt at their maxima)
constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
// LDS-DMA instructions per wave for one KT-row tile
template <int D> constexpr int tile_glds() { return KT * (D / 8) / (64 * NW); }

// NS: LDS stages of the streamed tiles.  2: the DMA of tile it+1 is issued after the barrier of
// tile it and drained before the next barrier -- one tile's compute (~1 us at D = 64) to cover
// the HBM latency.  3: tile it+2 is issued instead and each wait leaves the younger tile in
// flight (cdna_hip_programming.md 'Pipelining across barriers').
template <int NS> __device__ __forceinline__ void wait_tile(bool younger, int n_younger) {
  if (NS == 3 && younger) {
    // n_younger is one of two wave-uniform counts (the rowstat DMA of wave 0): immediates only
    if (n_younger == 5) __builtin_amdgcn_s_waitcnt(waitcnt_vm(5));
    else if (n_younger == 4) __builtin_amdgcn_s_waitcnt(waitcnt_vm(4));
    else if (n_younger == 9) __builtin_amdgcn_s_waitcnt(waitcnt_vm(9));
    else if (n_younger == 8) __builtin_amdgcn_s_waitcnt(waitcnt_vm(8));
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// row of accumulator register r for lane half h (32x32 C layout)
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// 4 consecutive d values (one accumulator register group) as 8 bytes of bf16
__device__ __forceinline__ void store4(uint16_t* p, float a, float b, float c, float d) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf16x2(a, b), pack_bf16x2(c, d));
}

// ------------------------------------------------------------------------------------ forward
template <int D, bool CAUSAL, int NS = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_attn_fwd(Args a) {
  constexpr int DK = D / 16, DB = D / 32, TILE = KT * 2 * D;
  __shared__ __attribute__((aligned(16))) char lds[NS][2 * TILE];
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int h = lane >> 5;
  const int nbh = a.B * a.Hq, bid = blockIdx.x;
  const int qblk = CAUSAL ? a.nblk - 1 - bid / nbh : bid / nbh;  // causal: heaviest blocks first
  const int bh = bid % nbh, b = bh / a.Hq, hq = bh - b * a.Hq, hk = hq / (a.Hq / a.Hkv);
  const int q0 = qblk * QB, qw0 = q0 + 32 * w, qrow = qw0 + (lane & 31);
  int kv_end = a.Sk;
  if (a.kvlen != nullptr) kv_end = min(kv_end, a.kvlen[b]);
  const int kv_stop = CAUSAL ? min(kv_end, q0 + QB) : kv_end;
  const int ntile = (kv_stop + KT - 1) / KT;
  const uint16_t* kb = a.k + b * a.ksb + hk * a.ksh;
  const uint16_t* vb = a.v + b * a.vsb + hk * a.vsh;
  const uint16_t* qp = a.q + b * a.qsb + hq * a.qsh + (int64_t)min(qrow, a.Sq - 1) * a.qss + 8 * h;
  bf16x8 qf[DK];
#pragma unroll
  for (int dk = 0; dk < DK; ++dk) qf[dk] = *reinterpret_cast<const bf16x8*>(qp + 16 * dk);
  f32x16 o[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m = -INFINITY, lsum = 0.f;
  const float c = a.scale * kLog2e;
  for (int p = 0; p < NS - 1 && p < ntile; ++p) {
    stage_tile<D>(lds[p], kb, a.kss, p * KT, kv_end, w, lane);
    stage_tile<D>(lds[p] + TILE, vb, a.vss, p * KT, kv_end, w, lane);
  }
  for (int it = 0; it < ntile; ++it) {
    wait_tile<NS>(it + 1 < ntile, 2 * tile_glds<D>());
    __syncthreads();  // tile it landed for every wave; the slot of tile it-1 is free
    if (it + NS - 1 < ntile) {
      char* nb = lds[(it + NS - 1) % NS];
      stage_tile<D>(nb, kb, a.kss, (it + NS - 1) * KT, kv_end, w, lane);
      stage_tile<D>(nb + TILE, vb, a.vss, (it + NS - 1) * KT, kv_end, w, lane);
    }
    const int k0 = it * KT;
    if (CAUSAL && k0 > qw0 + 31) continue;  // (wave-uniform) every key above this wave's rows
    const char* Kt = lds[it % NS];
    const char* Vt = Kt + TILE;
    f32x16 s[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kk][r] = 0.f;
#pragma unroll
      for (int dk = 0; dk < DK; ++dk) s[kk] = MFMA32(row_frag<D>(Kt, 32 * kk, dk, lane), qf[dk], s[kk]);
    }
    if (k0 + KT > kv_end || (CAUSAL && k0 + KT - 1 > qw0)) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * kk + crow(r, h);
          if (key >= kv_end || (CAUSAL && key > qrow)) s[kk][r] = -INFINITY;
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kk][r]);
    mx = half_max(mx);
    const float mn = fmaxf(m, mx * c);
    const float mu = mn == -INFINITY ? 0.f : mn;
    const float alpha = fast_exp2(m - mu);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fast_exp2(fmaf(s[kk][r], c, -mu));
        s[kk][r] = p;
        ps += p;
      }
    lsum = lsum * alpha + ps;
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {  // (the max moved for some row)
#pragma unroll
      for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(s[kk], s2);
#pragma unroll
        for (int db = 0; db < DB; ++db) o[db] = MFMA32(tr_frag<D>(Vt, 32 * kk + 16 * s2, db, lane), pf, o[db]);
      }
  }
  const float lt = half_sum(lsum);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (qrow < a.Sq) {
    uint16_t* op = a.out + b * a.osb + hq * a.osh + (int64_t)qrow * a.oss;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(op + 32 * db + 8 * g + 4 * h, o[db][4 * g] * inv, o[db][4 * g + 1] * inv, o[db][4 * g + 2] * inv,
               o[db][4 * g + 3] * inv);
    if (h == 0) a.lse[((int64_t)b * a.Hq + hq) * a.Sq + qrow] = lt > 0.f ? (m + __log2f(lt)) * 0.69314718055994531f : INFINITY;
  }
}

// ------------------------------------------------------------------------------- backward: dQ
// Also computes delta = rowsum(dO * O) and publishes the per-row constants the dK/dV kernel
// initialises its accumulators with (rowstat), so no separate preprocess pass reads dO and O.
template <int D, bool CAUSAL, int NS>
__device__ __forceinline__ void attn_dq_body(const Args& a) {
  constexpr int DK = D / 16, DB = D / 32, TILE = KT * 2 * D;
  __shared__ __attribute__((aligned(16))) char lds[NS][2 * TILE];
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int h = lane >> 5;
  const int nbh = a.B * a.Hq, bid = blockIdx.x;
  const int qblk = CAUSAL ? a.nblk - 1 - bid / nbh : bid / nbh;
  const int bh = bid % nbh, b = bh / a.Hq, hq = bh - b * a.Hq, hk = hq / (a.Hq / a.Hkv);
  const int q0 = qblk * QB, qw0 = q0 + 32 * w, qrow = qw0 + (lane & 31);
  int kv_end = a.Sk;
  if (a.kvlen != nullptr) kv_end = min(kv_end, a.kvlen[b]);
  const int kv_stop = CAUSAL ? min(kv_end, q0 + QB) : kv_end;
  const int ntile = (kv_stop + KT - 1) / KT;
  const uint16_t* kb = a.k + b * a.ksb + hk * a.ksh;
  const uint16_t* vb = a.v + b * a.vsb + hk * a.vsh;
  const bool qok = qrow < a.Sq;
  const int qr = min(qrow, a.Sq - 1);
  const uint16_t* qp = a.q + b * a.qsb + hq * a.qsh + (int64_t)qr * a.qss + 8 * h;
  const uint16_t* dp_ = a.dout + b * a.dosb + hq * a.dosh + (int64_t)qr * a.doss + 8 * h;
  const uint16_t* op = a.o + b * a.osb + hq * a.osh + (int64_t)qr * a.oss + 8 * h;
  bf16x8 qf[DK], df[DK];
  float dl = 0.f;
#pragma unroll
  for (int dk = 0; dk < DK; ++dk) {
    qf[dk] = *reinterpret_cast<const bf16x8*>(qp + 16 * dk);
    df[dk] = *reinterpret_cast<const bf16x8*>(dp_ + 16 * dk);
    const bf16x8 of = *reinterpret_cast<const bf16x8*>(op + 16 * dk);
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += bf16_to_f32((uint16_t)df[dk][j]) * bf16_to_f32((uint16_t)of[j]);
  }
  const float delta = qok ? half_sum(dl) : 0.f;
  const float c = a.scale * kLog2e;
  const float lse2 = qok ? a.lse[((int64_t)b * a.Hq + hq) * a.Sq + qrow] * kLog2e : INFINITY;
  if (h == 0) {
    float* rs = a.rowstat + ((int64_t)bh * (2 * a.nqblk) + (qrow >> 6)) * 128 + (qrow & 63);
    rs[0] = -lse2 / c;
    rs[64] = -delta;
  }
  f32x16 dq[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[db][r] = 0.f;
  for (int p = 0; p < NS - 1 && p < ntile; ++p) {
    stage_tile<D>(lds[p], kb, a.kss, p * KT, kv_end, w, lane);
    stage_tile<D>(lds[p] + TILE, vb, a.vss, p * KT, kv_end, w, lane);
  }
  for (int it = 0; it < ntile; ++it) {
    wait_tile<NS>(it + 1 < ntile, 2 * tile_glds<D>());
    __syncthreads();
    if (it + NS - 1 < ntile) {
      char* nb = lds[(it + NS - 1) % NS];
      stage_tile<D>(nb, kb, a.kss, (it + NS - 1) * KT, kv_end, w, lane);
      stage_tile<D>(nb + TILE, vb, a.vss, (it + NS - 1) * KT, kv_end, w, lane);
    }
    const int k0 = it * KT;
    if (CAUSAL && k0 > qw0 + 31) continue;
    const char* Kt = lds[it % NS];
    const char* Vt = Kt + TILE;
    f32x16 s[2], dp[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[kk][r] = 0.f;
        dp[kk][r] = -delta;
      }
#pragma unroll
      for (int dk = 0; dk < DK; ++dk) s[kk] = MFMA32(row_frag<D>(Kt, 32 * kk, dk, lane), qf[dk], s[kk]);
#pragma unroll
      for (int dk = 0; dk < DK; ++dk) dp[kk] = MFMA32(row_frag<D>(Vt, 32 * kk, dk, lane), df[dk], dp[kk]);
    }
    const bool msk = k0 + KT > kv_end || (CAUSAL && k0 + KT - 1 > qw0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = fast_exp2(fmaf(s[kk][r], c, -lse2));
        if (msk) {
          const int key = k0 + 32 * kk + crow(r, h);
          if (key >= kv_end || (CAUSAL && key > qrow)) p = 0.f;
        }
        s[kk][r] = p * dp[kk][r];  // dS^T
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 dsf = pack8(s[kk], s2);
#pragma unroll
        for (int db = 0; db < DB; ++db) dq[db] = MFMA32(tr_frag<D>(Kt, 32 * kk + 16 * s2, db, lane), dsf, dq[db]);
      }
  }
  if (qok) {
    uint16_t* gp = a.dq + b * a.gqb + (int64_t)qrow * a.gqs + hq * a.gqh;
    const float sc = a.scale;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4(gp + 32 * db + 8 * g + 4 * h, dq[db][4 * g] * sc, dq[db][4 * g + 1] * sc, dq[db][4 * g + 2] * sc,
               dq[db][4 * g + 3] * sc);
  }
}

// ---------------------------------------------------------------------------- backward: dK, dV
template <int D, bool CAUSAL, int NS>
__device__ __forceinline__ void attn_dkdv_body(const Args& a) {
  constexpr int DK = D / 16, DB = D / 32, TILE = KT * 2 * D, STG = 2 * TILE + 512;
  __shared__ __attribute__((aligned(16))) char lds[NS][STG];
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int h = lane >> 5;
  const int G = a.Hq / a.Hkv, gper = G / a.gsplit;
  const int nbk = a.B * a.Hkv * a.gsplit, bid = blockIdx.x;
  const int kblk = bid / nbk, rr = bid - kblk * nbk;  // (causal: low key blocks carry the most work)
  const int b = rr / (a.Hkv * a.gsplit), hk = (rr / a.gsplit) % a.Hkv, gs = rr % a.gsplit;
  const int k0 = kblk * QB, kw0 = k0 + 32 * w, key = kw0 + (lane & 31);
  int kv_end = a.Sk;
  if (a.kvlen != nullptr) kv_end = min(kv_end, a.kvlen[b]);
  const int kr = min(key, a.Sk - 1);
  const uint16_t* kp = a.k + b * a.ksb + hk * a.ksh + (int64_t)kr * a.kss + 8 * h;
  const uint16_t* vp = a.v + b * a.vsb + hk * a.vsh + (int64_t)kr * a.vss + 8 * h;
  bf16x8 kf[DK], vf[DK];
#pragma unroll
  for (int dk = 0; dk < DK; ++dk) {
    kf[dk] = *reinterpret_cast<const bf16x8*>(kp + 16 * dk);
    vf[dk] = *reinterpret_cast<const bf16x8*>(vp + 16 * dk);
  }
  f32x16 dka[DB], dva[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dka[db][r] = 0.f;
      dva[db][r] = 0.f;
    }
  const float c = a.scale * kLog2e;
  const int ntq64 = 2 * a.nqblk;      // rowstat tiles per (b, hq)
  const int nqt = (a.Sq + KT - 1) / KT;
  const int qt0 = CAUSAL ? k0 / KT : 0;
  const int per = nqt - qt0 > 0 ? nqt - qt0 : 0;
  const int niter = gper * per;
  const bool wave_live = kw0 < kv_end;  // (wave-uniform) some key of this wave is valid
  auto stage = [&](int it, char* buf) {
    const int hq = hk * G + gs * gper + it / per, qt = qt0 + it % per;
    const uint16_t* qb = a.q + b * a.qsb + hq * a.qsh;
    const uint16_t* db_ = a.dout + b * a.dosb + hq * a.dosh;
    stage_tile<D>(buf, qb, a.qss, qt * KT, a.Sq, w, lane);
    stage_tile<D>(buf + TILE, db_, a.doss, qt * KT, a.Sq, w, lane);
    if (w == 0 && lane < 32)
      glds16(a.rowstat + (((int64_t)b * a.Hq + hq) * ntq64 + qt) * 128 + 4 * lane, buf + 2 * TILE);
  };
  for (int p = 0; p < NS - 1 && p < niter; ++p) stage(p, lds[p]);
  for (int it = 0; it < niter; ++it) {
    // wave 0 also issues the rowstat DMA of each stage
    wait_tile<NS>(it + 1 < niter, 2 * tile_glds<D>() + (w == 0 ? 1 : 0));
    __syncthreads();
    if (it + NS - 1 < niter) stage(it + NS - 1, lds[(it + NS - 1) % NS]);
    const int qt = qt0 + it % per, qs0 = qt * KT;
    if (!wave_live || (CAUSAL && qs0 + KT - 1 < kw0)) continue;  // every query row before the wave's keys
    const char* Qt = lds[it % NS];
    const char* Ot = Qt + TILE;  // dO
    const float* rs = reinterpret_cast<const float*>(Qt + 2 * TILE);
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      if (CAUSAL && qs0 + 32 * qb + 31 < kw0) continue;
      f32x16 s, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 nl = *reinterpret_cast<const float4*>(rs + 32 * qb + 8 * g + 4 * h);
        const float4 nd = *reinterpret_cast<const float4*>(rs + 64 + 32 * qb + 8 * g + 4 * h);
        s[4 * g] = nl.x; s[4 * g + 1] = nl.y; s[4 * g + 2] = nl.z; s[4 * g + 3] = nl.w;
        dp[4 * g] = nd.x; dp[4 * g + 1] = nd.y; dp[4 * g + 2] = nd.z; dp[4 * g + 3] = nd.w;
      }
#pragma unroll
      for (int dk = 0; dk < DK; ++dk) s = MFMA32(row_frag<D>(Qt, 32 * qb, dk, lane), kf[dk], s);
#pragma unroll
      for (int dk = 0; dk < DK; ++dk) dp = MFMA32(row_frag<D>(Ot, 32 * qb, dk, lane), vf[dk], dp);
      const bool msk = CAUSAL && qs0 + 32 * qb < kw0 + 31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = fast_exp2(c * s[r]);
        if (msk && key > qs0 + 32 * qb + crow(r, h)) p = 0.f;
        s[r] = p;
        dp[r] = p * dp[r];
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(s, s2), dsf = pack8(dp, s2);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          dva[db] = MFMA32(tr_frag<D>(Ot, 32 * qb + 16 * s2, db, lane), pf, dva[db]);
          dka[db] = MFMA32(tr_frag<D>(Qt, 32 * qb + 16 * s2, db, lane), dsf, dka[db]);
        }
      }
    }
  }
  if (key >= a.Sk) return;
  const bool kok = key < kv_end;  // padded keys: zero gradient
  const float sc = a.scale;
  if (a.gsplit == 1) {
    const int64_t off = b * a.gkb + (int64_t)key * a.gks + hk * a.gkh;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * db + 8 * g + 4 * h;
        const float z = kok ? 1.f : 0.f;
        store4(a.dk + off + d, dka[db][4 * g] * sc * z, dka[db][4 * g + 1] * sc * z, dka[db][4 * g + 2] * sc * z,
               dka[db][4 * g + 3] * sc * z);
        store4(a.dv + off + d, dva[db][4 * g] * z, dva[db][4 * g + 1] * z, dva[db][4 * g + 2] * z,
               dva[db][4 * g + 3] * z);
      }
  } else {
    const int64_t n = (int64_t)a.B * a.Sk * a.Hkv * D;
    float* pk = a.part + (int64_t)gs * 2 * n + (((int64_t)b * a.Sk + key) * a.Hkv + hk) * D;
    float* pv = pk + n;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * db + 8 * g + 4 * h;
        const float z = kok ? 1.f : 0.f;
        *reinterpret_cast<float4*>(pk + d) = make_float4(dka[db][4 * g] * sc * z, dka[db][4 * g + 1] * sc * z,
                                                         dka[db][4 * g + 2] * sc * z, dka[db][4 * g + 3] * sc * z);
        *reinterpret_cast<float4*>(pv + d) =
            make_float4(dva[db][4 * g] * z, dva[db][4 * g + 1] * z, dva[db][4 * g + 2] * z, dva[db][4 * g + 3] * z);
      }
  }
}

// Register budgets: the head-dim-64 backward kernels fit two waves per SIMD (<= 256 registers);
// the head-dim-128 ones would spill there, so they keep one wave per SIMD and every register.
template <int D, bool CAUSAL, int NS = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_attn_dq(Args a) {
  attn_dq_body<D, CAUSAL, NS>(a);
}
template <int D, bool CAUSAL, int NS = 2>
__global__ __launch_bounds__(256) void k_attn_dq_wide(Args a) {
  attn_dq_body<D, CAUSAL, NS>(a);
}
template <int D, bool CAUSAL, int NS = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_attn_dkdv(Args a) {
  attn_dkdv_body<D, CAUSAL, NS>(a);
}
template <int D, bool CAUSAL, int NS = 2>
__global__ __launch_bounds__(256) void k_attn_dkdv_wide(Args a) {
  attn_dkdv_body<D, CAUSAL, NS>(a);
}

// dK / dV of a split GQA group: sum the slices in order (deterministic), cast to bf16 into the
// (possibly strided) outputs; the partials are contiguous [B, Sk, Hkv, D]
__global__ __launch_bounds__(256) void k_attn_gsum(const float* __restrict__ part, int gsplit, int64_t n, int D,
                                                   int Hkv, int Sk, int64_t sb, int64_t ss, int64_t sh,
                                                   uint16_t* __restrict__ dk, uint16_t* __restrict__ dv) {
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < 2 * n; i += (int64_t)gridDim.x * 1024) {
    float4 s = *reinterpret_cast<const float4*>(part + i);
    for (int g = 1; g < gsplit; ++g) {
      const float4 x = *reinterpret_cast<const float4*>(part + (int64_t)g * 2 * n + i);
      s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
    }
    const int64_t j = i < n ? i : i - n;
    const int d = (int)(j % D);
    int64_t r = j / D;
    const int hk = (int)(r % Hkv);
    r /= Hkv;
    const int key = (int)(r % Sk);
    const int64_t b = r / Sk;
    uint16_t* o = (i < n ? dk : dv) + b * sb + (int64_t)key * ss + hk * sh + d;
    store4(o, s.x, s.y, s.z, s.w);
  }
}

// ---------------------------------------------------------------------------------------- host
namespace {

void check_qkv(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4, "attn: ", name,
              " must be a bf16 [B, S, H, D] device tensor");
  TORCH_CHECK(t.stride(3) == 1 && t.stride(2) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "attn: ", name, " needs d contiguous and 16-byte aligned rows");
}

Args make_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal, double scale,
               const c10::optional<at::Tensor>& kvlen) {
  check_qkv(q, "q");
  check_qkv(k, "k");
  check_qkv(v, "v");
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "attn: head dim 64 or 128");
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && k.sizes() == v.sizes() && k.size(0) == q.size(0),
              "attn: k / v shapes");
  TORCH_CHECK(q.size(2) % k.size(2) == 0, "attn: query heads must be a multiple of kv heads");
  TORCH_CHECK(!causal || q.size(1) == k.size(1), "attn: causal needs Sq == Sk");
  TORCH_CHECK(q.size(1) > 0 && k.size(1) > 0 && q.size(1) < (1 << 24) && k.size(1) < (1 << 24), "attn: sizes");
  Args a{};
  a.q = (const uint16_t*)q.data_ptr();
  a.k = (const uint16_t*)k.data_ptr();
  a.v = (const uint16_t*)v.data_ptr();
  a.qsb = q.stride(0); a.qss = q.stride(1); a.qsh = q.stride(2);
  a.ksb = k.stride(0); a.kss = k.stride(1); a.ksh = k.stride(2);
  a.vsb = v.stride(0); a.vss = v.stride(1); a.vsh = v.stride(2);
  a.B = (int)q.size(0); a.Sq = (int)q.size(1); a.Hq = (int)q.size(2);
  a.Sk = (int)k.size(1); a.Hkv = (int)k.size(2);
  a.scale = (float)scale;
  a.gsplit = 1;
  if (kvlen.has_value() && kvlen->defined()) {
    TORCH_CHECK(kvlen->is_cuda() && kvlen->scalar_type() == at::kInt && kvlen->numel() == q.size(0) &&
                    kvlen->is_contiguous(), "attn: kv_len must be int32 [B] on the device");
    a.kvlen = kvlen->data_ptr<int>();
  }
  return a;
}

}  // namespace

// LDS stages of the streamed tiles: 2 (HIPPS_ATTN_STAGES=3: the three-stage form, A/B).  Measured
// same-box (profiles/r6/attn/attn_stages_ab.txt): 3 stages cost the forward and the BERT backward
// (the LDS of a third stage takes the second workgroup per CU) and did not help the causal
// backward either (Llama-3-1B 0.462 / 0.467 ms with 2 vs 0.488 / 0.501 with 3) -- the kernels are
// not waiting on the tile DMA
int attn_stages(bool causal, bool backward) {
  static const int env = [] {
    const char* e = std::getenv("HIPPS_ATTN_STAGES");
    return e ? std::atoi(e) : 0;
  }();
  (void)causal;
  (void)backward;
  return env == 3 ? 3 : 2;
}

#define ATTN_DISPATCH2(KER64, KER128, D_, CAUSAL_, BWD_, GRID, A)                                 \
  do {                                                                                             \
    auto st = c10::hip::getCurrentHIPStream();                                                     \
    const bool s3 = attn::attn_stages(CAUSAL_, BWD_) == 3;                                         \
    if ((D_) == 64) {                                                                              \
      if (CAUSAL_) {                                                                               \
        if (s3) hipLaunchKernelGGL((KER64<64, true, 3>), dim3(GRID), dim3(256), 0, st, A);          \
        else hipLaunchKernelGGL((KER64<64, true, 2>), dim3(GRID), dim3(256), 0, st, A);             \
      } else {                                                                                     \
        if (s3) hipLaunchKernelGGL((KER64<64, false, 3>), dim3(GRID), dim3(256), 0, st, A);         \
        else hipLaunchKernelGGL((KER64<64, false, 2>), dim3(GRID), dim3(256), 0, st, A);            \
      }                                                                                            \
    } else {                                                                                       \
      if (CAUSAL_) {                                                                               \
        if (s3) hipLaunchKernelGGL((KER128<128, true, 3>), dim3(GRID), dim3(256), 0, st, A);        \
        else hipLaunchKernelGGL((KER128<128, true, 2>), dim3(GRID), dim3(256), 0, st, A);           \
      } else {                                                                                     \
        if (s3) hipLaunchKernelGGL((KER128<128, false, 3>), dim3(GRID), dim3(256), 0, st, A);       \
        else hipLaunchKernelGGL((KER128<128, false, 2>), dim3(GRID), dim3(256), 0, st, A);          \
      }                                                                                            \
    }                                                                                              \
  } while (0)
#define ATTN_DISPATCH(KER, D_, CAUSAL_, GRID, A) ATTN_DISPATCH2(KER, KER, D_, CAUSAL_, false, GRID, A)

}  // namespace attn

// o = softmax(q k^T * scale + mask) v  for q [B, Sq, Hq, D], k / v [B, Sk, Hkv, D] (bf16);
// returns (o [B, Sq, Hq, D] contiguous, lse [B, Hq, Sq] f32 natural log)
std::vector<at::Tensor> attn_forward(at::Tensor q, at::Tensor k, at::Tensor v, bool causal, double scale,
                                     c10::optional<at::Tensor> kvlen) {
  attn::Args a = attn::make_args(q, k, v, causal, scale, kvlen);
  const int64_t D = q.size(3);
  at::Tensor o = at::empty({q.size(0), q.size(1), q.size(2), D}, q.options());
  at::Tensor lse = at::empty({q.size(0), q.size(2), q.size(1)}, q.options().dtype(at::kFloat));
  a.out = (uint16_t*)o.data_ptr();
  a.osb = o.stride(0); a.oss = o.stride(1); a.osh = o.stride(2);
  a.lse = lse.data_ptr<float>();
  a.nblk = a.nqblk = (a.Sq + attn::QB - 1) / attn::QB;
  const int64_t grid = (int64_t)a.nblk * a.B * a.Hq;
  TORCH_CHECK(grid < (int64_t(1) << 31), "attn: grid");
  ATTN_DISPATCH(attn::k_attn_fwd, D, causal, (unsigned)grid, a);
  return {o, lse};
}

// gradients of attn_forward: returns (dq, dk, dv) contiguous in the layouts of q, k, v
std::vector<at::Tensor> attn_backward(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o,
                                      at::Tensor lse, bool causal, double scale, c10::optional<at::Tensor> kvlen,
                                      c10::optional<at::Tensor> dq_out, c10::optional<at::Tensor> dk_out,
                                      c10::optional<at::Tensor> dv_out) {
  attn::Args a = attn::make_args(q, k, v, causal, scale, kvlen);
  attn::check_qkv(dout, "dout");
  attn::check_qkv(o, "o");
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes(), "attn: dout / o shapes");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() &&
                  lse.numel() == q.size(0) * q.size(1) * q.size(2), "attn: lse");
  const int64_t D = q.size(3);
  a.o = (const uint16_t*)o.data_ptr();
  a.osb = o.stride(0); a.oss = o.stride(1); a.osh = o.stride(2);
  a.dout = (const uint16_t*)dout.data_ptr();
  a.dosb = dout.stride(0); a.doss = dout.stride(1); a.dosh = dout.stride(2);
  a.lse = lse.data_ptr<float>();
  // outputs: contiguous, or caller-provided views (a packed [B, S, 3, H, D] QKV gradient: the
  // kernels write dq / dk / dv straight into it, no concatenation pass)
  auto out_or = [&](const c10::optional<at::Tensor>& t, const at::Tensor& like, const char* name) {
    if (t.has_value() && t->defined()) {
      attn::check_qkv(*t, name);
      TORCH_CHECK(t->sizes() == like.sizes(), "attn: ", name, " shape");
      return *t;
    }
    return at::empty(like.sizes(), like.options());
  };
  at::Tensor dq = out_or(dq_out, q, "dq_out");
  at::Tensor dk = out_or(dk_out, k, "dk_out");
  at::Tensor dv = out_or(dv_out, k, "dv_out");
  TORCH_CHECK(dk.strides() == dv.strides(), "attn: dk_out / dv_out must share strides");
  a.dq = (uint16_t*)dq.data_ptr();
  a.dk = (uint16_t*)dk.data_ptr();
  a.dv = (uint16_t*)dv.data_ptr();
  a.gqb = dq.stride(0); a.gqs = dq.stride(1); a.gqh = dq.stride(2);
  a.gkb = dk.stride(0); a.gks = dk.stride(1); a.gkh = dk.stride(2);
  a.nblk = a.nqblk = (a.Sq + attn::QB - 1) / attn::QB;
  at::Tensor rowstat = at::empty({(int64_t)a.B * a.Hq * 2 * a.nblk * 128}, q.options().dtype(at::kFloat));
  a.rowstat = rowstat.data_ptr<float>();
  const int64_t gq = (int64_t)a.nblk * a.B * a.Hq;
  ATTN_DISPATCH2(attn::k_attn_dq, attn::k_attn_dq_wide, D, causal, true, (unsigned)gq, a);
  // dK / dV: split the GQA group over workgroups when the (batch, kv head, key block) grid is
  // small: under the causal mask the first key block of a sequence sweeps every query tile and
  // the last one a single tile, so a grid that fits the GPU in one wave runs as long as its
  // heaviest workgroup (Llama-3-1B, 512 workgroups: 2x the mean); more, lighter workgroups
  // launched heaviest-first balance.  The slices' fp32 partials are summed in a fixed order.
  const int nkb = (a.Sk + attn::QB - 1) / attn::QB;
  const int G = a.Hq / a.Hkv;
  const int64_t want = causal ? 2048 : 512;
  int gsplit = 1;
  while (gsplit < G && (int64_t)nkb * a.B * a.Hkv * gsplit < want && G % (gsplit * 2) == 0) gsplit *= 2;
  a.gsplit = gsplit;
  at::Tensor part;
  if (gsplit > 1) {
    part = at::empty({(int64_t)gsplit * 2 * dk.numel()}, q.options().dtype(at::kFloat));
    a.part = part.data_ptr<float>();
  }
  a.nblk = nkb;
  const int64_t gk = (int64_t)nkb * a.B * a.Hkv * gsplit;
  ATTN_DISPATCH2(attn::k_attn_dkdv, attn::k_attn_dkdv_wide, D, causal, true, (unsigned)gk, a);
  if (gsplit > 1) {
    const int64_t n = dk.numel();
    const int grid = (int)std::min<int64_t>(2048, (2 * n / 4 + 255) / 256);
    hipLaunchKernelGGL(attn::k_attn_gsum, grid, 256, 0, c10::hip::getCurrentHIPStream(), a.part, gsplit, n, (int)D,
                       a.Hkv, a.Sk, a.gkb, a.gks, a.gkh, (uint16_t*)dk.data_ptr(), (uint16_t*)dv.data_ptr());
  }
  return {dq, dk, dv};
}

}  // namespace hipps
