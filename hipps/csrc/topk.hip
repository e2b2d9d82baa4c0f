// hipps — exact top-k magnitude sparsification (radix select + look-back compaction).
//
// Device replacement for the external codec's encode (ps.py:94) when the codec is top-k.
// Output is a fixed-size message (k = ceil(ratio*n) known at plan time), so no size round-trip
// is needed: the reference's per-tensor Iallgather of lengths (mpi_comms.py:150-158, M1) goes
// away.  Wire: int32 idx[k] + val[k] (f32 or bf16), idx in ascending order.
//
// Four full passes over the bucket (round 1 made five plus three single-workgroup histogram
// walks over all of it), everything else on ~1% of it:
//   P1  hist of |x| bits 30..20 over the whole bucket (fused with the error-feedback fold
//       r <- g + r, so later passes read one array)                               [full read]
//   pick   single workgroup: the bin holding the k-th largest key
//   P2  filter: keys in that bin -> candidate list (wave-aggregated append)         [full read]
//   P3/P4  histograms of bits 19..9 and 8..0 over the candidates only, + picks -> exact k-th
//       key T and how many == T to admit (lowest index first)
//   P5  compaction in index order: per-4096-element-chunk counts (> T, == T) [full read], one
//       workgroup scans the ~n/4096 counts, each chunk writes its selected (index, value) pairs
//       at its prefix [full read].  (A decoupled look-back would save the count pass, but its
//       chunk tickets are one atomic address and serialised to ~2 ms on a 25 M bucket.)
// If the threshold bin holds more candidates than the list can take (e.g. mostly-zero
// gradients) the candidate passes fall back to filtering the whole bucket (flag in device
// state, no host sync).  Ties are admitted lowest-index-first, so the message is bitwise
// deterministic and equal to the CPU reference.
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cmath>
#include <cstring>

namespace hipps {

constexpr int kHistBins = 2048;
constexpr int kCompactPer = 16;                     // elements per lane in P5 (4 x float4)
constexpr int kChunk = kBlock * kCompactPer;        // 4096 elements per look-back chunk

struct SelState {        // lives in a small device workspace
  uint32_t prefix;       // selected high bits of the k-th largest key
  uint32_t mask;         // which bits of prefix are decided
  uint32_t remaining;    // how many elements still to take inside the undecided bucket
  uint32_t ncand;        // candidates appended by P2
  uint32_t overflow;     // candidate list too small: later passes scan the whole bucket
  uint32_t ticket;       // P5 chunk tickets
  uint32_t cap_cand;
  uint32_t pad;
  uint32_t hist[kHistBins];
};

__device__ __forceinline__ uint32_t absbits(float x) { return __float_as_uint(x) & 0x7fffffffu; }

__global__ __launch_bounds__(kBlock) void k_topk_init(SelState* __restrict__ st, uint32_t prefix, uint32_t mask,
                                                      uint32_t k, uint32_t cap_cand) {
  if (threadIdx.x == 0) {
    st->prefix = prefix; st->mask = mask; st->remaining = k; st->ncand = 0; st->overflow = 0; st->ticket = 0;
    st->cap_cand = cap_cand; st->pad = 0;
  }
  for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) st->hist[b] = 0;
}

// P1 (and the overflow fallback of P3/P4): histogram over elements whose decided bits match
// prefix.  Four per-wave LDS sub-histograms cut same-address atomic serialisation 4x.
__global__ __launch_bounds__(kBlock) void k_topk_hist(const float* __restrict__ g, float* __restrict__ resid,
                                                      int fold_resid, int64_t n, int lo, int nbits,
                                                      SelState* __restrict__ st, int only_overflow) {
  __shared__ uint32_t h[4][kHistBins];
  if (only_overflow && !st->overflow) return;
  const int nb = 1 << nbits;
  const int w = threadIdx.x >> 6;
  for (int b = threadIdx.x; b < 4 * kHistBins; b += blockDim.x) (&h[0][0])[b] = 0;
  __syncthreads();
  const uint32_t prefix = st->prefix, mask = st->mask;
  const float* src = (resid && !fold_resid) ? resid : g;
  const int64_t nv = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    const int64_t i = v << 2;
    float4 x = *reinterpret_cast<const float4*>(src + i);
    if (fold_resid) {
      float4 r = *reinterpret_cast<const float4*>(resid + i);
      x.x += r.x; x.y += r.y; x.z += r.z; x.w += r.w;
      *reinterpret_cast<float4*>(resid + i) = x;
    }
    const uint32_t k0 = absbits(x.x), k1 = absbits(x.y), k2 = absbits(x.z), k3 = absbits(x.w);
    if ((k0 & mask) == prefix) atomicAdd(&h[w][(k0 >> lo) & (nb - 1)], 1u);
    if ((k1 & mask) == prefix) atomicAdd(&h[w][(k1 >> lo) & (nb - 1)], 1u);
    if ((k2 & mask) == prefix) atomicAdd(&h[w][(k2 >> lo) & (nb - 1)], 1u);
    if ((k3 & mask) == prefix) atomicAdd(&h[w][(k3 >> lo) & (nb - 1)], 1u);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nv << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float x = src[i];
      if (fold_resid) { x += resid[i]; resid[i] = x; }
      const uint32_t k = absbits(x);
      if ((k & mask) == prefix) atomicAdd(&h[w][(k >> lo) & (nb - 1)], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const uint32_t c = h[0][b] + h[1][b] + h[2][b] + h[3][b];
    if (c) atomicAdd(&st->hist[b], c);
  }
}

// single workgroup: locate the bucket holding the remaining-th largest key, descend one digit
__global__ __launch_bounds__(kBlock) void k_topk_pick(int lo, int nbits, SelState* __restrict__ st) {
  __shared__ uint32_t part[kBlock];
  __shared__ uint32_t sel_bin, sel_above;
  const int nb = 1 << nbits;
  const int per = nb / kBlock;  // 8 or 2 bins per thread
  const int t = threadIdx.x;
  // thread t owns bins [nb - (t+1)*per, nb - t*per): t = 0 holds the largest keys
  uint32_t s = 0;
  for (int j = 0; j < per; ++j) s += st->hist[nb - (t + 1) * per + j];
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    const uint32_t need = st->remaining;
    uint32_t cum = 0;
    int c = 0;
    for (; c < kBlock - 1; ++c) {
      if (cum + part[c] >= need) break;
      cum += part[c];
    }
    int bin = nb - c * per - 1;
    const int lowest = nb - (c + 1) * per;
    for (; bin > lowest; --bin) {
      const uint32_t hb = st->hist[bin];
      if (cum + hb >= need) break;
      cum += hb;
    }
    sel_bin = (uint32_t)bin;
    sel_above = cum;
  }
  __syncthreads();
  for (int b = t; b < nb; b += kBlock) st->hist[b] = 0;  // re-arm for the next digit
  if (t == 0) {
    st->prefix |= sel_bin << lo;
    st->mask |= (uint32_t)(nb - 1) << lo;
    st->remaining -= sel_above;
  }
}

// P2: append every element of the selected top-11-bit bin to the candidate list.  Each
// workgroup scans one contiguous range, collects its candidates in LDS and reserves global space
// with ONE atomic at the end (a per-wave atomic on one address serialises ~10^5 times on a
// 25 M-element bucket); an LDS overflow spills straight to global with per-element atomics.
constexpr int kCandLds = 2048;
__global__ __launch_bounds__(kBlock) void k_topk_filter(const float* __restrict__ src, int64_t n,
                                                        SelState* __restrict__ st, uint32_t* __restrict__ ckey,
                                                        uint32_t* __restrict__ cidx) {
  __shared__ uint32_t lkey[kCandLds], lidx[kCandLds];
  __shared__ uint32_t lcount, lbase;
  const uint32_t prefix = st->prefix, mask = st->mask, cap = st->cap_cand;
  if (threadIdx.x == 0) lcount = 0;
  __syncthreads();
  const int64_t nv = (n + 3) >> 2;
  const int64_t per = (nv + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = (int64_t)blockIdx.x * per, v1 = v0 + per < nv ? v0 + per : nv;
  for (int64_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    const int64_t i = v << 2;
    uint32_t k[4] = {0u, 0u, 0u, 0u};
    bool m[4] = {false, false, false, false};
    if (i + 4 <= n) {
      float4 x = *reinterpret_cast<const float4*>(src + i);
      k[0] = absbits(x.x); k[1] = absbits(x.y); k[2] = absbits(x.z); k[3] = absbits(x.w);
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] = (k[j] & mask) == prefix;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i + j < n) { k[j] = absbits(src[i + j]); m[j] = (k[j] & mask) == prefix; }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (m[j]) {
        const uint32_t p = atomicAdd(&lcount, 1u);
        if (p < kCandLds) {
          lkey[p] = k[j];
          lidx[p] = (uint32_t)(i + j);
        } else {  // spill (rare): straight to the global list
          const uint32_t g = atomicAdd(&st->ncand, 1u);
          if (g < cap) { ckey[g] = k[j]; cidx[g] = (uint32_t)(i + j); }
        }
      }
  }
  __syncthreads();
  const uint32_t cnt = lcount < kCandLds ? lcount : kCandLds;
  if (threadIdx.x == 0) lbase = cnt ? atomicAdd(&st->ncand, cnt) : 0u;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) {
    const uint32_t g = lbase + j;
    if (g < cap) { ckey[g] = lkey[j]; cidx[g] = lidx[j]; }
  }
}

// P3/P4: histogram of the candidates; if P2 overflowed the list, of the whole bucket instead
__global__ __launch_bounds__(kBlock) void k_topk_hist_cand(const uint32_t* __restrict__ ckey,
                                                           const float* __restrict__ src, int64_t n, int lo, int nbits,
                                                           SelState* __restrict__ st) {
  __shared__ uint32_t h[kHistBins];
  const uint32_t ncand = st->ncand;
  const bool full = ncand > st->cap_cand;
  const int nb = 1 << nbits;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t prefix = st->prefix, mask = st->mask;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (!full) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ncand; j += stride) {
      const uint32_t k = ckey[j];
      if ((k & mask) == prefix) atomicAdd(&h[(k >> lo) & (nb - 1)], 1u);
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const uint32_t k = absbits(src[i]);
      if ((k & mask) == prefix) atomicAdd(&h[(k >> lo) & (nb - 1)], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&st->hist[b], h[b]);
}

// ---- P5: compaction in index order: count -> scan -> write ------------------------------
// A 4096-element chunk per workgroup (16 elements per lane as 4 coalesced float4 segments).
// count: per-chunk (> T, == T) totals; scan: one workgroup turns them into exclusive prefixes
// (6 k chunks for a 25 M bucket); write: each chunk re-reads its elements and places the
// selected ones at prefix + local rank.  No spin-waits, no single-address atomics.
__device__ __forceinline__ void chunk_load(const float* __restrict__ src, int64_t n, int64_t c, float (&x)[kCompactPer]) {
#pragma unroll
  for (int j = 0; j < kCompactPer / 4; ++j) {
    const int64_t i = c * kChunk + (int64_t)j * (kBlock * 4) + threadIdx.x * 4;
    if (i + 4 <= n) {
      float4 t = *reinterpret_cast<const float4*>(src + i);
      x[4 * j] = t.x; x[4 * j + 1] = t.y; x[4 * j + 2] = t.z; x[4 * j + 3] = t.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[4 * j + e] = (i + e < n) ? src[i + e] : 0.f;
    }
  }
}

// per segment j: (eq << 16) | gt of this lane's 4 elements (each <= 4)
__device__ __forceinline__ void chunk_counts(int64_t n, int64_t c, uint32_t T, const float (&x)[kCompactPer],
                                             uint32_t (&cnt)[kCompactPer / 4]) {
#pragma unroll
  for (int j = 0; j < kCompactPer / 4; ++j) {
    const int64_t i = c * kChunk + (int64_t)j * (kBlock * 4) + threadIdx.x * 4;
    uint32_t gt = 0, eq = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool in = i + e < n;
      const uint32_t k = absbits(x[4 * j + e]);
      gt += in && k > T;
      eq += in && k == T;
    }
    cnt[j] = (eq << 16) | gt;
  }
}

__global__ __launch_bounds__(kBlock) void k_topk_count(const float* __restrict__ src, int64_t n,
                                                       const SelState* __restrict__ st, uint32_t* __restrict__ cgt,
                                                       uint32_t* __restrict__ ceq, int64_t nchunks) {
  __shared__ uint32_t red[4];
  const uint32_t T = st->prefix;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    float x[kCompactPer];
    uint32_t cnt[kCompactPer / 4];
    chunk_load(src, n, c, x);
    chunk_counts(n, c, T, x, cnt);
    uint32_t v = cnt[0] + cnt[1] + cnt[2] + cnt[3];  // <= 16 per field: packed sum stays exact
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t t = red[0] + red[1] + red[2] + red[3];  // <= 4096 per field
      cgt[c] = t & 0xffffu;
      ceq[c] = t >> 16;
    }
    __syncthreads();
  }
}

// exclusive scan of both count arrays in place (one workgroup; nchunks ~ n / 4096)
__global__ __launch_bounds__(1024) void k_topk_scan(uint32_t* __restrict__ cgt, uint32_t* __restrict__ ceq,
                                                    int64_t nchunks, int32_t* __restrict__ count_out, uint32_t cap) {
  __shared__ uint32_t sg[1024], se[1024];
  __shared__ uint32_t carry_g, carry_e;
  if (threadIdx.x == 0) { carry_g = 0; carry_e = 0; }
  __syncthreads();
  for (int64_t base = 0; base < nchunks; base += 1024) {
    const int64_t c = base + threadIdx.x;
    const uint32_t vg = c < nchunks ? cgt[c] : 0, ve = c < nchunks ? ceq[c] : 0;
    sg[threadIdx.x] = vg; se[threadIdx.x] = ve;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
      const uint32_t ag = threadIdx.x >= off ? sg[threadIdx.x - off] : 0;
      const uint32_t ae = threadIdx.x >= off ? se[threadIdx.x - off] : 0;
      __syncthreads();
      sg[threadIdx.x] += ag; se[threadIdx.x] += ae;
      __syncthreads();
    }
    if (c < nchunks) { cgt[c] = carry_g + sg[threadIdx.x] - vg; ceq[c] = carry_e + se[threadIdx.x] - ve; }
    __syncthreads();
    if (threadIdx.x == 1023) { carry_g += sg[1023]; carry_e += se[1023]; }
    __syncthreads();
  }
  if (count_out && threadIdx.x == 0) count_out[0] = (int32_t)(carry_g < cap ? carry_g : cap);
}

template <typename VT>
__global__ __launch_bounds__(kBlock) void k_topk_write(const float* __restrict__ src, float* __restrict__ resid,
                                                       int64_t n, const SelState* __restrict__ st,
                                                       const uint32_t* __restrict__ pgt, const uint32_t* __restrict__ peq,
                                                       int64_t nchunks, int32_t* __restrict__ idx, VT* __restrict__ val,
                                                       uint32_t cap) {
  __shared__ uint32_t wsum[kCompactPer / 4][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t T = st->prefix, need_eq = st->remaining;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    float x[kCompactPer];
    uint32_t cnt[kCompactPer / 4], incl[kCompactPer / 4];
    chunk_load(src, n, c, x);
    chunk_counts(n, c, T, x, cnt);
    if (pgt[c] >= cap && need_eq == 0) continue;  // nothing of this chunk fits (threshold overflow)
#pragma unroll
    for (int j = 0; j < kCompactPer / 4; ++j) {  // index order: segment, wave, lane
      uint32_t v = cnt[j];
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t a = __shfl_up(v, o, 64);
        if (lane >= o) v += a;
      }
      incl[j] = v;
      if (lane == 63) wsum[j][w] = v;
    }
    __syncthreads();
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < kCompactPer / 4; ++j) {
      uint32_t wb = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) wb += (q < w) ? wsum[j][q] : 0u;
      const uint32_t off = run + wb + incl[j] - cnt[j];
#pragma unroll
      for (int q = 0; q < 4; ++q) run += wsum[j][q];
      const int64_t i = c * kChunk + (int64_t)j * (kBlock * 4) + threadIdx.x * 4;
      uint32_t bg = pgt[c] + (off & 0xffffu), be = peq[c] + (off >> 16);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (i + e >= n) break;
        const uint32_t k = absbits(x[4 * j + e]);
        const bool isgt = k > T, iseq = k == T;
        const uint32_t pos = bg + (be < need_eq ? be : need_eq);
        if ((isgt || (iseq && be < need_eq)) && pos < cap) {
          idx[pos] = (int32_t)(i + e);
          Vec4<VT>::store1(val, pos, x[4 * j + e]);
          if (resid) resid[i + e] = x[4 * j + e] - Vec4<VT>::load1(val, pos);
        }
        bg += isgt;
        be += iseq;
      }
    }
    __syncthreads();  // wsum reuse
  }
}

// acc[idx[j]] (+)= gscale * val[j]; one message has unique indices, so no atomics are needed.
template <typename VT>
__global__ __launch_bounds__(kBlock) void k_scatter_acc(const int32_t* __restrict__ idx, const VT* __restrict__ val,
                                                        int64_t k, float* __restrict__ acc, float gscale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride)
    acc[idx[j]] += gscale * Vec4<VT>::load1(val, j);
}

// topk+int8: acc[idx[j]] += gscale * q[j] * scale[j / 256]
__global__ __launch_bounds__(kBlock) void k_scatter_acc_q8(const int32_t* __restrict__ idx,
                                                           const int8_t* __restrict__ q,
                                                           const float* __restrict__ scales, int64_t k,
                                                           float* __restrict__ acc, float gscale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride)
    acc[idx[j]] += gscale * (float)q[j] * scales[j >> 8];
}

// error feedback for topk+int8: r[idx[j]] += v[j] - deq(q[j])
__global__ __launch_bounds__(kBlock) void k_topk_q8_resid(const int32_t* __restrict__ idx,
                                                          const float* __restrict__ v, const int8_t* __restrict__ q,
                                                          const float* __restrict__ scales, int64_t k,
                                                          float* __restrict__ resid) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride)
    resid[idx[j]] += v[j] - (float)q[j] * scales[j >> 8];
}

// ------------------------------------------------------------------------------------------
namespace {

struct TopkWs {
  SelState* st;
  uint32_t* cgt;  // per-chunk counts, then exclusive prefixes
  uint32_t* ceq;
  uint32_t* ckey;
  uint32_t* cidx;
  int64_t nchunks;
  int64_t cap;
};

int64_t cand_cap(int64_t n) { return std::max<int64_t>(4096, n / 16); }

int64_t ws_bytes_for(int64_t n) {
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  return (int64_t)sizeof(SelState) + 8 * nchunks + 8 * cand_cap(n) + 64;
}

TopkWs carve(at::Tensor& workspace, int64_t n) {
  const int64_t need = ws_bytes_for(n);
  TORCH_CHECK(workspace.is_cuda() && workspace.numel() * workspace.element_size() >= need,
              "workspace too small: need ", need, " bytes (topk_workspace_bytes)");
  static_assert(sizeof(SelState) % 16 == 0, "SelState keeps the count arrays aligned");
  char* ws = (char*)workspace.data_ptr();
  TORCH_CHECK(reinterpret_cast<uintptr_t>(ws) % 16 == 0, "workspace must be 16-byte aligned");
  TopkWs w;
  w.st = reinterpret_cast<SelState*>(ws);
  w.nchunks = (n + kChunk - 1) / kChunk;
  w.cap = cand_cap(n);
  w.cgt = reinterpret_cast<uint32_t*>(ws + sizeof(SelState));
  w.ceq = w.cgt + w.nchunks;
  w.ckey = w.ceq + w.nchunks;
  w.cidx = w.ckey + w.cap;
  return w;
}

template <typename VT>
void launch_compact(hipStream_t stream, const float* src, float* rp, int64_t n, const TopkWs& w, int32_t* idx, VT* val,
                    uint32_t cap, int32_t* count_out) {
  const int grid = (int)std::min<int64_t>(w.nchunks, kMaxGrid);
  hipLaunchKernelGGL(k_topk_count, grid, kBlock, 0, stream, src, n, w.st, w.cgt, w.ceq, w.nchunks);
  hipLaunchKernelGGL(k_topk_scan, 1, 1024, 0, stream, w.cgt, w.ceq, w.nchunks, count_out, cap);
  hipLaunchKernelGGL(k_topk_write<VT>, grid, kBlock, 0, stream, src, rp, n, w.st, w.cgt, w.ceq, w.nchunks, idx, val,
                     cap);
}

}  // namespace

void topk_encode(at::Tensor g, c10::optional<at::Tensor> resid, int64_t k, at::Tensor idx, at::Tensor val,
                 at::Tensor workspace) {
  TORCH_CHECK(g.is_cuda() && g.is_contiguous() && g.scalar_type() == at::kFloat, "g: contiguous f32 device tensor");
  const int64_t n = g.numel();
  TORCH_CHECK(k >= 1 && k <= n, "need 1 <= k <= n");
  TORCH_CHECK(n < (int64_t)1 << 31, "top-k bucket must have < 2^31 elements");
  TORCH_CHECK(idx.numel() == k && idx.scalar_type() == at::kInt, "idx must be int32[k]");
  TORCH_CHECK(val.numel() == k && (val.scalar_type() == at::kFloat || val.scalar_type() == at::kBFloat16),
              "val must be f32/bf16[k]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0, "g must be 16-byte aligned");
  TopkWs w = carve(workspace, n);
  float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->numel() == n && resid->scalar_type() == at::kFloat && resid->is_contiguous(), "residual");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(resid->data_ptr()) % 16 == 0, "residual must be 16-byte aligned");
    rp = resid->data_ptr<float>();
  }
  auto stream = c10::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(k_topk_init, 1, kBlock, 0, stream, w.st, 0u, 0u, (uint32_t)k, (uint32_t)w.cap);
  const int grid = grid_for(n >> 2);
  // histogram grids stay <= 1024 workgroups: every workgroup merges its bins with global atomics
  const int hgrid = std::min(grid, 1024);
  // P1: fold + top-11-bit histogram over the whole bucket
  hipLaunchKernelGGL(k_topk_hist, hgrid, kBlock, 0, stream, g.data_ptr<float>(), rp, (int)(rp != nullptr), n, 20, 11,
                     w.st, 0);
  hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, 20, 11, w.st);
  const float* src = rp ? rp : g.data_ptr<float>();
  // P2: candidates of the selected bin (one contiguous range per workgroup)
  hipLaunchKernelGGL(k_topk_filter, grid, kBlock, 0, stream, src, n, w.st, w.ckey, w.cidx);
  // P3/P4 on the candidates
  const int cgrid = (int)std::max<int64_t>(1, std::min<int64_t>(1024, w.cap / 1024));
  hipLaunchKernelGGL(k_topk_hist_cand, cgrid, kBlock, 0, stream, w.ckey, src, n, 9, 11, w.st);
  hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, 9, 11, w.st);
  hipLaunchKernelGGL(k_topk_hist_cand, cgrid, kBlock, 0, stream, w.ckey, src, n, 0, 9, w.st);
  hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, 0, 9, w.st);
  // P5: look-back compaction in index order
  if (val.scalar_type() == at::kFloat)
    launch_compact<float>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), val.data_ptr<float>(), (uint32_t)k, nullptr);
  else
    launch_compact<uint16_t>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), (uint16_t*)val.data_ptr(), (uint32_t)k,
                             nullptr);
}

// ---- threshold sparsification (variable-size message, count in a device header) -----------
__global__ __launch_bounds__(kBlock) void k_fold(const float* __restrict__ g, float* __restrict__ r, int64_t n) {
  const int64_t nv = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += stride) {
    float4 a = *reinterpret_cast<const float4*>(g + 4 * v), b = *reinterpret_cast<const float4*>(r + 4 * v);
    *reinterpret_cast<float4*>(r + 4 * v) = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
  if (blockIdx.x == 0)
    for (int64_t i = (nv << 2) + threadIdx.x; i < n; i += blockDim.x) r[i] += g[i];
}

template <typename VT>
__global__ __launch_bounds__(kBlock) void k_scatter_acc_count(const int32_t* __restrict__ idx,
                                                              const VT* __restrict__ val,
                                                              const int32_t* __restrict__ count, int64_t cap,
                                                              float* __restrict__ acc, float gscale) {
  const int64_t k = min((int64_t)count[0], cap);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride)
    acc[idx[j]] += gscale * Vec4<VT>::load1(val, j);
}

// Every |x| > tau (x = g [+ residual]) in ascending index order, at most cap of them; the true
// count (clamped) goes to count[0] on the device, so decode needs no host round trip.
void thresh_encode(at::Tensor g, c10::optional<at::Tensor> resid, double tau, at::Tensor count, at::Tensor idx,
                   at::Tensor val, at::Tensor workspace) {
  TORCH_CHECK(g.is_cuda() && g.is_contiguous() && g.scalar_type() == at::kFloat, "g: contiguous f32 device tensor");
  const int64_t n = g.numel(), cap = idx.numel();
  TORCH_CHECK(val.numel() == cap && count.scalar_type() == at::kInt && count.numel() >= 1, "count/idx/val");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0, "g must be 16-byte aligned");
  TORCH_CHECK(n < (int64_t)1 << 31, "bucket must have < 2^31 elements");
  TopkWs w = carve(workspace, n);
  auto stream = c10::hip::getCurrentHIPStream();
  float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->numel() == n && resid->scalar_type() == at::kFloat, "residual");
    rp = resid->data_ptr<float>();
    hipLaunchKernelGGL(k_fold, grid_for(n >> 2), kBlock, 0, stream, g.data_ptr<float>(), rp, n);
  }
  float t = (float)std::fabs(tau);
  uint32_t tbits;
  std::memcpy(&tbits, &t, 4);
  // T = tau exactly, no ties admitted: every |x| > tau, in index order (one look-back pass)
  hipLaunchKernelGGL(k_topk_init, 1, kBlock, 0, stream, w.st, tbits, 0xffffffffu, 0u, (uint32_t)w.cap);
  const float* src = rp ? rp : g.data_ptr<float>();
  if (val.scalar_type() == at::kFloat)
    launch_compact<float>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), val.data_ptr<float>(), (uint32_t)cap,
                          count.data_ptr<int32_t>());
  else
    launch_compact<uint16_t>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), (uint16_t*)val.data_ptr(), (uint32_t)cap,
                             count.data_ptr<int32_t>());
}

// Copy a threshold message [count header | idx[cap] | val[cap]] moving only what the count says:
// the async PS push of a variable-size code costs 16 + count * (4 + value bytes) over xGMI instead
// of the static capacity (README.md:28-31 "unknown size" without a size round trip).
__global__ __launch_bounds__(kBlock) void k_copy_counted(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                         int64_t idx_off, int64_t val_off, int val_esz, int64_t cap) {
  const int64_t k = min((int64_t)reinterpret_cast<const int32_t*>(src)[0], cap);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t0 < 4) reinterpret_cast<int32_t*>(dst)[t0] = reinterpret_cast<const int32_t*>(src)[t0];
  const int32_t* si = reinterpret_cast<const int32_t*>(src + idx_off);
  int32_t* di = reinterpret_cast<int32_t*>(dst + idx_off);
  for (int64_t j = t0; j < k; j += stride) di[j] = si[j];
  if (val_esz == 4) {
    const float* sv = reinterpret_cast<const float*>(src + val_off);
    float* dv = reinterpret_cast<float*>(dst + val_off);
    for (int64_t j = t0; j < k; j += stride) dv[j] = sv[j];
  } else {
    const uint16_t* sv = reinterpret_cast<const uint16_t*>(src + val_off);
    uint16_t* dv = reinterpret_cast<uint16_t*>(dst + val_off);
    for (int64_t j = t0; j < k; j += stride) dv[j] = sv[j];
  }
}

void copy_counted(at::Tensor src, at::Tensor dst, int64_t idx_off, int64_t val_off, int64_t val_esz, int64_t cap) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.scalar_type() == at::kByte && dst.scalar_type() == at::kByte,
              "copy_counted: uint8 device buffers");
  TORCH_CHECK(val_esz == 2 || val_esz == 4, "value size 2 or 4");
  TORCH_CHECK(src.numel() >= val_off + cap * val_esz && dst.numel() >= val_off + cap * val_esz, "message too small");
  TORCH_CHECK(idx_off % 4 == 0 && val_off % 4 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0, "alignment");
  hipLaunchKernelGGL(k_copy_counted, grid_for(std::max<int64_t>(cap, 4)), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     src.data_ptr<uint8_t>(), dst.data_ptr<uint8_t>(), idx_off, val_off, (int)val_esz, cap);
}

void thresh_accumulate(at::Tensor count, at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat, "acc: f32 device tensor");
  const int64_t cap = idx.numel();
  if (cap == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  if (val.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(k_scatter_acc_count<float>, grid_for(cap), kBlock, 0, stream, idx.data_ptr<int32_t>(),
                       val.data_ptr<float>(), count.data_ptr<int32_t>(), cap, acc.data_ptr<float>(), (float)gscale);
  else
    hipLaunchKernelGGL(k_scatter_acc_count<uint16_t>, grid_for(cap), kBlock, 0, stream, idx.data_ptr<int32_t>(),
                       (const uint16_t*)val.data_ptr(), count.data_ptr<int32_t>(), cap, acc.data_ptr<float>(),
                       (float)gscale);
}

int64_t topk_workspace_bytes(int64_t n) { return ws_bytes_for(n); }

void topk_accumulate(at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat, "acc: f32 device tensor");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.numel() == val.numel(), "idx/val mismatch");
  const int64_t k = idx.numel();
  if (k == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = grid_for(k);
  if (val.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(k_scatter_acc<float>, grid, kBlock, 0, stream, idx.data_ptr<int32_t>(), val.data_ptr<float>(),
                       k, acc.data_ptr<float>(), (float)gscale);
  else if (val.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(k_scatter_acc<uint16_t>, grid, kBlock, 0, stream, idx.data_ptr<int32_t>(),
                       (const uint16_t*)val.data_ptr(), k, acc.data_ptr<float>(), (float)gscale);
  else
    TORCH_CHECK(false, "val must be f32 or bf16");
}

void topk_q8_accumulate(at::Tensor idx, at::Tensor q, at::Tensor scales, at::Tensor acc, double gscale) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat, "acc: f32 device tensor");
  TORCH_CHECK(idx.scalar_type() == at::kInt && q.scalar_type() == at::kChar && idx.numel() == q.numel(), "idx/q");
  const int64_t k = idx.numel();
  TORCH_CHECK(scales.numel() == (k + 255) / 256, "scales size");
  if (k == 0) return;
  hipLaunchKernelGGL(k_scatter_acc_q8, grid_for(k), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     idx.data_ptr<int32_t>(), (const int8_t*)q.data_ptr(), scales.data_ptr<float>(), k,
                     acc.data_ptr<float>(), (float)gscale);
}

void topk_q8_residual(at::Tensor idx, at::Tensor v, at::Tensor q, at::Tensor scales, at::Tensor resid) {
  const int64_t k = idx.numel();
  if (k == 0) return;
  hipLaunchKernelGGL(k_topk_q8_resid, grid_for(k), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     idx.data_ptr<int32_t>(), v.data_ptr<float>(), (const int8_t*)q.data_ptr(),
                     scales.data_ptr<float>(), k, resid.data_ptr<float>());
}

}  // namespace hipps
