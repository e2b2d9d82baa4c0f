// hipps — exact top-k magnitude sparsification and threshold sparsification.
//
// Device replacement for the external codec's encode (ps.py:94) when the codec is top-k.
// Output is a fixed-size message (k = ceil(ratio*n) known at plan time), so no size round-trip
// is needed: the reference's per-tensor Iallgather of lengths (mpi_comms.py:150-158, M1) goes
// away.  Wire: int32 idx[k] + val[k] (f32 or bf16), idx in ascending order.
//
// ONE full pass over the bucket in the steady state (round 1 made five, plus three
// single-workgroup histogram walks over all of it); everything else works on a short list:
//   P1  per workgroup a contiguous range of 4096-element chunks ("region"): error-feedback fold
//       r <- g + r, histogram of key bits 30..20 (key = |x| as bits), and an index-ordered list
//       of every element with key >= spec_lo = 0.95 x the threshold the previous call on this
//       workspace found (the threshold of an error-feedback gradient moves little from step to
//       step)                                                           [read g, r; write r]
//       A chunk whose entries do not fit the region's slot spills them to a shared pool
//       (one atomic per spilled chunk, on one of 8 pool shards).
//   pick   one workgroup: the bin B holding the k-th largest key
//   P3/P4  histograms of bits 19..9 and 8..0 over the listed keys of bin B + picks -> the exact
//       k-th key T and how many keys == T to admit (lowest index first).  P3's pick first checks
//       that the list reaches the k-th key (listed keys of B >= the number still needed);
//   P2  only when it does not (first call, or the gradient shrank by > 5 %): every region
//       re-reads its range and lists keys >= B's lower edge, and P3 is redone
//   P5  per region: count the listed keys > T and == T, one workgroup scans the region counts,
//       each region writes its selected (index, value) pairs at its prefix (list order = index
//       order), clearing their residuals.
// If a pool shard runs out (e.g. a mostly-constant bucket), P3-P5 fall back to full passes
// over the bucket (flag in device state, no host sync).  Ties are admitted lowest-index-first,
// so a message is bitwise deterministic and equal to the CPU reference.
//
// The threshold codec (variable size) is P1 with the fixed bound key > tau (no histogram), then
// the scan and the write: one full pass.
//
// No spin-waits and no single-address atomic hot spots: a decoupled look-back compaction was
// measured slower (its chunk tickets are one atomic address, serialised to ~2 ms on 25 M).
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>

namespace hipps {

constexpr int kHistBins = 2048;
constexpr int kCompactPer = 16;                 // elements per lane per chunk (4 x float4)
constexpr int kChunk = kBlock * kCompactPer;    // 4096 elements
constexpr int kMaxRegions = 1024;               // workgroups of the region passes
constexpr uint32_t kBinMask = 0x7ff00000u;      // key bits 30..20: the first radix digit
constexpr float kSpecMargin = 0.95f;            // P1 lists keys >= 0.95 x the previous call's threshold

constexpr uint32_t kNoList = 0x80000000u;       // a bound no key reaches
constexpr int kHistCopies = 8;
constexpr int kPoolShards = 8;                  // spill counters, one 128-byte line each
constexpr int kMaxCpw = 512;                    // chunks per region (n < 2^31)

struct SelState {        // lives at the head of the workspace
  uint32_t prefix;       // selected high bits of the k-th largest key (threshold codec: T)
  uint32_t mask;         // which bits of prefix are decided
  uint32_t remaining;    // how many elements still to take inside the undecided bucket
  uint32_t capw;         // list slot entries per region
  uint32_t pool_cap;     // entries per pool shard
  uint32_t full;         // a pool shard ran out: P3-P5 take full passes over the bucket
  uint32_t spec_lo;      // P1's list bound
  uint32_t prev_T;       // final key of the previous call (persists in the workspace)
  uint32_t redo;         // the list missed part of the k-th key's range: repair + recount
  uint32_t ticket[4];    // arrival counters of the in-launch picks (zero between launches)
  uint32_t pad[19];
  uint32_t pool_used[kPoolShards * 32];
  // kHistCopies histograms: workgroup b merges into copy b % kHistCopies, so a bin's global
  // atomics come from 1/8 of the workgroups (depth ~110 instead of ~900 on a 25 M bucket); the
  // pick sums the copies
  uint32_t hist[kHistCopies][kHistBins];
};

__device__ __forceinline__ uint32_t absbits(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// Workgroup barrier for LDS hand-offs only: __syncthreads() also drains every outstanding global
// load (s_waitcnt vmcnt(0)), which would retire k_collect's prefetch of the next chunk at each
// chunk's list barriers.  Only LDS traffic is ordered here.
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// in-launch digit pick (defined with k_topk_pick below)
__device__ __forceinline__ void pick_body(int lo, int nbits, SelState* __restrict__ st, int flags, uint32_t* wtot);
__device__ __forceinline__ bool last_arriver(uint32_t* ticket, uint32_t* flag);


// mode: 0 = top-k, 1 = threshold (prefix = T, no ties)
__global__ __launch_bounds__(kBlock) void k_sel_init(SelState* __restrict__ st, uint32_t prefix, uint32_t mask,
                                                     uint32_t k, uint32_t capw, uint32_t pool_cap, int topk) {
  if (threadIdx.x == 0) {
    st->prefix = prefix; st->mask = mask; st->remaining = k; st->capw = capw;
    st->pool_cap = pool_cap; st->full = 0;
    st->redo = 0;
    if (topk) {
      // no usable previous threshold (first call, or a zero / non-finite one): P1 lists nothing
      // and the repair pass lists from bin B's edge
      const float pt = __uint_as_float(st->prev_T & 0x7fffffffu);
      st->spec_lo = (pt > 0.f && pt < __builtin_inff()) ? absbits(pt * kSpecMargin) : kNoList;
    } else {
      st->spec_lo = 0;
    }
  }
  if (threadIdx.x < kPoolShards) st->pool_used[threadIdx.x * 32] = 0;
  if (topk)
    for (int b = threadIdx.x; b < kHistCopies * kHistBins; b += blockDim.x) (&st->hist[0][0])[b] = 0;
}

// ---- chunked streaming ------------------------------------------------------------------
// Lane t holds elements c*4096 + j*1024 + 4t + e (segment j < 4, e < 4): four coalesced 16-byte
// loads per array in flight per lane.  Index order within a chunk = (segment, wave, lane, e).
__device__ __forceinline__ int64_t seg_index(int64_t c, int j) {
  return c * kChunk + (int64_t)j * (kBlock * 4) + threadIdx.x * 4;
}

__device__ __forceinline__ void chunk_load(const float* __restrict__ src, int64_t n, int64_t c, float (&x)[kCompactPer]) {
#pragma unroll
  for (int j = 0; j < kCompactPer / 4; ++j) {
    const int64_t i = seg_index(c, j);
    if (i + 4 <= n) {
      float4 t = *reinterpret_cast<const float4*>(src + i);
      x[4 * j] = t.x; x[4 * j + 1] = t.y; x[4 * j + 2] = t.z; x[4 * j + 3] = t.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[4 * j + e] = (i + e < n) ? src[i + e] : 0.f;
    }
  }
}

__device__ __forceinline__ void chunk_store(float* __restrict__ dst, int64_t n, int64_t c, const float (&x)[kCompactPer]) {
#pragma unroll
  for (int j = 0; j < kCompactPer / 4; ++j) {
    const int64_t i = seg_index(c, j);
    if (i + 4 <= n) {
      *reinterpret_cast<float4*>(dst + i) = make_float4(x[4 * j], x[4 * j + 1], x[4 * j + 2], x[4 * j + 3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (i + e < n) dst[i + e] = x[4 * j + e];
    }
  }
}

// x = src (+ r, and r <- x when fold_r is given): both arrays' loads issued together
__device__ __forceinline__ void chunk_fold(const float* __restrict__ src, float* __restrict__ fold_r, int64_t n,
                                           int64_t c, float (&x)[kCompactPer]) {
  chunk_load(src, n, c, x);
  if (fold_r) {
    float y[kCompactPer];
    chunk_load(fold_r, n, c, y);
#pragma unroll
    for (int e = 0; e < kCompactPer; ++e) x[e] += y[e];
    chunk_store(fold_r, n, c, x);
  }
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* red4) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = v;
  __syncthreads();
  const uint32_t t = red4[0] + red4[1] + red4[2] + red4[3];
  __syncthreads();
  return t;
}

// exclusive workgroup scan; *total gets the workgroup sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* red4, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = __shfl_up(incl, o, 64);
    if (lane >= o) incl += a;
  }
  if (lane == 63) red4[w] = incl;
  __syncthreads();
  uint32_t wb = 0, t = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    wb += (q < w) ? red4[q] : 0u;
    t += red4[q];
  }
  __syncthreads();
  *total = t;
  return wb + incl - v;
}

struct Regions {       // region r = chunks [first(r), first(r + 1)) = [r*cpw, min((r+1)*cpw, nchunks))
  uint32_t* lval;      // list entries: raw f32 bits
  uint32_t* lidx;      //               element index
  uint32_t* coff;      // per chunk: first list entry (slot or pool)
  uint32_t* ccnt;      //            entries
  uint32_t* sfill;     // per region: entries in its slot
  uint32_t* cgt;       //             selected count (> T), then exclusive prefix
  uint32_t* ceq;       //             == T count, then exclusive prefix
  int64_t nchunks;
  int64_t cpw;         // chunks per region
  int64_t pool_off;    // first pool entry (after nreg * capw slot entries)
  // (an even split, 1024 regions of 6-7 chunks at 25.6 M instead of 892 of 7, measured no faster:
  // 183.8 / 184.1 vs 182.6 / 181.2 us, profiles/codec/r5/ab_topk.txt)
  __device__ __forceinline__ int64_t first(int64_t r) const { return std::min<int64_t>(r * cpw, nchunks); }
};

constexpr uint32_t kNoBase = 0xffffffffu;

// Index-ordered list of the chunk's elements with key >= bound (entry = raw f32 bits + index).
// The entries go to the region's slot if they fit, else to a pool shard (one atomic); the chunk's
// record (first entry, count) goes to coff / ccnt.  Returns the count (workgroup-uniform).
__device__ __forceinline__ uint32_t collect_chunk(const float (&x)[kCompactPer], int64_t n, int64_t c, uint32_t bound,
                                                  uint32_t& slot_pos, uint32_t slot_end, SelState* __restrict__ st,
                                                  const Regions& R, uint32_t (*wsum)[4], uint32_t* sbase) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t m[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t i = seg_index(c, j);
    uint32_t cnt = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) cnt += (i + e < n) && absbits(x[4 * j + e]) >= bound;
    m[j] = cnt;
  }
  // two segments per 32-bit word: a wave's segment total is <= 256, so 16-bit fields never carry
  uint32_t ia = m[0] | (m[1] << 16), ib = m[2] | (m[3] << 16);
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t ta = __shfl_up(ia, o, 64), tb = __shfl_up(ib, o, 64);
    if (lane >= o) { ia += ta; ib += tb; }
  }
  if (lane == 63) { wsum[0][w] = ia & 0xffffu; wsum[1][w] = ia >> 16; wsum[2][w] = ib & 0xffffu; wsum[3][w] = ib >> 16; }
  lds_sync();
  const uint32_t incl[4] = {ia & 0xffffu, ia >> 16, ib & 0xffffu, ib >> 16};
  uint32_t off[4], run = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t wb = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      wb += (q < w) ? wsum[j][q] : 0u;
      tot += wsum[j][q];
    }
    off[j] = run + wb + incl[j] - m[j];
    run += tot;
  }
  uint32_t base;
  if (slot_pos + run <= slot_end) {  // uniform: every thread computed the same run
    base = slot_pos;
    slot_pos += run;
  } else {
    if (threadIdx.x == 0) {
      const int shard = blockIdx.x & (kPoolShards - 1);
      const uint32_t p = atomicAdd(&st->pool_used[shard * 32], run);
      uint32_t b = kNoBase;
      if ((uint64_t)p + run <= st->pool_cap) b = (uint32_t)R.pool_off + shard * st->pool_cap + p;
      else atomicOr(&st->full, 1u);
      *sbase = b;
    }
    __syncthreads();
    base = *sbase;
  }
  if (base != kNoBase) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!m[j]) continue;
      uint32_t p = base + off[j];
      const int64_t i = seg_index(c, j);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if ((i + e < n) && absbits(x[4 * j + e]) >= bound) {
          R.lval[p] = __float_as_uint(x[4 * j + e]);
          R.lidx[p] = (uint32_t)(i + e);
          ++p;
        }
    }
  }
  if (threadIdx.x == 0) { R.coff[c] = base; R.ccnt[c] = run; }
  lds_sync();  // wsum / sbase reuse
  return run;
}

// P1 / P2: [fold] + [histogram of bits 30..20] + the region's ordered list of keys >= bound.
// mode 0: top-k P1 (bound = spec_lo); 1: threshold (bound = T + 1, counts -> cgt / ceq);
// 2: top-k repair (bound = bin B's lower edge; nothing to do when P1's bound covered bin B).
// PF: the next chunk's loads (g, and r when folding) are issued before the current chunk is
// processed, so a region's chunks stream with one HBM round trip exposed per region instead of
// one per chunk (HIPPS_TOPK_PF=0: the unpipelined loop, for A/B)
template <bool HIST, bool PF = true>
__global__ __launch_bounds__(kBlock) void k_collect(const float* __restrict__ src, float* __restrict__ fold_r,
                                                    int64_t n, SelState* __restrict__ st, Regions R, int mode,
                                                    int fold_pick = 0) {
  __shared__ uint32_t h[HIST ? 4 : 1][HIST ? kHistBins : 1];
  __shared__ uint32_t wsum[4][4], sbase;
  if (mode == 2 && !st->redo) return;  // grid-uniform
  const int w = threadIdx.x >> 6;
  if (HIST) {
    for (int b = threadIdx.x; b < 4 * kHistBins; b += blockDim.x) (&h[0][0])[b] = 0;
    __syncthreads();
  }
  const uint32_t bound = mode == 0 ? st->spec_lo : mode == 1 ? st->prefix + 1u : (st->prefix & kBinMask);
  const uint32_t capw = st->capw;
  uint32_t slot_pos = blockIdx.x * capw;
  const uint32_t slot_end = slot_pos + capw;
  uint32_t total = 0;
  const int64_t c0 = R.first(blockIdx.x), c1 = R.first(blockIdx.x + 1);
  float gx[PF ? kCompactPer : 1], rx[PF ? kCompactPer : 1];
  if constexpr (PF) {
    if (c0 < c1) {
      chunk_load(src, n, c0, gx);
      if (fold_r) chunk_load(fold_r, n, c0, rx);
    }
  }
  for (int64_t c = c0; c < c1; ++c) {
    float x[kCompactPer];
    if constexpr (PF) {
#pragma unroll
      for (int e = 0; e < kCompactPer; ++e) x[e] = fold_r ? gx[e] + rx[e] : gx[e];
      if (c + 1 < c1) {  // next chunk in flight during this one's histogram, list and stores
        chunk_load(src, n, c + 1, gx);
        if (fold_r) chunk_load(fold_r, n, c + 1, rx);
      }
      if (fold_r) chunk_store(fold_r, n, c, x);
    } else {
      chunk_fold(src, fold_r, n, c, x);
    }
    if (HIST) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t i = seg_index(c, j);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (i + e < n) atomicAdd(&h[w][absbits(x[4 * j + e]) >> 20], 1u);
      }
    }
    total += collect_chunk(x, n, c, bound, slot_pos, slot_end, st, R, wsum, &sbase);
  }
  if (threadIdx.x == 0) {
    R.sfill[blockIdx.x] = slot_pos - blockIdx.x * capw;
    if (mode == 1) { R.cgt[blockIdx.x] = total; R.ceq[blockIdx.x] = 0; }
  }
  if (HIST) {
    __syncthreads();
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) {
      const uint32_t c = h[0][b] + h[1][b] + h[2][b] + h[3][b];
      if (c) atomicAdd(&st->hist[blockIdx.x % kHistCopies][b], c);
    }
    if (fold_pick && last_arriver(&st->ticket[0], &h[0][0]))  // (h is free after the merge)
      pick_body(20, 11, st, 0, &h[0][4]);
  }
}

// A region's list, chunk by chunk: records in LDS with exclusive prefixes, so list entry j of the
// region (index order) is found by a binary search over <= cpw chunks.
struct RegionView {
  uint32_t* off;  // [kMaxCpw] chunk's first entry
  uint32_t* pre;  // [kMaxCpw] entries of the region before the chunk
  int nc;
  uint32_t total;
  __device__ __forceinline__ uint32_t entry(uint32_t j) const {
    int lo = 0, hi = nc - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= j) lo = mid; else hi = mid - 1;
    }
    return off[lo] + (j - pre[lo]);
  }
  // entries j, j+1, ..., j+U-1 (those < total): one search, then walk forward
  template <int U>
  __device__ __forceinline__ void entries(uint32_t j, uint32_t (&e)[U]) const {
    int lo = 0, hi = nc - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= j) lo = mid; else hi = mid - 1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      while (lo + 1 < nc && pre[lo + 1] <= j + u) ++lo;
      e[u] = off[lo] + (j + u - pre[lo]);
    }
  }
};

constexpr int kListU = 8;  // list entries per lane per step: 8 independent loads in flight

__device__ __forceinline__ RegionView load_region(const Regions& R, uint32_t* s_off, uint32_t* s_pre, uint32_t* red4) {
  RegionView v;
  const int64_t c0 = R.first(blockIdx.x);
  v.nc = (int)(R.first(blockIdx.x + 1) - c0);
  // two chunks per thread (cpw <= 512)
  const int t = threadIdx.x;
  uint32_t a = 0, b = 0;
  if (2 * t < v.nc) { a = R.ccnt[c0 + 2 * t]; s_off[2 * t] = R.coff[c0 + 2 * t]; }
  if (2 * t + 1 < v.nc) { b = R.ccnt[c0 + 2 * t + 1]; s_off[2 * t + 1] = R.coff[c0 + 2 * t + 1]; }
  uint32_t tot;
  const uint32_t ex = block_excl_scan(a + b, red4, &tot);
  if (2 * t < v.nc) s_pre[2 * t] = ex;
  if (2 * t + 1 < v.nc) s_pre[2 * t + 1] = ex + a;
  __syncthreads();
  v.off = s_off;
  v.pre = s_pre;
  v.total = tot;
  return v;
}

// The list storage walked flat, for passes that need no index order: every region's slot
// (filled part), then every pool shard's used part.  v = virtual position; the walk is coalesced.
struct FlatList {
  uint32_t slot_total, capw, pool_cap, size;
  uint32_t pre[kPoolShards + 1];  // virtual start of each pool shard
  int64_t pool_off;
  __device__ __forceinline__ void init(const SelState* st, const Regions& R, int nreg) {
    capw = st->capw;
    pool_cap = st->pool_cap;
    slot_total = (uint32_t)nreg * capw;
    pool_off = R.pool_off;
    uint32_t v = slot_total;
#pragma unroll
    for (int s = 0; s < kPoolShards; ++s) {
      pre[s] = v;
      const uint32_t u = st->pool_used[s * 32];
      v += u < pool_cap ? u : pool_cap;
    }
    pre[kPoolShards] = v;
    size = v;
  }
  // storage position of virtual position v, or kNoBase for an unfilled slot position
  __device__ __forceinline__ uint32_t at(uint32_t v, const Regions& R) const {
    if (v < slot_total) {
      const uint32_t b = v / capw;
      return v - b * capw < R.sfill[b] ? v : kNoBase;
    }
    int s = 0;
#pragma unroll
    for (int q = 1; q < kPoolShards; ++q) s += v >= pre[q];
    return (uint32_t)pool_off + s * pool_cap + (v - pre[s]);
  }
};

// One workgroup: find the bin holding the remaining-th largest key and descend one digit.
// Thread t owns bins [nb - (t+1)*per, nb - t*per) (t = 0 the largest keys); a wave-shuffle scan
// of the per-thread sums finds the owning thread in log steps.  flags: kPickFinal records T for
// the next call's speculative bound; kPickCheck (first digit over the list) verifies that the
// listed keys of bin B reach down to the remaining-th one -- the list holds every key >= spec_lo,
// so that holds iff their count >= remaining -- and otherwise raises redo (repair pass, fresh
// pool) without descending; kPickRetry runs only after such a redo.
constexpr int kPickFinal = 1, kPickCheck = 2, kPickRetry = 4;
__device__ __forceinline__ void pick_body(int lo, int nbits, SelState* __restrict__ st, int flags, uint32_t* wtot) {
  if ((flags & kPickRetry) && !st->redo) return;
  const int nb = 1 << nbits;
  const int per = nb / kBlock;  // 8 or 2
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t hv[kHistBins / kBlock];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kHistBins / kBlock; ++j) {
    uint32_t c = 0;
    if (j < per) {
#pragma unroll
      for (int q = 0; q < kHistCopies; ++q) c += st->hist[q][nb - t * per - 1 - j];  // descending
    }
    hv[j] = c;
    s += c;
  }
  const uint32_t need = st->remaining;
  uint32_t incl = s;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = __shfl_up(incl, o, 64);
    if (lane >= o) incl += a;
  }
  if (lane == 63) wtot[w] = incl;
  __syncthreads();  // every hist read and the remaining read happened before this barrier
#pragma unroll
  for (int q = 0; q < 4; ++q) incl += (q < w) ? wtot[q] : 0u;
  const uint32_t excl = incl - s;
  for (int b = t; b < nb; b += kBlock)  // re-arm for the next digit
#pragma unroll
    for (int q = 0; q < kHistCopies; ++q) st->hist[q][b] = 0;
  if (flags & kPickCheck) {
    const uint32_t total = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    if (total < need && !st->full) {  // (full mode counted every key of bin B)
      if (t == 0) {
        st->redo = 1;
        st->full = 0;
        for (int q = 0; q < kPoolShards; ++q) st->pool_used[q * 32] = 0;
      }
      return;
    }
  }
  if ((excl < need && need <= incl) || (t == kBlock - 1 && incl < need)) {
    uint32_t cum = excl;
    int bin = nb - t * per - 1;
#pragma unroll
    for (int j = 0; j < kHistBins / kBlock; ++j) {
      if (j >= per - 1) break;
      if (cum + hv[j] >= need) break;
      cum += hv[j];
      --bin;
    }
    const uint32_t prefix = st->prefix | ((uint32_t)bin << lo);
    st->prefix = prefix;
    st->mask |= (uint32_t)(nb - 1) << lo;
    st->remaining = need - cum;
    if (flags & kPickFinal) st->prev_T = prefix;
    if (flags & kPickRetry) st->redo = 0;
  }
}

__global__ __launch_bounds__(kBlock) void k_topk_pick(int lo, int nbits, SelState* __restrict__ st, int flags) {
  __shared__ uint32_t wtot[4];
  pick_body(lo, nbits, st, flags, wtot);
}

// The pick of a digit inside the launch that built its histogram: every workgroup merges its
// histogram with global atomics, drains, and one lane releases (agent scope) and takes an arrival
// ticket; the workgroup that arrives last acquires and runs the pick (cdna_hip_programming.md
// 'In-launch split-K reduction': correct for any placement over XCDs).  Saves one dependent
// single-workgroup launch per digit.  ``flag`` is a word of the caller's LDS.
__device__ __forceinline__ bool last_arriver(uint32_t* ticket, uint32_t* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t last = old == gridDim.x - 1 ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0u;
}

// P3/P4: histogram of the listed keys of the selected bin; full pass over the bucket if the pool ran out
__global__ __launch_bounds__(kBlock) void k_hist_list(const float* __restrict__ src, int64_t n, int lo, int nbits,
                                                      SelState* __restrict__ st, Regions R, int nreg, int retry,
                                                      int pick_flags = -1, int ticket = 1) {
  __shared__ uint32_t h[kHistBins];
  if (retry && !st->redo) return;
  const int nb = 1 << nbits;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t prefix = st->prefix, mask = st->mask;
  if (!st->full) {
    FlatList L;
    L.init(st, R, nreg);
    const uint32_t step = gridDim.x * blockDim.x * kListU;
    for (uint32_t v0 = blockIdx.x * blockDim.x * kListU + threadIdx.x; v0 < L.size; v0 += step) {
      uint32_t k[kListU];
#pragma unroll
      for (int u = 0; u < kListU; ++u) {
        const uint32_t v = v0 + u * blockDim.x;
        const uint32_t p = v < L.size ? L.at(v, R) : kNoBase;
        k[u] = p != kNoBase ? (R.lval[p] & 0x7fffffffu) : 0xffffffffu;
      }
#pragma unroll
      for (int u = 0; u < kListU; ++u)
        if (k[u] != 0xffffffffu && (k[u] & mask) == prefix) atomicAdd(&h[(k[u] >> lo) & (nb - 1)], 1u);
    }
  } else {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      const uint32_t k = absbits(src[i]);
      if ((k & mask) == prefix) atomicAdd(&h[(k >> lo) & (nb - 1)], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&st->hist[blockIdx.x % kHistCopies][b], h[b]);
  if (pick_flags >= 0) {
    __syncthreads();  // h is reused for the arrival flag and the pick's wave totals
    if (last_arriver(&st->ticket[ticket], &h[0])) pick_body(lo, nbits, st, pick_flags, &h[4]);
  }
}

// P5a (top-k): per region, the counts of keys > T and == T, from its list -- or, when a pool
// shard ran out (full mode), from the region's chunks of the bucket (one launch for both: a
// separate full-mode twin cost an empty 1024-workgroup launch per call)
__global__ __launch_bounds__(kBlock) void k_count_list(const float* __restrict__ src, int64_t n,
                                                       const SelState* __restrict__ st, Regions R) {
  __shared__ uint32_t red[4], s_off[kMaxCpw], s_pre[kMaxCpw];
  const uint32_t T = st->prefix;
  uint32_t gt = 0, eq = 0;
  if (!st->full) {
    const RegionView v = load_region(R, s_off, s_pre, red);
    for (uint32_t j0 = threadIdx.x * kListU; j0 < v.total; j0 += blockDim.x * kListU) {
      uint32_t e[kListU], k[kListU];
      v.entries<kListU>(j0, e);
#pragma unroll
      for (int u = 0; u < kListU; ++u) k[u] = j0 + u < v.total ? (R.lval[e[u]] & 0x7fffffffu) : 0u;
#pragma unroll
      for (int u = 0; u < kListU; ++u) {
        gt += k[u] > T;
        eq += j0 + u < v.total && k[u] == T;
      }
    }
  } else {
    const int64_t c0 = R.first(blockIdx.x), c1 = R.first(blockIdx.x + 1);
    for (int64_t c = c0; c < c1; ++c) {
      float x[kCompactPer];
      chunk_load(src, n, c, x);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t i = seg_index(c, j);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t k = absbits(x[4 * j + e]);
          gt += (i + e < n) && k > T;
          eq += (i + e < n) && k == T;
        }
      }
    }
  }
  gt = block_sum(gt, red);
  eq = block_sum(eq, red);
  if (threadIdx.x == 0) { R.cgt[blockIdx.x] = gt; R.ceq[blockIdx.x] = eq; }
}

// P5b: exclusive scan of the (<= 1024) region counts, one 1024-thread workgroup
__global__ __launch_bounds__(1024) void k_scan_regions(uint32_t* __restrict__ cgt, uint32_t* __restrict__ ceq, int nreg,
                                                       int32_t* __restrict__ count_out, uint32_t cap) {
  __shared__ uint32_t wg[16], we[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t sg = t < nreg ? cgt[t] : 0u, se = t < nreg ? ceq[t] : 0u;
  uint32_t ig = sg, ie = se;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = __shfl_up(ig, o, 64), b = __shfl_up(ie, o, 64);
    if (lane >= o) { ig += a; ie += b; }
  }
  if (lane == 63) { wg[w] = ig; we[w] = ie; }
  __syncthreads();
  uint32_t og = 0, oe = 0, tg = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    og += (q < w) ? wg[q] : 0u;
    oe += (q < w) ? we[q] : 0u;
    tg += wg[q];
  }
  if (t < nreg) { cgt[t] = og + ig - sg; ceq[t] = oe + ie - se; }
  if (count_out && t == 0) count_out[0] = (int32_t)(tg < cap ? tg : cap);
}

// place one element: rank-th > T / eq-th == T of the bucket in index order
template <typename VT>
__device__ __forceinline__ void place(uint32_t bits, uint32_t i, bool isgt, bool iseq, uint32_t g, uint32_t e,
                                      uint32_t need_eq, uint32_t cap, int32_t* __restrict__ idx, VT* __restrict__ val,
                                      float* __restrict__ resid) {
  if (!(isgt || (iseq && e < need_eq))) return;
  const uint32_t pos = g + (e < need_eq ? e : need_eq);
  if (pos >= cap) return;
  const float x = __uint_as_float(bits);
  idx[pos] = (int32_t)i;
  Vec4<VT>::store1(val, pos, x);
  if (resid) resid[i] = x - Vec4<VT>::load1(val, pos);  // error feedback keeps the rounding residue
}

// P5c: each region writes its selected pairs at its prefix, in index order
template <typename VT>
__global__ __launch_bounds__(kBlock) void k_write_regions(const float* __restrict__ src, float* __restrict__ resid,
                                                          int64_t n, const SelState* __restrict__ st, Regions R,
                                                          int32_t* __restrict__ idx, VT* __restrict__ val,
                                                          uint32_t cap) {
  __shared__ uint32_t red[4], wsum[4][4], s_off[kMaxCpw], s_pre[kMaxCpw];
  const uint32_t T = st->prefix, need_eq = st->remaining;
  uint32_t bg = R.cgt[blockIdx.x], be = R.ceq[blockIdx.x];
  if (bg >= cap) return;  // every position of this region is past the message
  if (!st->full) {
    const RegionView v = load_region(R, s_off, s_pre, red);
    const uint32_t m = v.total;
    // each lane takes kListU consecutive entries (index order), one workgroup scan per step
    for (uint32_t j0 = 0; j0 < m; j0 += blockDim.x * kListU) {
      const uint32_t j = j0 + threadIdx.x * kListU;
      uint32_t e[kListU], bits[kListU];
      v.entries<kListU>(j, e);
#pragma unroll
      for (int u = 0; u < kListU; ++u) bits[u] = j + u < m ? R.lval[e[u]] : 0u;
      uint32_t cnt = 0;  // (eq << 16) | gt of this lane's entries
#pragma unroll
      for (int u = 0; u < kListU; ++u) {
        const uint32_t k = bits[u] & 0x7fffffffu;
        cnt += (j + u < m) ? ((uint32_t)(k > T) | ((uint32_t)(k == T) << 16)) : 0u;
      }
      uint32_t tot;
      const uint32_t ex = block_excl_scan(cnt, red, &tot);  // <= 2048 per field per step
      uint32_t g = bg + (ex & 0xffffu), q = be + (ex >> 16);
#pragma unroll
      for (int u = 0; u < kListU; ++u) {
        if (j + u >= m) break;
        const uint32_t k = bits[u] & 0x7fffffffu;
        const bool isgt = k > T, iseq = k == T;
        if (isgt || iseq) place<VT>(bits[u], R.lidx[e[u]], isgt, iseq, g, q, need_eq, cap, idx, val, resid);
        g += isgt;
        q += iseq;
      }
      bg += tot & 0xffffu;
      be += tot >> 16;
    }
    return;
  }
  // full mode: the region's chunks in order, ordered positions within each chunk
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c0 = R.first(blockIdx.x), c1 = R.first(blockIdx.x + 1);
  for (int64_t c = c0; c < c1; ++c) {
    float x[kCompactPer];
    chunk_load(src, n, c, x);
    uint32_t cnt[4], incl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t i = seg_index(c, j);
      uint32_t gt = 0, eq = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t k = absbits(x[4 * j + e]);
        gt += (i + e < n) && k > T;
        eq += (i + e < n) && k == T;
      }
      cnt[j] = (eq << 16) | gt;
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
    for (int j = 0; j < 4; ++j) {
      uint32_t wb = 0, tot = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        wb += (q < w) ? wsum[j][q] : 0u;
        tot += wsum[j][q];
      }
      const uint32_t off = run + wb + incl[j] - cnt[j];
      run += tot;
      const int64_t i = seg_index(c, j);
      uint32_t g = bg + (off & 0xffffu), e = be + (off >> 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (i + q >= n) break;
        const uint32_t k = absbits(x[4 * j + q]);
        const bool isgt = k > T, iseq = k == T;
        place<VT>(__float_as_uint(x[4 * j + q]), (uint32_t)(i + q), isgt, iseq, g, e, need_eq, cap, idx, val, resid);
        g += isgt;
        e += iseq;
      }
    }
    bg += run & 0xffffu;
    be += run >> 16;
    __syncthreads();  // wsum reuse
  }
}

// acc[idx[j]] (+)= gscale * val[j]; one message has unique indices, so no atomics are needed.
template <typename VT>
__global__ __launch_bounds__(kBlock) void k_scatter_acc(const int32_t* __restrict__ idx, const VT* __restrict__ val,
                                                        int64_t k, float* __restrict__ acc, float gscale, int acquire) {
  if (acquire) acquire_remote_block();  // the message was written by another GPU (common.h)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < k; j += stride)
    acc[idx[j]] += gscale * Vec4<VT>::load1(val, j);
}

// topk+int8: acc[idx[j]] += gscale * q[j] * scale[j / 256]
__global__ __launch_bounds__(kBlock) void k_scatter_acc_q8(const int32_t* __restrict__ idx,
                                                           const int8_t* __restrict__ q,
                                                           const float* __restrict__ scales, int64_t k,
                                                           float* __restrict__ acc, float gscale, int acquire) {
  if (acquire) acquire_remote_block();
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

struct Geo {
  int64_t nchunks, cpw, nreg, capw, pool;
};

// regions of cpw chunks, <= kMaxRegions of them; a region's list slot holds 1/16 of its elements
// (or 2k / nreg if larger); the pool (8 shards) takes 1/8 of the bucket (or 3k)
Geo geo_for(int64_t n, int64_t k) {
  Geo g;
  g.nchunks = std::max<int64_t>(1, (n + kChunk - 1) / kChunk);
  g.cpw = (g.nchunks + kMaxRegions - 1) / kMaxRegions;
  g.nreg = (g.nchunks + g.cpw - 1) / g.cpw;
  const int64_t per = g.cpw * kChunk;
  int64_t capw = std::max<int64_t>(per / 16, (2 * k + g.nreg - 1) / g.nreg);
  capw = std::min<int64_t>(per, (capw + 63) / 64 * 64);
  g.capw = capw;
  g.pool = (std::max<int64_t>(n / 8, 3 * k) / kPoolShards + 64) / 64 * 64 * kPoolShards;
  return g;
}

int64_t ws_bytes_for(int64_t n, int64_t k) {
  const Geo g = geo_for(n, k);
  const int64_t entries = g.nreg * g.capw + g.pool;
  return (int64_t)sizeof(SelState) + 4 * (2 * g.nchunks + 3 * g.nreg) + 8 * entries + 64;
}

struct Ws {
  SelState* st;
  Regions R;
  Geo g;
};

Ws carve(at::Tensor& workspace, int64_t n, int64_t k) {
  const int64_t need = ws_bytes_for(n, k);
  TORCH_CHECK(workspace.is_cuda() && workspace.numel() * workspace.element_size() >= need,
              "workspace too small: need ", need, " bytes (topk_workspace_bytes(n, k))");
  static_assert(sizeof(SelState) % 16 == 0, "SelState keeps the arrays aligned");
  char* ws = (char*)workspace.data_ptr();
  TORCH_CHECK(reinterpret_cast<uintptr_t>(ws) % 16 == 0, "workspace must be 16-byte aligned");
  Ws w;
  w.g = geo_for(n, k);
  w.st = reinterpret_cast<SelState*>(ws);
  uint32_t* a = reinterpret_cast<uint32_t*>(ws + sizeof(SelState));
  const int64_t entries = w.g.nreg * w.g.capw + w.g.pool;
  TORCH_CHECK(entries < ((int64_t)1 << 32), "top-k list too large");
  w.R.coff = a;
  w.R.ccnt = a + w.g.nchunks;
  w.R.sfill = a + 2 * w.g.nchunks;
  w.R.cgt = w.R.sfill + w.g.nreg;
  w.R.ceq = w.R.cgt + w.g.nreg;
  w.R.lval = w.R.ceq + w.g.nreg;
  w.R.lidx = w.R.lval + entries;
  w.R.nchunks = w.g.nchunks;
  w.R.cpw = w.g.cpw;
  w.R.pool_off = w.g.nreg * w.g.capw;
  return w;
}

template <typename VT>
void launch_scan_write(hipStream_t stream, const float* src, float* rp, int64_t n, const Ws& w, int32_t* idx, VT* val,
                       uint32_t cap, int32_t* count_out) {
  hipLaunchKernelGGL(k_scan_regions, 1, 1024, 0, stream, w.R.cgt, w.R.ceq, (int)w.g.nreg, count_out, cap);
  hipLaunchKernelGGL(k_write_regions<VT>, (int)w.g.nreg, kBlock, 0, stream, src, rp, n, w.st, w.R, idx, val, cap);
}

// ------------------------------------------------------------------------------------------
// Small buckets (n <= kSmallMax, e.g. the reference notebook's n = 10 .. 10^4): ONE launch of one
// 1024-thread workgroup.  The folded values live in LDS (128 KB at n = 32768); the radix select
// runs its three digit passes (bits 30..20, 19..9, 8..0 of |x|) as LDS-atomic histograms (two
// copies, even / odd waves, for the clustered exponent digit) and picks each digit with a block
// suffix scan (every thread owns two bins).  Then each thread owns a contiguous index range of
// ODD length (so the 64 lanes of a wave start in 64 different LDS banks), counts keys > T and
// == T, two block scans give its tie admission (lowest index first) and its output offset, it
// writes its selected (index, value) pairs in index order and leaves each element's residual in
// LDS, and a last coalesced loop stores the residuals.  The multi-pass path above costs ~12
// launches, which dominates at these sizes.
// Speculative list (steady state, as P1 of the multi-pass path): with the previous call's
// threshold T' in the workspace, one atomic-free pass counts the keys >= 0.95 T' per thread range;
// if there are at least k and at most kCandCap of them, their indices are listed in index order
// (block scan offsets) and the three digit passes and the selection walk that short list instead
// of all n keys (the k-th largest key is >= 0.95 T' whenever >= k keys are).  Otherwise (first
// call, a shrinking gradient) the full passes run.  The final key is stored back as T'.
constexpr int kSmallMax = 32768;
constexpr int kSmallThreads = 1024;
constexpr int kCandCap = 3072;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (wv == 0) {
    uint32_t s = lane < kSmallThreads / 64 ? wsum[lane] : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(s, o, 64);
      if (lane >= o) s += y;
    }
    if (lane < kSmallThreads / 64) wsum[lane] = s;  // inclusive wave totals
  }
  __syncthreads();
  total = wsum[kSmallThreads / 64 - 1];
  const uint32_t before = wv ? wsum[wv - 1] : 0u;
  __syncthreads();  // wsum is reused by the next scan
  return before + x - v;
}

// h[bin] += 1 for every lane with ``want``.  Gradient magnitudes cluster in a few exponent bins,
// so plain LDS atomics serialise up to 64-way inside a wave on the top-digit pass: the first
// rounds let one leader lane add the popcount of all lanes that share its bin, the lanes left
// after them (diverse bins, little contention) add one each.
__device__ __forceinline__ void wave_hist_add(uint32_t* h, uint32_t bin, bool want) {
  const int lane = threadIdx.x & 63;
  uint64_t pending = __ballot(want);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (!pending) break;
    const int leader = __ffsll((unsigned long long)pending) - 1;
    const uint32_t lb = __shfl(bin, leader, 64);
    const uint64_t same = __ballot(want && bin == lb) & pending;
    if (lane == leader) atomicAdd(&h[lb], (uint32_t)__popcll(same));
    pending &= ~same;
  }
  if ((pending >> lane) & 1ull) atomicAdd(&h[bin], 1u);
}

template <typename VT>
__global__ __launch_bounds__(kSmallThreads) void k_topk_small(const float* __restrict__ g, float* __restrict__ resid,
                                                             int n, int k, int32_t* __restrict__ idx,
                                                             VT* __restrict__ val, int flags,
                                                             SelState* __restrict__ st) {
  // flags bit 0: wave-aggregated histogram adds (else one LDS atomic per lane); bit 1: all fold
  // loads issued before the LDS writes (else a strided loop); bit 2: no speculative list --
  // HIPPS_TOPK_SMALL=<flags> for A/B
  __shared__ __attribute__((aligned(16))) float sv[kSmallMax];
  __shared__ uint32_t hist[2][kHistBins];
  __shared__ uint32_t wsum[64];
  __shared__ uint32_t sel[2];  // chosen bin, keys above it
  __shared__ uint32_t cand[kCandCap];  // speculative list: indices in index order
  const int t = threadIdx.x, wv = t >> 6;
  const float ptf = __uint_as_float(st->prev_T & 0x7fffffffu);
  // The fold: one CU pulls up to 256 KB, so it is a latency problem -- a strided loop of dependent
  // single loads left one HBM round trip per 1024 elements exposed (~40 us cold at n = 32768).
  // Every lane issues all its 16-byte loads of g and r first (8 + 8 in flight), then writes LDS.
  {
    const bool vec = (flags & 2) && ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(resid)) & 15) == 0;
    const int n4 = vec ? n >> 2 : 0;
    constexpr int U = kSmallMax / 4 / kSmallThreads;  // 8 float4 per lane at n = kSmallMax
    float4 a[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = t + u * kSmallThreads;
      const int vc = v < n4 ? v : 0;  // clamped index, result discarded: no branch around a load
      a[u] = n4 ? reinterpret_cast<const float4*>(g)[vc] : make_float4(0.f, 0.f, 0.f, 0.f);
      r[u] = (n4 && resid) ? reinterpret_cast<const float4*>(resid)[vc] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = t + u * kSmallThreads;
      if (v < n4)
        reinterpret_cast<float4*>(sv)[v] = make_float4(a[u].x + r[u].x, a[u].y + r[u].y, a[u].z + r[u].z, a[u].w + r[u].w);
    }
    for (int i = 4 * n4 + t; i < n; i += kSmallThreads) sv[i] = g[i] + (resid ? resid[i] : 0.f);
  }
  // the walk: all n keys, or the speculative list of the keys >= 0.95 T'
  int N = n;
  bool listed = false;
  const int per0 = ((n + kSmallThreads - 1) / kSmallThreads) | 1;  // odd: bank-conflict-free LDS walks
  const int lo0 = min(n, t * per0), hi0 = min(n, lo0 + per0);
  if (!(flags & 4) && ptf > 0.f && ptf < __builtin_inff()) {  // (workgroup-uniform)
    const uint32_t lo_key = absbits(ptf * kSpecMargin);
    __syncthreads();  // sv complete
    uint32_t c = 0;
    for (int i = lo0; i < hi0; ++i) c += (__float_as_uint(sv[i]) & 0x7fffffffu) >= lo_key;
    uint32_t tot;
    uint32_t o = block_excl_scan(c, wsum, tot);
    if (tot >= (uint32_t)k && tot <= (uint32_t)kCandCap) {
      for (int i = lo0; i < hi0; ++i)
        if ((__float_as_uint(sv[i]) & 0x7fffffffu) >= lo_key) cand[o++] = (uint32_t)i;
      N = (int)tot;
      listed = true;
    }
  }
  auto at = [&](int j) -> int { return listed ? (int)cand[j] : j; };
  uint32_t prefix = 0, pmask = 0, rem = (uint32_t)k;
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    const int sh = pass == 0 ? 20 : pass == 1 ? 9 : 0, nb = pass == 2 ? 512 : 2048;
    for (int b = t; b < 2 * kHistBins; b += kSmallThreads) (&hist[0][0])[b] = 0u;
    __syncthreads();
    uint32_t* h = hist[pass == 0 ? (wv & 1) : 0];
    for (int i0 = 0; i0 < N; i0 += kSmallThreads) {  // whole waves iterate together (ballots)
      const int i = i0 + t;
      const uint32_t key = i < N ? __float_as_uint(sv[at(i)]) & 0x7fffffffu : 0u;
      const bool want = i < N && (key & pmask) == prefix;
      if (flags & 1) wave_hist_add(h, (key >> sh) & (nb - 1), want);
      else if (want) atomicAdd(&h[(key >> sh) & (nb - 1)], 1u);
    }
    __syncthreads();
    // thread t owns bins hi = nb-1-2t and lo = nb-2-2t (t < nb/2); exclusive scan from the top
    const int bh = nb - 1 - 2 * t, bl = bh - 1;
    uint32_t ch = 0, cl = 0;
    if (bl >= 0) {
      ch = hist[0][bh] + hist[1][bh];
      cl = hist[0][bl] + hist[1][bl];
    }
    uint32_t tot;
    const uint32_t above = block_excl_scan(ch + cl, wsum, tot);
    if (above < rem && above + ch + cl >= rem) {  // exactly one thread holds the rem-th key
      if (above + ch >= rem) {
        sel[0] = (uint32_t)bh;
        sel[1] = above;
      } else {
        sel[0] = (uint32_t)bl;
        sel[1] = above + ch;
      }
    }
    __syncthreads();
    prefix |= sel[0] << sh;
    pmask |= (uint32_t)(nb - 1) << sh;
    rem -= sel[1];
  }
  // prefix = T (the k-th largest key); admit rem keys == T, lowest index first
  const uint32_t T = prefix;
  if (t == 0) st->prev_T = T;  // the next call's speculative bound
  const int per = ((N + kSmallThreads - 1) / kSmallThreads) | 1;  // odd: bank-conflict-free LDS walks
  const int lo = min(N, t * per), hi = min(N, lo + per);
  uint32_t gt = 0, eq = 0;
  for (int j = lo; j < hi; ++j) {
    const uint32_t key = __float_as_uint(sv[at(j)]) & 0x7fffffffu;
    gt += key > T;
    eq += key == T;
  }
  uint32_t tot;
  const uint32_t eq_before = block_excl_scan(eq, wsum, tot);
  const uint32_t adm = eq_before >= rem ? 0u : min(eq, rem - eq_before);
  const uint32_t off = block_excl_scan(gt + adm, wsum, tot);
  uint32_t o = off, taken = 0;
  for (int j = lo; j < hi; ++j) {
    const int i = at(j);
    const float v = sv[i];
    const uint32_t key = __float_as_uint(v) & 0x7fffffffu;
    bool take = key > T;
    if (key == T && taken < adm) {
      take = true;
      ++taken;
    }
    if (take) {
      idx[o] = i;
      Vec4<VT>::store1(val, o, v);
      sv[i] = v - Vec4<VT>::load1(val, o);  // what the wire dropped (bf16 rounding), fed back
      ++o;
    }
  }
  if (resid) {
    __syncthreads();
    for (int i = t; i < n; i += kSmallThreads) resid[i] = sv[i];
  }
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
  Ws w = carve(workspace, n, k);
  float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->numel() == n && resid->scalar_type() == at::kFloat && resid->is_contiguous(), "residual");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(resid->data_ptr()) % 16 == 0, "residual must be 16-byte aligned");
    rp = resid->data_ptr<float>();
  }
  auto stream = c10::hip::getCurrentHIPStream();
  if (n <= kSmallMax) {  // one workgroup, one launch
    static const int sflags = [] {
      const char* e = std::getenv("HIPPS_TOPK_SMALL");
      return e ? std::atoi(e) : 2;  // measured: the wave-aggregated adds were slower (see k_topk_small)
    }();
    if (val.scalar_type() == at::kFloat)
      hipLaunchKernelGGL(k_topk_small<float>, 1, kSmallThreads, 0, stream, g.data_ptr<float>(), rp, (int)n, (int)k,
                         idx.data_ptr<int32_t>(), val.data_ptr<float>(), sflags, w.st);
    else
      hipLaunchKernelGGL(k_topk_small<uint16_t>, 1, kSmallThreads, 0, stream, g.data_ptr<float>(), rp, (int)n,
                         (int)k, idx.data_ptr<int32_t>(), (uint16_t*)val.data_ptr(), sflags, w.st);
    return;
  }
  const int nreg = (int)w.g.nreg;
  TORCH_CHECK(w.g.cpw <= kMaxCpw, "bucket too large for the region geometry");
  hipLaunchKernelGGL(k_sel_init, 1, kBlock, 0, stream, w.st, 0u, 0u, (uint32_t)k, (uint32_t)w.g.capw,
                     (uint32_t)(w.g.pool / kPoolShards), 1);
  // P1: fold + top-digit histogram + speculative ordered list (the only full pass)
  static const bool pf = [] {
    const char* e = std::getenv("HIPPS_TOPK_PF");
    return !(e && e[0] == '0');
  }();
  // picks inside the histogram launches (last-arriving block) instead of their own launches:
  // opt-in, HIPPS_TOPK_FOLD=1 -- measured slower on 25.6 M elements (236 vs 183 us cold,
  // profiles/codec/r4/): every region block's agent-scope release before its ticket writes back
  // its dirty L2 lines (the folded residual), where the separate launch boundary costs ~2 us
  static const bool fold = [] {
    const char* e = std::getenv("HIPPS_TOPK_FOLD");
    return e && e[0] == '1';
  }();
  const float* src = rp ? rp : g.data_ptr<float>();
  if (fold) {
    if (pf)
      hipLaunchKernelGGL((k_collect<true, true>), nreg, kBlock, 0, stream, g.data_ptr<float>(), rp, n, w.st, w.R, 0, 1);
    else
      hipLaunchKernelGGL((k_collect<true, false>), nreg, kBlock, 0, stream, g.data_ptr<float>(), rp, n, w.st, w.R, 0,
                         1);
    // P3 over the listed keys of bin B; its pick checks that the list reaches the remaining-th key
    hipLaunchKernelGGL(k_hist_list, nreg, kBlock, 0, stream, src, n, 9, 11, w.st, w.R, nreg, 0, kPickCheck, 1);
    // only after a miss (first call, shrinking gradients): re-list from bin B's edge, P3 again
    hipLaunchKernelGGL(k_collect<false>, nreg, kBlock, 0, stream, src, (float*)nullptr, n, w.st, w.R, 2, 0);
    hipLaunchKernelGGL(k_hist_list, nreg, kBlock, 0, stream, src, n, 9, 11, w.st, w.R, nreg, 1, kPickRetry, 2);
    // P4
    hipLaunchKernelGGL(k_hist_list, nreg, kBlock, 0, stream, src, n, 0, 9, w.st, w.R, nreg, 0, kPickFinal, 3);
  } else {
    hipLaunchKernelGGL(k_collect<true>, nreg, kBlock, 0, stream, g.data_ptr<float>(), rp, n, w.st, w.R, 0, 0);
    hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, 20, 11, w.st, 0);
    hipLaunchKernelGGL(k_hist_list, nreg, kBlock, 0, stream, src, n, 9, 11, w.st, w.R, nreg, 0, -1, 1);
    hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, 9, 11, w.st, kPickCheck);
    hipLaunchKernelGGL(k_collect<false>, nreg, kBlock, 0, stream, src, (float*)nullptr, n, w.st, w.R, 2, 0);
    hipLaunchKernelGGL(k_hist_list, nreg, kBlock, 0, stream, src, n, 9, 11, w.st, w.R, nreg, 1, -1, 2);
    hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, 9, 11, w.st, kPickRetry);
    hipLaunchKernelGGL(k_hist_list, nreg, kBlock, 0, stream, src, n, 0, 9, w.st, w.R, nreg, 0, -1, 3);
    hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, 0, 9, w.st, kPickFinal);
  }
  // P5: region counts, scan, ordered write
  hipLaunchKernelGGL(k_count_list, nreg, kBlock, 0, stream, src, n, w.st, w.R);
  if (val.scalar_type() == at::kFloat)
    launch_scan_write<float>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), val.data_ptr<float>(), (uint32_t)k,
                             nullptr);
  else
    launch_scan_write<uint16_t>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), (uint16_t*)val.data_ptr(),
                                (uint32_t)k, nullptr);
}

// ---- threshold sparsification (variable-size message, count in a device header) -----------
template <typename VT>
__global__ __launch_bounds__(kBlock) void k_scatter_acc_count(const int32_t* __restrict__ idx,
                                                              const VT* __restrict__ val,
                                                              const int32_t* count, int64_t cap,
                                                              float* __restrict__ acc, float gscale, int acquire) {
  if (acquire) acquire_remote_block();
  // the count header through the VECTOR path (a uniform `const __restrict__` load may go through
  // the scalar cache, which the acquire does not refresh)
  const int64_t k = min((int64_t)__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), cap);
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
  TORCH_CHECK(n >= 1, "empty bucket");
  TORCH_CHECK(val.numel() == cap && count.scalar_type() == at::kInt && count.numel() >= 1, "count/idx/val");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0, "g must be 16-byte aligned");
  TORCH_CHECK(n < (int64_t)1 << 31, "bucket must have < 2^31 elements");
  Ws w = carve(workspace, n, cap);
  auto stream = c10::hip::getCurrentHIPStream();
  float t = (float)std::fabs(tau);
  uint32_t tbits;
  std::memcpy(&tbits, &t, 4);
  float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->numel() == n && resid->scalar_type() == at::kFloat && resid->is_contiguous(), "residual");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(resid->data_ptr()) % 16 == 0, "residual must be 16-byte aligned");
    rp = resid->data_ptr<float>();
  }
  const int nreg = (int)w.g.nreg;
  // T = tau exactly, no ties admitted: every |x| > tau, in index order
  TORCH_CHECK(w.g.cpw <= kMaxCpw, "bucket too large for the region geometry");
  hipLaunchKernelGGL(k_sel_init, 1, kBlock, 0, stream, w.st, tbits, 0xffffffffu, 0u, (uint32_t)w.g.capw,
                     (uint32_t)(w.g.pool / kPoolShards), 0);
  hipLaunchKernelGGL(k_collect<false>, nreg, kBlock, 0, stream, g.data_ptr<float>(), rp, n, w.st, w.R, 1, 0);
  const float* src = rp ? rp : g.data_ptr<float>();
  if (val.scalar_type() == at::kFloat)
    launch_scan_write<float>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), val.data_ptr<float>(), (uint32_t)cap,
                             count.data_ptr<int32_t>());
  else
    launch_scan_write<uint16_t>(stream, src, rp, n, w, idx.data_ptr<int32_t>(), (uint16_t*)val.data_ptr(),
                                (uint32_t)cap, count.data_ptr<int32_t>());
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

void thresh_accumulate(at::Tensor count, at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale,
                       bool acquire) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat, "acc: f32 device tensor");
  const int64_t cap = idx.numel();
  if (cap == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  if (val.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(k_scatter_acc_count<float>, grid_for(cap), kBlock, 0, stream, idx.data_ptr<int32_t>(),
                       val.data_ptr<float>(), count.data_ptr<int32_t>(), cap, acc.data_ptr<float>(), (float)gscale,
                       (int)acquire);
  else
    hipLaunchKernelGGL(k_scatter_acc_count<uint16_t>, grid_for(cap), kBlock, 0, stream, idx.data_ptr<int32_t>(),
                       (const uint16_t*)val.data_ptr(), count.data_ptr<int32_t>(), cap, acc.data_ptr<float>(),
                       (float)gscale, (int)acquire);
}

int64_t topk_workspace_bytes(int64_t n, int64_t k) { return ws_bytes_for(n, k); }

void topk_accumulate(at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale, bool acquire) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat, "acc: f32 device tensor");
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.numel() == val.numel(), "idx/val mismatch");
  const int64_t k = idx.numel();
  if (k == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  const int grid = grid_for(k);
  if (val.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(k_scatter_acc<float>, grid, kBlock, 0, stream, idx.data_ptr<int32_t>(), val.data_ptr<float>(),
                       k, acc.data_ptr<float>(), (float)gscale, (int)acquire);
  else if (val.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(k_scatter_acc<uint16_t>, grid, kBlock, 0, stream, idx.data_ptr<int32_t>(),
                       (const uint16_t*)val.data_ptr(), k, acc.data_ptr<float>(), (float)gscale, (int)acquire);
  else
    TORCH_CHECK(false, "val must be f32 or bf16");
}

void topk_q8_accumulate(at::Tensor idx, at::Tensor q, at::Tensor scales, at::Tensor acc, double gscale,
                        bool acquire) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat, "acc: f32 device tensor");
  TORCH_CHECK(idx.scalar_type() == at::kInt && q.scalar_type() == at::kChar && idx.numel() == q.numel(), "idx/q");
  const int64_t k = idx.numel();
  TORCH_CHECK(scales.numel() == (k + 255) / 256, "scales size");
  if (k == 0) return;
  hipLaunchKernelGGL(k_scatter_acc_q8, grid_for(k), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     idx.data_ptr<int32_t>(), (const int8_t*)q.data_ptr(), scales.data_ptr<float>(), k,
                     acc.data_ptr<float>(), (float)gscale, (int)acquire);
}

void topk_q8_residual(at::Tensor idx, at::Tensor v, at::Tensor q, at::Tensor scales, at::Tensor resid) {
  const int64_t k = idx.numel();
  if (k == 0) return;
  hipLaunchKernelGGL(k_topk_q8_resid, grid_for(k), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     idx.data_ptr<int32_t>(), v.data_ptr<float>(), (const int8_t*)q.data_ptr(),
                     scales.data_ptr<float>(), k, resid.data_ptr<float>());
}

}  // namespace hipps
