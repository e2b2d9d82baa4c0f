// hipps — exact top-k magnitude sparsification (radix select + deterministic compaction).
//
// Device replacement for the external codec's encode (ps.py:94) when the codec is top-k.
// Output is a fixed-size message (k = ceil(ratio*n) known at plan time), so no size round-trip
// is needed: the reference's per-tensor Iallgather of lengths (mpi_comms.py:150-158, M1) goes
// away.  Wire: int32 idx[k] + val[k] (f32 or bf16), idx in ascending order.
//
// Pipeline (all stream-ordered, no host sync):
//   hist(bits 30..20) -> pick -> hist(19..9) -> pick -> hist(8..0) -> pick   (exact k-th |x|)
//   count per 1024-element chunk (> T, == T) -> exclusive scan -> write  (index order; ties
//   admitted lowest-index-first, so the message is bitwise deterministic)
// Optional error feedback: pass 0 folds the residual in (r <- g + r) and the write pass clears
// the residual at transmitted positions (r[i] <- x - wire(x)).
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cmath>
#include <cstring>

namespace hipps {

constexpr int kHistBins = 2048;
constexpr int kChunk = 1024;  // elements per compaction chunk = 256 lanes x float4

struct SelState {        // lives in a small device workspace
  uint32_t prefix;       // selected high bits of the k-th largest key
  uint32_t mask;         // which bits of prefix are decided
  uint32_t remaining;    // how many elements still to take inside the undecided bucket
  uint32_t pad;
  uint32_t hist[kHistBins];
};

__device__ __forceinline__ uint32_t absbits(float x) { return __float_as_uint(x) & 0x7fffffffu; }

__global__ __launch_bounds__(kBlock) void k_topk_init(SelState* __restrict__ st, uint32_t k) {
  if (threadIdx.x == 0) { st->prefix = 0; st->mask = 0; st->remaining = k; st->pad = 0; }
  for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) st->hist[b] = 0;
}

// pass p histogram over elements whose decided bits match prefix
__global__ __launch_bounds__(kBlock) void k_topk_hist(const float* __restrict__ g, float* __restrict__ resid,
                                                      int fold_resid, int64_t n, int lo, int nbits,
                                                      SelState* __restrict__ st) {
  __shared__ uint32_t h[kHistBins];
  const int nb = 1 << nbits;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
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
    if ((k0 & mask) == prefix) atomicAdd(&h[(k0 >> lo) & (nb - 1)], 1u);
    if ((k1 & mask) == prefix) atomicAdd(&h[(k1 >> lo) & (nb - 1)], 1u);
    if ((k2 & mask) == prefix) atomicAdd(&h[(k2 >> lo) & (nb - 1)], 1u);
    if ((k3 & mask) == prefix) atomicAdd(&h[(k3 >> lo) & (nb - 1)], 1u);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (nv << 2) + threadIdx.x; i < n; i += blockDim.x) {
      float x = src[i];
      if (fold_resid) { x += resid[i]; resid[i] = x; }
      const uint32_t k = absbits(x);
      if ((k & mask) == prefix) atomicAdd(&h[(k >> lo) & (nb - 1)], 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&st->hist[b], h[b]);
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

__device__ __forceinline__ void wg_counts(uint32_t gt, uint32_t eq, uint32_t* red, uint32_t& tg, uint32_t& te) {
  // 256 threads, 4 waves: reduce two counters
  float a = (float)gt, b = (float)eq;  // counts <= 4 per thread -> exact in f32 sums up to 2^24
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[w] = (uint32_t)a; red[4 + w] = (uint32_t)b; }
  __syncthreads();
  tg = red[0] + red[1] + red[2] + red[3];
  te = red[4] + red[5] + red[6] + red[7];
  __syncthreads();
}

__global__ __launch_bounds__(kBlock) void k_topk_count(const float* __restrict__ src, int64_t n,
                                                       const SelState* __restrict__ st, uint32_t* __restrict__ cgt,
                                                       uint32_t* __restrict__ ceq, int64_t nchunks) {
  __shared__ uint32_t red[8];
  const uint32_t T = st->prefix;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t i = c * kChunk + threadIdx.x * 4;
    uint32_t gt = 0, eq = 0;
    if (i + 4 <= n) {
      float4 x = *reinterpret_cast<const float4*>(src + i);
      const uint32_t k[4] = {absbits(x.x), absbits(x.y), absbits(x.z), absbits(x.w)};
#pragma unroll
      for (int j = 0; j < 4; ++j) { gt += k[j] > T; eq += k[j] == T; }
    } else {
      for (int j = 0; j < 4; ++j)
        if (i + j < n) { const uint32_t k = absbits(src[i + j]); gt += k > T; eq += k == T; }
    }
    uint32_t tg, te;
    wg_counts(gt, eq, red, tg, te);
    if (threadIdx.x == 0) { cgt[c] = tg; ceq[c] = te; }
  }
}

// exclusive scan of both count arrays in place (one workgroup; nchunks ~ n/1024)
__global__ __launch_bounds__(1024) void k_topk_scan(uint32_t* __restrict__ cgt, uint32_t* __restrict__ ceq,
                                                    int64_t nchunks, int32_t* __restrict__ count_out,
                                                    uint32_t cap) {
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
      uint32_t ag = threadIdx.x >= off ? sg[threadIdx.x - off] : 0;
      uint32_t ae = threadIdx.x >= off ? se[threadIdx.x - off] : 0;
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
                                                       const uint32_t* __restrict__ pgt,
                                                       const uint32_t* __restrict__ peq, int64_t nchunks,
                                                       int32_t* __restrict__ idx, VT* __restrict__ val, uint32_t cap) {
  __shared__ uint32_t wg[4], we[4];
  const uint32_t T = st->prefix, need_eq = st->remaining;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t i = c * kChunk + threadIdx.x * 4;
    float x[4];
    uint32_t k[4];
    if (i + 4 <= n) {
      float4 t = *reinterpret_cast<const float4*>(src + i);
      x[0] = t.x; x[1] = t.y; x[2] = t.z; x[3] = t.w;
    } else {
      for (int j = 0; j < 4; ++j) x[j] = (i + j < n) ? src[i + j] : 0.f;
    }
    for (int j = 0; j < 4; ++j) k[j] = (i + j < n) ? absbits(x[j]) : 0u;
    uint32_t gt = 0, eq = 0;
    for (int j = 0; j < 4; ++j) { gt += (i + j < n) && k[j] > T; eq += (i + j < n) && k[j] == T; }
    // exclusive scan of (gt, eq) across the workgroup in index order
    uint32_t sg = gt, se = eq;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t ag = __shfl_up(sg, o, 64), ae = __shfl_up(se, o, 64);
      if (lane >= o) { sg += ag; se += ae; }
    }
    if (lane == 63) { wg[w] = sg; we[w] = se; }
    __syncthreads();
    uint32_t bg = pgt[c], be = peq[c];
    for (int q = 0; q < w; ++q) { bg += wg[q]; be += we[q]; }
    bg += sg - gt;
    be += se - eq;
    for (int j = 0; j < 4; ++j) {
      if (i + j >= n) break;
      const bool isgt = k[j] > T, iseq = k[j] == T;
      const uint32_t pos = bg + (be < need_eq ? be : need_eq);
      if ((isgt || (iseq && be < need_eq)) && pos < cap) {
        idx[pos] = (int32_t)(i + j);
        Vec4<VT>::store1(val, pos, x[j]);
        if (resid) resid[i + j] = x[j] - Vec4<VT>::load1(val, pos);
      }
      bg += isgt;
      be += iseq;
    }
    __syncthreads();
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
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  const int64_t ws_bytes = (int64_t)sizeof(SelState) + 8 * nchunks + 16;
  TORCH_CHECK(workspace.is_cuda() && workspace.numel() * workspace.element_size() >= ws_bytes,
              "workspace too small: need ", ws_bytes, " bytes (topk_workspace_bytes)");
  float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->numel() == n && resid->scalar_type() == at::kFloat && resid->is_contiguous(), "residual");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(resid->data_ptr()) % 16 == 0, "residual must be 16-byte aligned");
    rp = resid->data_ptr<float>();
  }
  auto stream = c10::hip::getCurrentHIPStream();
  char* ws = (char*)workspace.data_ptr();
  SelState* st = reinterpret_cast<SelState*>(ws);
  uint32_t* cgt = reinterpret_cast<uint32_t*>(ws + sizeof(SelState));
  uint32_t* ceq = cgt + nchunks;
  hipLaunchKernelGGL(k_topk_init, 1, kBlock, 0, stream, st, (uint32_t)k);
  const int grid = grid_for(n >> 2);
  const int los[3] = {20, 9, 0}, bits[3] = {11, 11, 9};
  for (int p = 0; p < 3; ++p) {
    hipLaunchKernelGGL(k_topk_hist, grid, kBlock, 0, stream, g.data_ptr<float>(), rp, (int)(p == 0 && rp), n, los[p],
                       bits[p], st);
    hipLaunchKernelGGL(k_topk_pick, 1, kBlock, 0, stream, los[p], bits[p], st);
  }
  const float* src = rp ? rp : g.data_ptr<float>();
  const int cgrid = (int)std::min<int64_t>(nchunks, kMaxGrid);
  hipLaunchKernelGGL(k_topk_count, cgrid, kBlock, 0, stream, src, n, st, cgt, ceq, nchunks);
  hipLaunchKernelGGL(k_topk_scan, 1, 1024, 0, stream, cgt, ceq, nchunks, nullptr, 0u);
  if (val.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(k_topk_write<float>, cgrid, kBlock, 0, stream, src, rp, n, st, cgt, ceq, nchunks,
                       idx.data_ptr<int32_t>(), val.data_ptr<float>(), (uint32_t)k);
  else
    hipLaunchKernelGGL(k_topk_write<uint16_t>, cgrid, kBlock, 0, stream, src, rp, n, st, cgt, ceq, nchunks,
                       idx.data_ptr<int32_t>(), (uint16_t*)val.data_ptr(), (uint32_t)k);
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

__global__ void k_thresh_init(SelState* __restrict__ st, uint32_t tbits) {
  if (threadIdx.x == 0) { st->prefix = tbits; st->mask = 0xffffffffu; st->remaining = 0; st->pad = 0; }
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
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  TORCH_CHECK(workspace.numel() * workspace.element_size() >= (int64_t)sizeof(SelState) + 8 * nchunks + 16,
              "workspace too small");
  auto stream = c10::hip::getCurrentHIPStream();
  float* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    TORCH_CHECK(resid->numel() == n && resid->scalar_type() == at::kFloat, "residual");
    rp = resid->data_ptr<float>();
    hipLaunchKernelGGL(k_fold, grid_for(n >> 2), kBlock, 0, stream, g.data_ptr<float>(), rp, n);
  }
  char* ws = (char*)workspace.data_ptr();
  SelState* st = reinterpret_cast<SelState*>(ws);
  uint32_t* cgt = reinterpret_cast<uint32_t*>(ws + sizeof(SelState));
  uint32_t* ceq = cgt + nchunks;
  float t = (float)std::fabs(tau);
  uint32_t tbits;
  std::memcpy(&tbits, &t, 4);
  hipLaunchKernelGGL(k_thresh_init, 1, 64, 0, stream, st, tbits);
  const float* src = rp ? rp : g.data_ptr<float>();
  const int cgrid = (int)std::min<int64_t>(nchunks, kMaxGrid);
  hipLaunchKernelGGL(k_topk_count, cgrid, kBlock, 0, stream, src, n, st, cgt, ceq, nchunks);
  hipLaunchKernelGGL(k_topk_scan, 1, 1024, 0, stream, cgt, ceq, nchunks, count.data_ptr<int32_t>(), (uint32_t)cap);
  if (val.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(k_topk_write<float>, cgrid, kBlock, 0, stream, src, rp, n, st, cgt, ceq, nchunks,
                       idx.data_ptr<int32_t>(), val.data_ptr<float>(), (uint32_t)cap);
  else
    hipLaunchKernelGGL(k_topk_write<uint16_t>, cgrid, kBlock, 0, stream, src, rp, n, st, cgt, ceq, nchunks,
                       idx.data_ptr<int32_t>(), (uint16_t*)val.data_ptr(), (uint32_t)cap);
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

int64_t topk_workspace_bytes(int64_t n) {
  return (int64_t)sizeof(SelState) + 8 * ((n + kChunk - 1) / kChunk) + 16;
}

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
