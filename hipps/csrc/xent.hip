// hipps — fused softmax cross-entropy over bf16 logits (the transformer LM / MLM heads).
//
// PyTorch's route for a bf16 head in mixed precision is logits.float() (a full fp32 copy of a
// [tokens, vocab] tensor: 2 GB for BERT-base's MLM head at batch 32 x 512, 4.2 GB for Llama-3 at
// 4 x 2048 x 128256), log_softmax over it (another fp32 write), and in the backward a softmax
// gradient in fp32 plus the cast back: ~5 full passes of fp32 traffic.  Here the forward reads
// each bf16 row ONCE with an online max / sum-exp (fp32 math), keeping only the row's
// log-sum-exp; the backward reads the row once more and writes the bf16 gradient
// (softmax - onehot) * g / n.  One workgroup per row, 16-byte loads, fp32 accumulation.
#include "common.h"

#include <mutex>
#include <unordered_map>

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <algorithm>

namespace hipps {

namespace {
constexpr int kXBlock = 256;

__device__ __forceinline__ void online(float& m, float& s, float x) {
  if (x == -INFINITY) return;  // (masked logits)
  if (x > m) {
    s = s * __expf(m - x) + 1.f;
    m = x;
  } else {
    s += __expf(x - m);
  }
}

// (m, s) of two partial online-softmax states merged
__device__ __forceinline__ void merge(float& m, float& s, float m2, float s2) {
  const float mm = fmaxf(m, m2);
  s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
  m = mm;
}

__device__ __forceinline__ void block_lse(float& m, float& s) {
  __shared__ float sm[kXBlock / 64], ss[kXBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    merge(m, s, m2, s2);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  m = sm[0];
  s = ss[0];
#pragma unroll
  for (int q = 1; q < kXBlock / 64; ++q) merge(m, s, sm[q], ss[q]);
}
}  // namespace

// one 16-byte chunk (8 bf16) into the running (max, sum-exp): one rescale per chunk, not per element
__device__ __forceinline__ void online8(float& m, float& s, const uint4 u) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  float x[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x[2 * j] = __uint_as_float(w[j] << 16);
    x[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
  const float cm = fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])), fmaxf(fmaxf(x[4], x[5]), fmaxf(x[6], x[7])));
  if (cm == -INFINITY) return;  // (all masked)
  if (cm > m) {
    s *= __expf(m - cm);  // m == -inf: s == 0 stays 0
    m = cm;
  }
  float a = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) a += __expf(x[j] - m);
  s += a;
}

// elements before a row's first 16-byte boundary (rows of an odd-sized vocab start at any 2-byte
// offset: BERT's V = 30522 puts 3 of every 4 rows off the boundary, which used to send the whole
// row down the 2-byte scalar path)
__device__ __forceinline__ int64_t head_elems(const uint16_t* row, int64_t V) {
  const int64_t h = ((16 - (reinterpret_cast<uintptr_t>(row) & 15)) & 15) >> 1;
  return h < V ? h : V;
}

// loss[r] = lse(x_r) - x_r[label_r] (0 for ignored rows), lse[r] kept for the backward
__global__ __launch_bounds__(kXBlock) void k_xent_fwd(const uint16_t* __restrict__ x, const int64_t* __restrict__ labels,
                                                      int64_t V, int64_t ignore, float* __restrict__ loss,
                                                      float* __restrict__ lse) {
  const int64_t r = blockIdx.x;
  const uint16_t* row = x + r * V;
  float m = -INFINITY, s = 0.f;
  const int64_t h = head_elems(row, V);
  if (threadIdx.x < h) online(m, s, bf16_to_f32(row[threadIdx.x]));
  const uint4* vrow = reinterpret_cast<const uint4*>(row + h);
  const int64_t nv = (V - h) >> 3;
  // software pipeline: the next two chunks are in flight while the current two are reduced
  const uint4 z = make_uint4(0xff80ff80u, 0xff80ff80u, 0xff80ff80u, 0xff80ff80u);  // -inf x 8
  int64_t v = threadIdx.x;
  uint4 a = v < nv ? vrow[v] : z, b = v + kXBlock < nv ? vrow[v + kXBlock] : z;
  for (; v < nv; v += 2 * kXBlock) {
    const int64_t n0 = v + 2 * kXBlock, n1 = v + 3 * kXBlock;
    const uint4 na = n0 < nv ? vrow[n0] : z, nb = n1 < nv ? vrow[n1] : z;
    online8(m, s, a);
    online8(m, s, b);
    a = na;
    b = nb;
  }
  for (int64_t i = h + nv * 8 + threadIdx.x; i < V; i += kXBlock) online(m, s, bf16_to_f32(row[i]));
  block_lse(m, s);
  if (threadIdx.x == 0) {
    const float l = m + __logf(s);
    const int64_t lab = labels[r];
    lse[r] = l;
    loss[r] = (lab == ignore || lab < 0 || lab >= V) ? 0.f : l - bf16_to_f32(row[lab]);
  }
}

// dx_r = (softmax(x_r) - onehot(label_r)) * scale (0 rows for ignored labels)
__global__ __launch_bounds__(kXBlock) void k_xent_bwd(const uint16_t* __restrict__ x, const int64_t* __restrict__ labels,
                                                      const float* __restrict__ lse, int64_t V, int64_t ignore,
                                                      const float* __restrict__ gscale, float scale,
                                                      const float* __restrict__ ndiv, uint16_t* __restrict__ dx) {
  const int64_t r = blockIdx.x;
  const uint16_t* row = x + r * V;
  uint16_t* drow = dx + r * V;
  const int64_t lab = labels[r];
  const bool skip = lab == ignore || lab < 0 || lab >= V;
  const float l = lse[r];
  const float k = skip ? 0.f : scale * gscale[0] / (ndiv ? ndiv[0] : 1.f);
  // the vector loop needs x and dx rows at the same offset from a 16-byte boundary (true for
  // tensors of one shape allocated by the caching allocator); then peel the head elements
  const bool vec = ((reinterpret_cast<uintptr_t>(row) ^ reinterpret_cast<uintptr_t>(drow)) & 15) == 0;
  const int64_t h = vec ? head_elems(row, V) : V;
  for (int64_t i = threadIdx.x; i < h; i += kXBlock)
    drow[i] = f32_to_bf16((__expf(bf16_to_f32(row[i]) - l) - (i == lab ? 1.f : 0.f)) * k);
  if (!vec) return;
  const int64_t nv = (V - h) >> 3;
  const uint4* vrow = reinterpret_cast<const uint4*>(row + h);
  uint4* vd = reinterpret_cast<uint4*>(drow + h);
  auto one = [&](int64_t v, const uint4 u) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    float g[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g[2 * j] = __expf(__uint_as_float(w[j] << 16) - l);
      g[2 * j + 1] = __expf(__uint_as_float(w[j] & 0xffff0000u) - l);
    }
    const int64_t i0 = h + v * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (g[j] - (i0 + j == lab ? 1.f : 0.f)) * k;
    vd[v] = make_uint4(pack_bf16x2(g[0], g[1]), pack_bf16x2(g[2], g[3]), pack_bf16x2(g[4], g[5]), pack_bf16x2(g[6], g[7]));
  };
  // software pipeline: the next two chunks' loads are issued before this pair's stores, so the
  // wait for them (vmcnt counts stores too) does not wait for the stores' completion
  int64_t v = threadIdx.x;
  uint4 a = v < nv ? vrow[v] : uint4{}, b = v + kXBlock < nv ? vrow[v + kXBlock] : uint4{};
  for (; v < nv; v += 2 * kXBlock) {
    const int64_t n0 = v + 2 * kXBlock, n1 = v + 3 * kXBlock;
    const uint4 na = n0 < nv ? vrow[n0] : uint4{}, nb = n1 < nv ? vrow[n1] : uint4{};
    one(v, a);
    if (v + kXBlock < nv) one(v + kXBlock, b);
    a = na;
    b = nb;
  }
  for (int64_t i = h + nv * 8 + threadIdx.x; i < V; i += kXBlock)
    drow[i] = f32_to_bf16((__expf(bf16_to_f32(row[i]) - l) - (i == lab ? 1.f : 0.f)) * k);
}

// mean over the rows that carry a loss (label not ignored, inside [0, V)): one workgroup sums
// the per-row losses and counts the rows in a fixed order (deterministic); out = [mean, count].
// Folds the ~8 PyTorch scalar kernels of "mask, count, sum, divide" (each a host round of
// dispatch at the forward -> backward turn, where the GPU waits on the host) into one launch.
__global__ __launch_bounds__(kXBlock) void k_xent_mean(const float* __restrict__ loss, const int64_t* __restrict__ labels,
                                                       int64_t R, int64_t V, int64_t ignore, float* __restrict__ mean,
                                                       float* __restrict__ count) {
  __shared__ float ss[kXBlock / 64];
  __shared__ int sn[kXBlock / 64];
  float s = 0.f;
  int n = 0;
  for (int64_t r = threadIdx.x; r < R; r += kXBlock) {
    const int64_t lab = labels[r];
    if (!(lab == ignore || lab < 0 || lab >= V)) {
      s += loss[r];
      ++n;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    n += __shfl_xor(n, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    ss[w] = s;
    sn[w] = n;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    int c = 0;
#pragma unroll
    for (int q = 0; q < kXBlock / 64; ++q) {
      a += ss[q];
      c += sn[q];
    }
    mean[0] = a / (float)c;  // every row ignored -> 0 / 0 = NaN, as F.cross_entropy
    count[0] = (float)c;
  }
}

// logits: bf16 [R, V] contiguous; labels int64 [R]; returns (mean loss f32 [], row count f32 [1],
// lse f32 [R] for the backward)
std::vector<at::Tensor> xent_forward(at::Tensor logits, at::Tensor labels, int64_t ignore_index) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kBFloat16 && logits.dim() == 2 && logits.is_contiguous(),
              "xent: logits must be a contiguous bf16 [rows, vocab] device tensor");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                  labels.numel() == logits.size(0), "xent: labels must be int64 [rows] on the device");
  const int64_t R = logits.size(0), V = logits.size(1);
  TORCH_CHECK(V > 0 && R > 0 && R < (int64_t(1) << 24), "xent: sizes");
  auto f32 = logits.options().dtype(at::kFloat);
  at::Tensor rows = at::empty({R}, f32), lse = at::empty({R}, f32), mean = at::empty({}, f32), count = at::empty({1}, f32);
  auto stream = c10::hip::getCurrentHIPStream();
  hipLaunchKernelGGL(k_xent_fwd, (int)R, kXBlock, 0, stream, (const uint16_t*)logits.data_ptr(),
                     labels.data_ptr<int64_t>(), V, ignore_index, rows.data_ptr<float>(), lse.data_ptr<float>());
  hipLaunchKernelGGL(k_xent_mean, 1, kXBlock, 0, stream, rows.data_ptr<float>(), labels.data_ptr<int64_t>(), R, V,
                     ignore_index, mean.data_ptr<float>(), count.data_ptr<float>());
  return {mean, count, lse};
}

// dx = (softmax - onehot) * gout[0] * scale / count[0] (count: xent_forward's row count, or
// None for 1), bf16 like the logits
void xent_backward(at::Tensor logits, at::Tensor labels, at::Tensor lse, at::Tensor gout, double scale,
                   int64_t ignore_index, at::Tensor dx, c10::optional<at::Tensor> count) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kBFloat16 && logits.dim() == 2 && logits.is_contiguous(),
              "xent: logits must be a contiguous bf16 [rows, vocab] device tensor");
  TORCH_CHECK(dx.sizes() == logits.sizes() && dx.scalar_type() == at::kBFloat16 && dx.is_contiguous(), "xent: dx");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0) && lse.numel() == logits.size(0) &&
                  lse.scalar_type() == at::kFloat, "xent: labels / lse");
  TORCH_CHECK(gout.is_cuda() && gout.scalar_type() == at::kFloat && gout.numel() == 1, "xent: gout f32 scalar");
  const float* nd = nullptr;
  if (count.has_value() && count->defined()) {
    TORCH_CHECK(count->is_cuda() && count->scalar_type() == at::kFloat && count->numel() == 1, "xent: count f32 [1]");
    nd = count->data_ptr<float>();
  }
  const int64_t R = logits.size(0), V = logits.size(1);
  if (R == 0) return;
  hipLaunchKernelGGL(k_xent_bwd, (int)R, kXBlock, 0, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(), V,
                     ignore_index, gout.data_ptr<float>(), (float)scale, nd, (uint16_t*)dx.data_ptr());
}

}  // namespace hipps

// ------------------------------------------------------------------------------------------
// Column sums of a bf16 [R, N] matrix into fp32 [N] (a Linear layer's bias gradient, dy.sum(0)):
// PyTorch's reduce kernel ran these at ~0.7 TB/s (1.8 ms of a BERT-base step over 73 biases,
// profiles/r4/r4n/).  Pass 1: block (column tile of 64, row chunk) -- 8 lanes x 16-byte loads
// span the tile, 32 row lanes stride the chunk, fp32 sums combined through LDS in a fixed order
// -> partial[chunk][col]; pass 2 sums the chunks in order (deterministic).
namespace hipps {

// fixed-order sum of the P partial rows of 64 columns (4 waves, 8 loads in flight per lane)
__device__ __forceinline__ void colsum_fold(const float* __restrict__ part, int64_t P, int64_t N, int64_t c,
                                            float* __restrict__ out, float (*red)[64]) {
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t cc = c < N ? c : N - 1;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  int64_t p = wv;
  for (; p + 28 < P; p += 32) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = part[(p + 4 * j) * N + cc];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  for (; p < P; p += 4) acc[0] += part[p * N + cc];
  float a = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  red[wv][lane] = a;
  __syncthreads();
  if (wv == 0 && c < N) out[c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// tickets (optional, opt-in: see colsum_bf16): one arrival counter per 64-column tile, zero on
// entry; the block of a tile that arrives last (agent-scope release / acquire, correct for any
// placement over the XCDs) folds the tile's P partial rows into out and re-arms the counter --
// one launch instead of a part + fin pair
__global__ __launch_bounds__(256) void k_colsum_part(const uint16_t* __restrict__ x, int64_t R, int64_t N,
                                                     int64_t rows_per, float* __restrict__ part,
                                                     uint32_t* __restrict__ tickets, float* __restrict__ out) {
  __shared__ float red[32][65];
  __shared__ float red4[4][64];
  __shared__ uint32_t lastf;
  const int t = threadIdx.x, g = t & 7, rl = t >> 3;
  const int64_t c0 = (int64_t)blockIdx.x * 64 + g * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per, r1 = min(R, r0 + rows_per);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (c0 < N) {
    int64_t r = r0 + rl;
    for (; r + 32 < r1; r += 64) {  // two rows in flight per lane
      const uint4 a = *reinterpret_cast<const uint4*>(x + r * N + c0);
      const uint4 b = *reinterpret_cast<const uint4*>(x + (r + 32) * N + c0);
      const uint32_t wa[4] = {a.x, a.y, a.z, a.w}, wb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[2 * j] += __uint_as_float(wa[j] << 16) + __uint_as_float(wb[j] << 16);
        s[2 * j + 1] += __uint_as_float(wa[j] & 0xffff0000u) + __uint_as_float(wb[j] & 0xffff0000u);
      }
    }
    for (; r < r1; r += 32) {
      const uint4 a = *reinterpret_cast<const uint4*>(x + r * N + c0);
      const uint32_t wa[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[2 * j] += __uint_as_float(wa[j] << 16);
        s[2 * j + 1] += __uint_as_float(wa[j] & 0xffff0000u);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][g * 8 + j] = s[j];
  __syncthreads();
  if (t < 64) {
    float a = 0.f;
    for (int q = 0; q < 32; ++q) a += red[q][t];
    const int64_t c = (int64_t)blockIdx.x * 64 + t;
    if (c < N) part[(int64_t)blockIdx.y * N + c] = a;
  }
  if (tickets == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t old = __hip_atomic_fetch_add(tickets + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t last = old == gridDim.y - 1 ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(tickets + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
    }
    lastf = last;
  }
  __syncthreads();
  if (lastf == 0u) return;
  colsum_fold(part, gridDim.y, N, (int64_t)blockIdx.x * 64 + (t & 63), out, red4);
}

// 64 columns per block: lane (t & 63) owns a column, the 4 waves take every 4th partial row with
// 8 loads in flight per lane (a dependent walk over ~170 rows ran ~37 us), then a fixed-order
// combine of the 4 wave sums in LDS (deterministic)
__global__ __launch_bounds__(256) void k_colsum_fin(const float* __restrict__ part, int64_t P, int64_t N,
                                                    float* __restrict__ out) {
  __shared__ float red[4][64];
  colsum_fold(part, P, N, (int64_t)blockIdx.x * 64 + (threadIdx.x & 63), out, red);
}

namespace {
// per-stream arrival counters of the one-launch column sum (zeroed once; each fold re-arms its own)
constexpr int64_t kColsumTickets = 4096;
uint32_t* colsum_tickets(hipStream_t s, const at::Tensor& like) {
  static std::mutex mu;
  static std::unordered_map<hipStream_t, at::Tensor> bufs;
  std::lock_guard<std::mutex> g(mu);
  auto it = bufs.find(s);
  if (it == bufs.end()) {
    at::Tensor t = at::zeros({kColsumTickets}, like.options().dtype(at::kInt));
    it = bufs.emplace(s, t).first;
  }
  return reinterpret_cast<uint32_t*>(it->second.data_ptr());
}
}  // namespace

// out[N] (f32) = part.sum(0), fixed order, for fp32 partial rows [P, N] (a producing kernel's
// per-tile column sums, e.g. gemm2's kGeluBS)
void colsum_fold(at::Tensor part, at::Tensor out) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 2 && part.is_contiguous(),
              "colsum_fold: part must be a contiguous fp32 [P, N] device tensor");
  const int64_t P = part.size(0), N = part.size(1);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == N,
              "colsum_fold: out");
  if (N == 0) return;
  hipLaunchKernelGGL(k_colsum_fin, (int)((N + 63) / 64), 256, 0, c10::hip::getCurrentHIPStream(),
                     part.data_ptr<float>(), P, N, out.data_ptr<float>());
}

// out[N] (f32) = x.sum(0) for a contiguous bf16 [R, N], N % 8 == 0, 16-byte aligned
void colsum_bf16(at::Tensor x, at::Tensor out) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(),
              "colsum: x must be a contiguous bf16 [rows, cols] device tensor");
  const int64_t R = x.size(0), N = x.size(1);
  TORCH_CHECK(N % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "colsum: cols % 8, 16-byte aligned");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == N, "colsum: out");
  if (N == 0) return;
  const int64_t ct = (N + 63) / 64;
  int64_t P = std::max<int64_t>(1, std::min<int64_t>(2048 / ct, (R + 63) / 64));
  const int64_t rows_per = (R + P - 1) / P;
  P = std::max<int64_t>(1, (R + rows_per - 1) / rows_per);
  auto stream = c10::hip::getCurrentHIPStream();
  at::Tensor part = at::empty({P, N}, out.options());
  // opt-in (HIPPS_COLSUM_ONE=1): measured SLOWER in the BERT-base step, 735 k vs 794 k tokens/s on
  // one box (profiles/r6/bert_mlp/colsum_one_*.json) -- each of the ~2000 blocks' agent-scope
  // release writes back its XCD's dirty L2 lines, which costs the neighbouring kernels far more
  // than the fin launch it saves
  static const bool one = [] {
    const char* e = std::getenv("HIPPS_COLSUM_ONE");
    return e && e[0] == '1';
  }();
  if (one && ct <= kColsumTickets) {
    hipLaunchKernelGGL(k_colsum_part, dim3((unsigned)ct, (unsigned)P), 256, 0, stream, (const uint16_t*)x.data_ptr(),
                       R, N, rows_per, part.data_ptr<float>(), colsum_tickets(stream, out), out.data_ptr<float>());
    return;
  }
  hipLaunchKernelGGL(k_colsum_part, dim3((unsigned)ct, (unsigned)P), 256, 0, stream, (const uint16_t*)x.data_ptr(), R,
                     N, rows_per, part.data_ptr<float>(), nullptr, nullptr);
  hipLaunchKernelGGL(k_colsum_fin, (int)ct, 256, 0, stream, part.data_ptr<float>(), P, N,
                     out.data_ptr<float>());
}

}  // namespace hipps
