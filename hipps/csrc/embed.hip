// hipps — BERT's input embedding (word + position + token type) in one pass each way.
//
// PyTorch's route is three gathers, two fp32 adds and a bf16 cast forward, and backward a cast,
// a broadcast reduction over the batch for the position table, and per table
// embedding_dense_backward: sort, segment offsets, partial sums, sum_and_scatter -- ~1 ms per
// BERT-base step at batch 32 x 512 (profiles/r6/bert_mlp/steady.txt: sum_and_scatter alone 415 us,
// all its token-type rows land on one segment).  Here:
//   forward   out[r] = bf16((word[ids[r]] + pos[r % S]) + type[tt[r]])      (PyTorch's add order)
//   backward  dpos[s] = sum_b dout[b S + s]                       (fixed order, no atomics)
//             dword[v] = sum over the rows r with ids[r] == v, in row order: the rows sorted by id
//                        (a stable sort, on the host side by torch.sort), one wave per id segment
//   (the token-type gradient of BERT's all-zero type ids is a column sum: xent.hip k_colsum)
// Deterministic: every output element is summed in a fixed order by one thread.
#include "common.h"

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

namespace hipps {

namespace {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void ld8f(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void st8f(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}
__device__ __forceinline__ void add8b(const uint16_t* p, float* f) {
  const u32x4 v = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] += __uint_as_float(v[j] << 16);
    f[2 * j + 1] += __uint_as_float(v[j] & 0xffff0000u);
  }
}

// one thread per (row, 8-element chunk)
__global__ __launch_bounds__(kBlock) void k_embed_fwd(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                      const float* __restrict__ word, const float* __restrict__ pos,
                                                      const float* __restrict__ typ, uint16_t* __restrict__ out,
                                                      int64_t R, int S, int D, int64_t V, int64_t T) {
  const int nch = D >> 3;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= R * nch) return;
  const int64_t r = i / nch;
  const int c = (int)(i - r * nch) * 8;
  const int64_t id = ids[r];
  const int64_t t = tt ? tt[r] : 0;
  float w[8], p[8], y[8];
  if (id < 0 || id >= V || t < 0 || t >= T) {  // out-of-range index: NaN row, no wild read
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = __int_as_float(0x7fc00000);
  } else {
    ld8f(word + id * D + c, w);
    ld8f(pos + (int64_t)(r % S) * D + c, p);
    ld8f(typ + t * D + c, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = (w[j] + p[j]) + y[j];
  }
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(y[2 * j], y[2 * j + 1]);
  *reinterpret_cast<u32x4*>(out + r * D + c) = o;
}

// dpos [P, D] fp32: rows s < S get sum_b dout[b S + s] (b ascending), rows >= S zero
__global__ __launch_bounds__(kBlock) void k_embed_pos_bwd(const uint16_t* __restrict__ dout, float* __restrict__ dpos,
                                                          int B, int S, int P, int D) {
  const int nch = D >> 3;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (int64_t)P * nch) return;
  const int s = (int)(i / nch);
  const int c = (int)(i - (int64_t)s * nch) * 8;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (s < S) {
    for (int b = 0; b < B; ++b) add8b(dout + ((int64_t)b * S + s) * D + c, a);
  }
  st8f(dpos + (int64_t)s * D + c, a);
}

// one wave per position i of the id-sorted rows; the wave at the start of a segment (first i with
// that id) sums its rows in sorted (= row, stable sort) order and writes the table row; the others
// exit.  dtab is zero-filled by the caller (ids that never occur keep a zero gradient).
__global__ __launch_bounds__(64) void k_embed_seg_bwd(const uint16_t* __restrict__ dout,
                                                      const int64_t* __restrict__ sid, const int64_t* __restrict__ perm,
                                                      float* __restrict__ dtab, int64_t R, int D, int64_t V) {
  const int64_t i = blockIdx.x;
  const int64_t v = sid[i];
  if ((i > 0 && sid[i - 1] == v) || v < 0 || v >= V) return;
  int64_t e = i + 1;
  while (e < R && sid[e] == v) ++e;
  const int nch = D >> 3;
  for (int ch = threadIdx.x; ch < nch; ch += 64) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int64_t j = i;
    for (; j + 4 <= e; j += 4) {  // four row loads in flight
      const int64_t r0 = perm[j], r1 = perm[j + 1], r2 = perm[j + 2], r3 = perm[j + 3];
      const u32x4 v0 = *reinterpret_cast<const u32x4*>(dout + r0 * D + ch * 8);
      const u32x4 v1 = *reinterpret_cast<const u32x4*>(dout + r1 * D + ch * 8);
      const u32x4 v2 = *reinterpret_cast<const u32x4*>(dout + r2 * D + ch * 8);
      const u32x4 v3 = *reinterpret_cast<const u32x4*>(dout + r3 * D + ch * 8);
      const u32x4 vs[4] = {v0, v1, v2, v3};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          a[2 * k] += __uint_as_float(vs[q][k] << 16);
          a[2 * k + 1] += __uint_as_float(vs[q][k] & 0xffff0000u);
        }
    }
    for (; j < e; ++j) add8b(dout + perm[j] * D + ch * 8, a);
    st8f(dtab + v * D + ch * 8, a);
  }
}

void check_tab(const at::Tensor& t, int64_t D, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 2 && t.size(1) == D &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "embed: ", what, " must be a contiguous 16-byte aligned fp32 [rows, D] device tensor");
}
}  // namespace

// ids int64 [B, S]; tt (optional) int64 [B, S]; word [V, D], pos [P >= S, D], typ [T, D] fp32;
// out bf16 [B, S, D]
void embed_forward(at::Tensor ids, c10::optional<at::Tensor> tt, at::Tensor word, at::Tensor pos, at::Tensor typ,
                   at::Tensor out) {
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.dim() == 2,
              "embed: ids must be contiguous int64 [B, S]");
  const int64_t D = word.size(1), R = ids.numel(), S = ids.size(1);
  TORCH_CHECK(D % 8 == 0 && D >= 8, "embed: D % 8 == 0");
  check_tab(word, D, "word");
  check_tab(pos, D, "pos");
  check_tab(typ, D, "type");
  TORCH_CHECK(S <= pos.size(0), "embed: sequence longer than the position table");
  const int64_t* ttp = nullptr;
  if (tt.has_value() && tt->defined()) {
    TORCH_CHECK(tt->is_cuda() && tt->scalar_type() == at::kLong && tt->is_contiguous() && tt->numel() == R,
                "embed: type ids must be contiguous int64 shaped like ids");
    ttp = tt->data_ptr<int64_t>();
  }
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.numel() == R * D &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "embed: out must be contiguous bf16 [B, S, D]");
  const int64_t n = R * (D / 8);
  if (n == 0) return;
  hipLaunchKernelGGL(k_embed_fwd, (int)((n + kBlock - 1) / kBlock), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     ids.data_ptr<int64_t>(), ttp, word.data_ptr<float>(), pos.data_ptr<float>(), typ.data_ptr<float>(),
                     (uint16_t*)out.data_ptr(), R, (int)S, (int)D, word.size(0), typ.size(0));
}

// dout bf16 [B, S, D] -> dpos fp32 [P, D]
void embed_pos_backward(at::Tensor dout, at::Tensor dpos, int64_t B, int64_t S) {
  const int64_t D = dpos.size(1), P = dpos.size(0);
  check_tab(dpos, D, "dpos");
  TORCH_CHECK(dout.is_cuda() && dout.scalar_type() == at::kBFloat16 && dout.is_contiguous() &&
                  dout.numel() == B * S * D && reinterpret_cast<uintptr_t>(dout.data_ptr()) % 16 == 0 && S <= P &&
                  D % 8 == 0,
              "embed: dout must be contiguous bf16 [B, S, D], S <= P");
  const int64_t n = P * (D / 8);
  if (n == 0) return;
  hipLaunchKernelGGL(k_embed_pos_bwd, (int)((n + kBlock - 1) / kBlock), kBlock, 0, c10::hip::getCurrentHIPStream(),
                     (const uint16_t*)dout.data_ptr(), dpos.data_ptr<float>(), (int)B, (int)S, (int)P, (int)D);
}

// dout bf16 [R, D]; sid / perm int64 [R] (ids sorted stably, and their rows); dtab fp32 [V, D]
// zero-filled by the caller
void embed_seg_backward(at::Tensor dout, at::Tensor sid, at::Tensor perm, at::Tensor dtab) {
  const int64_t D = dtab.size(1), R = sid.numel();
  check_tab(dtab, D, "dtab");
  TORCH_CHECK(sid.is_cuda() && perm.is_cuda() && sid.scalar_type() == at::kLong && perm.scalar_type() == at::kLong &&
                  sid.is_contiguous() && perm.is_contiguous() && perm.numel() == R,
              "embed: sorted ids / rows must be contiguous int64 [R]");
  TORCH_CHECK(dout.is_cuda() && dout.scalar_type() == at::kBFloat16 && dout.is_contiguous() && dout.numel() == R * D &&
                  reinterpret_cast<uintptr_t>(dout.data_ptr()) % 16 == 0 && D % 8 == 0,
              "embed: dout must be contiguous bf16 [R, D]");
  TORCH_CHECK(R < ((int64_t)1 << 31), "embed: rows");
  if (R == 0) return;
  hipLaunchKernelGGL(k_embed_seg_bwd, (int)R, 64, 0, c10::hip::getCurrentHIPStream(), (const uint16_t*)dout.data_ptr(),
                     sid.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), dtab.data_ptr<float>(), R, (int)D,
                     dtab.size(0));
}

}  // namespace hipps
