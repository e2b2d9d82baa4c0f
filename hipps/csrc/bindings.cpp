// hipps._C — pybind11 bindings for the CDNA4 kernels and the native PS runtime.
#include <torch/extension.h>
#include <vector>

namespace hipps {
// flat.hip
void aggregate(const std::vector<at::Tensor>& slots, at::Tensor acc, double gscale, bool accumulate, bool acquire);
void copy_acquire(at::Tensor src, at::Tensor dst);
void convert(at::Tensor src, at::Tensor dst, double scale);
void gather_flat(const std::vector<at::Tensor>& srcs, at::Tensor table, at::Tensor dst, double scale);
void transpose_cast(at::Tensor src, at::Tensor dst, at::Tensor tiles);
void sgd_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, c10::optional<at::Tensor> buf,
              c10::optional<at::Tensor> pub, bool zero_src, double lr, double wd, double momentum, double dampening,
              bool nesterov, bool first, c10::optional<at::Tensor> mask, c10::optional<at::Tensor> csteps,
              double lookahead);
void adam_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, at::Tensor exp_avg,
               at::Tensor exp_avg_sq, c10::optional<at::Tensor> max_exp_avg_sq, c10::optional<at::Tensor> pub,
               bool zero_src, double lr, double beta1, double beta2, double eps, double wd, int64_t step,
               bool amsgrad, bool torch_mode, c10::optional<at::Tensor> mask, c10::optional<at::Tensor> csteps);
// quant.hip
void q8_encode(at::Tensor x, c10::optional<at::Tensor> resid, at::Tensor q, at::Tensor scales, bool stochastic,
               int64_t seed);
void q8_aggregate(const std::vector<at::Tensor>& qs, const std::vector<at::Tensor>& ss, at::Tensor acc, double gscale,
                  bool accumulate, bool acquire);
// topk.hip
void topk_encode(at::Tensor g, c10::optional<at::Tensor> resid, int64_t k, at::Tensor idx, at::Tensor val,
                 at::Tensor workspace);
int64_t topk_workspace_bytes(int64_t n, int64_t k);
void topk_accumulate(at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale, bool acquire);
void topk_q8_accumulate(at::Tensor idx, at::Tensor q, at::Tensor scales, at::Tensor acc, double gscale,
                        bool acquire);
void topk_q8_residual(at::Tensor idx, at::Tensor v, at::Tensor q, at::Tensor scales, at::Tensor resid);
void thresh_encode(at::Tensor g, c10::optional<at::Tensor> resid, double tau, at::Tensor count, at::Tensor idx,
                   at::Tensor val, at::Tensor workspace);
void thresh_accumulate(at::Tensor count, at::Tensor idx, at::Tensor val, at::Tensor acc, double gscale,
                       bool acquire);
void copy_counted(at::Tensor src, at::Tensor dst, int64_t idx_off, int64_t val_off, int64_t val_esz, int64_t cap);
// norm.hip
void bn_forward_train(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y, at::Tensor weight, at::Tensor bias,
                      c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var, at::Tensor mean,
                      at::Tensor invstd, at::Tensor scale, at::Tensor shift, int64_t C, double eps, double momentum,
                      bool relu, c10::optional<at::Tensor> mask_out);
void bn_apply(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y, at::Tensor scale, at::Tensor shift, int64_t C,
              bool relu);
void bn_backward(at::Tensor dy, at::Tensor x, c10::optional<at::Tensor> y, int64_t mask_mode, at::Tensor weight,
                 at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift, at::Tensor dx,
                 c10::optional<at::Tensor> dres, at::Tensor dweight, at::Tensor dbias, int64_t C,
                 c10::optional<at::Tensor> mask_in);
void bn_forward_partials(at::Tensor part, int64_t nrb, at::Tensor x, c10::optional<at::Tensor> res, at::Tensor y,
                         at::Tensor weight, at::Tensor bias, c10::optional<at::Tensor> running_mean,
                         c10::optional<at::Tensor> running_var, at::Tensor mean, at::Tensor invstd, at::Tensor scale,
                         at::Tensor shift, int64_t C, double eps, double momentum, bool relu,
                         c10::optional<at::Tensor> mask_out);
void bn_backward_partials(at::Tensor part, int64_t nrb, at::Tensor dy, at::Tensor x, int64_t mask_mode,
                          at::Tensor weight, at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift,
                          at::Tensor dx, c10::optional<at::Tensor> dres, at::Tensor dweight, at::Tensor dbias, int64_t C,
                          c10::optional<at::Tensor> mask_in, int64_t unr);
// gemm.hip
int64_t conv1x1_mtiles(int64_t M);
void conv1x1_forward(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part, int64_t Hi,
                     int64_t Wi, int64_t stride, c10::optional<at::Tensor> add, c10::optional<at::Tensor> add_mask,
                     c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_bits,
                     c10::optional<at::Tensor> bn_mean, c10::optional<at::Tensor> bn_invstd,
                     c10::optional<at::Tensor> bn_scale, c10::optional<at::Tensor> bn_shift,
                     c10::optional<at::Tensor> pro_scale, c10::optional<at::Tensor> pro_shift);
// norm.hip dual BN (downsample block tail)
void bn_dual_forward(at::Tensor part3, int64_t nrb3, at::Tensor partd, int64_t nrbd, at::Tensor x3, at::Tensor xd,
                     at::Tensor z, at::Tensor mask, at::Tensor w3, at::Tensor b3, at::Tensor rm3, at::Tensor rv3,
                     at::Tensor mean3, at::Tensor invstd3, at::Tensor scale3, at::Tensor shift3, at::Tensor wd,
                     at::Tensor bd, at::Tensor rmd, at::Tensor rvd, at::Tensor meand, at::Tensor invstdd,
                     at::Tensor scaled, at::Tensor shiftd, int64_t C, double eps3, double mom3, double epsd,
                     double momd);
void bn_dual_backward(c10::optional<at::Tensor> part3, int64_t nrb3, at::Tensor dz, at::Tensor x3, at::Tensor xd,
                      at::Tensor mask, at::Tensor w3, at::Tensor mean3, at::Tensor invstd3, at::Tensor wd,
                      at::Tensor meand, at::Tensor invstdd, at::Tensor dx3, at::Tensor dxd, at::Tensor dw3,
                      at::Tensor db3, at::Tensor dwd, at::Tensor dbd, int64_t C, int64_t unr);
// gemm2.hip
at::Tensor gemm2_dgrad_s2(at::Tensor dy, at::Tensor wf, at::Tensor dx, int64_t bm, int64_t bn,
                          c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_bits,
                          c10::optional<at::Tensor> bn_mean, c10::optional<at::Tensor> bn_invstd,
                          c10::optional<at::Tensor> bn_scale, c10::optional<at::Tensor> bn_shift);
int64_t gemm2_mtiles(int64_t M, int64_t N, int64_t K, int64_t bm);
void gemm2_conv(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part,
                c10::optional<at::Tensor> add, c10::optional<at::Tensor> add_mask, int64_t Hi, int64_t Wi,
                int64_t stride, int64_t KH, int64_t KW, int64_t pad, int64_t bm, int64_t bn,
                c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_bits, c10::optional<at::Tensor> bn_mean,
                c10::optional<at::Tensor> bn_invstd, c10::optional<at::Tensor> bn_scale,
                c10::optional<at::Tensor> bn_shift, int64_t stages, bool add_s2,
                c10::optional<at::Tensor> pro_scale, c10::optional<at::Tensor> pro_shift,
                c10::optional<at::Tensor> bias, c10::optional<at::Tensor> gelu_pre, int64_t gelu);
void gemm2_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
                 int64_t Hi, int64_t Wi, int64_t cfg, int64_t stages,
                 c10::optional<at::Tensor> pro_scale, c10::optional<at::Tensor> pro_shift, int64_t sdiv);
// pool.hip
void maxpool3s2_forward(at::Tensor x, at::Tensor y, at::Tensor code, c10::optional<at::Tensor> scale,
                        c10::optional<at::Tensor> shift);
void bn_finalize_partials(at::Tensor part, int64_t nrb, int64_t M, at::Tensor weight, at::Tensor bias,
                          c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
                          at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift, int64_t C, double eps,
                          double momentum);
void maxpool3s2_backward(at::Tensor dy, at::Tensor code, at::Tensor dx);
std::vector<at::Tensor> xent_forward(at::Tensor logits, at::Tensor labels, int64_t ignore_index);
void colsum_fold(at::Tensor part, at::Tensor out);
void colsum_bf16(at::Tensor x, at::Tensor out);
std::vector<at::Tensor> attn_forward(at::Tensor q, at::Tensor k, at::Tensor v, bool causal, double scale,
                                     c10::optional<at::Tensor> kvlen);
std::vector<at::Tensor> attn_backward(at::Tensor dout, at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o,
                                      at::Tensor lse, bool causal, double scale, c10::optional<at::Tensor> kvlen,
                                      c10::optional<at::Tensor> dq_out, c10::optional<at::Tensor> dk_out,
                                      c10::optional<at::Tensor> dv_out);
void swiglu_forward(at::Tensor a, at::Tensor b, at::Tensor c);
void ln_forward(at::Tensor x, at::Tensor w, at::Tensor b, at::Tensor y, at::Tensor mean, at::Tensor rstd, double eps);
void ln_backward(at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor rstd, at::Tensor w, at::Tensor dx,
                 at::Tensor dw, at::Tensor db, c10::optional<at::Tensor> dxsum);
void embed_forward(at::Tensor ids, c10::optional<at::Tensor> tt, at::Tensor word, at::Tensor pos, at::Tensor typ,
                   at::Tensor out);
void embed_pos_backward(at::Tensor dout, at::Tensor dpos, int64_t B, int64_t S);
void embed_seg_backward(at::Tensor dout, at::Tensor sid, at::Tensor perm, at::Tensor dtab);
void rms_forward(at::Tensor x, at::Tensor w, at::Tensor y, at::Tensor rstd, double eps, c10::optional<at::Tensor> add,
                 c10::optional<at::Tensor> xsum);
void rms_backward(at::Tensor dy, at::Tensor x, at::Tensor rstd, at::Tensor w, at::Tensor dx, at::Tensor dw,
                  c10::optional<at::Tensor> dres, c10::optional<at::Tensor> dx16);
void swiglu_backward(at::Tensor g, at::Tensor a, at::Tensor b, at::Tensor da, at::Tensor db);
void rope_apply(at::Tensor x, at::Tensor y, at::Tensor cs, at::Tensor sn, int64_t S, int64_t hd, double sign);
void swiglu_rows_forward(at::Tensor y, at::Tensor c);
void swiglu_rows_backward(at::Tensor g, at::Tensor y, at::Tensor dy);
void xent_backward(at::Tensor logits, at::Tensor labels, at::Tensor lse, at::Tensor gout, double scale,
                   int64_t ignore_index, at::Tensor dx, c10::optional<at::Tensor> count);
void bn_finalize_bwd_partials(at::Tensor part, int64_t nrb, int64_t M, at::Tensor weight, at::Tensor mean,
                              at::Tensor invstd, at::Tensor dweight, at::Tensor dbias, at::Tensor coef);
void conv1x1_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw, int64_t Hi, int64_t Wi, int64_t stride,
                   c10::optional<at::Tensor> pro_scale, c10::optional<at::Tensor> pro_shift);
void bn_forward_stats(at::Tensor x, at::Tensor weight, at::Tensor bias, c10::optional<at::Tensor> running_mean,
                      c10::optional<at::Tensor> running_var, at::Tensor mean, at::Tensor invstd, at::Tensor scale,
                      at::Tensor shift, int64_t C, double eps, double momentum);
void conv_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw, int64_t KH, int64_t KW, int64_t stride, int64_t pad);
void convkxk_forward(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part, int64_t stride,
                     int64_t pad);
// stem.hip
int64_t stem_mtiles(int64_t imgs, int64_t Ho);
void stem_forward(at::Tensor x, at::Tensor w, at::Tensor y, c10::optional<at::Tensor> part);
void stem_wgrad(at::Tensor dy, at::Tensor x, at::Tensor dw);
void stem_bnpool_backward(at::Tensor dp, at::Tensor code, at::Tensor y, at::Tensor x, at::Tensor bn_weight,
                          at::Tensor mean, at::Tensor invstd, at::Tensor scale, at::Tensor shift, at::Tensor dbn_w,
                          at::Tensor dbn_b, at::Tensor dw, bool materialize_dy, bool quad);
namespace rt {
void pull_params(at::Tensor sel, int64_t pub_ver, int64_t buf_ver, int64_t reading, int64_t applied, at::Tensor pub,
                 int64_t stride, int64_t npub, bool bf16, at::Tensor dst, int64_t ring_slot, int64_t tries);
void pull_select(at::Tensor sel, int64_t pub_ver, int64_t buf_ver, int64_t reading, int64_t applied, int64_t npub,
                 int64_t tries);
void pull_copy_ptrs(at::Tensor sel, std::vector<int64_t> ptrs, int64_t npub, bool bf16, at::Tensor dst, int64_t lo,
                    int64_t hi, c10::optional<at::Tensor> shadow);
void pull_copy_b_ptrs(at::Tensor selb, at::Tensor boff, std::vector<int64_t> ptrs, int64_t npub, bool bf16,
                      at::Tensor dst, int64_t lo, int64_t hi, c10::optional<at::Tensor> shadow, int64_t b0,
                      int64_t b1);
void pull_copy(at::Tensor sel, at::Tensor pub, int64_t stride, int64_t npub, bool bf16, at::Tensor dst, int64_t lo,
               int64_t hi, c10::optional<at::Tensor> shadow);
void pull_done(at::Tensor sel, int64_t pub_ver, int64_t buf_ver, int64_t reading, int64_t applied, int64_t ring_slot);
void pull_select_b(at::Tensor selb, int64_t bpub, int64_t bbuf, int64_t reading_b, int64_t applied, int64_t npub,
                   int64_t tries);
void pull_copy_b(at::Tensor selb, at::Tensor boff, at::Tensor pub, int64_t stride, int64_t npub, bool bf16,
                 at::Tensor dst, int64_t lo, int64_t hi, c10::optional<at::Tensor> shadow);
void emu_sweep(at::Tensor wr, at::Tensor rd, at::Tensor sink, int64_t stamp, int64_t blocks);
void pull_done_b(at::Tensor selb, int64_t bpub, int64_t bbuf, int64_t reading_b, int64_t applied, at::Tensor sel,
                 int64_t ring_slot);
void bind_control(pybind11::module& m);
void bind_rccl(pybind11::module& m);
void bind_ipc(pybind11::module& m);
void bind_psloop(pybind11::module& m);
void bind_trace(pybind11::module& m);
}  // namespace rt
}  // namespace hipps

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "hipps native kernels (gfx950) and parameter-server runtime";
  m.def("aggregate", &hipps::aggregate, "acc (+)= gscale * sum_w slots[w] (rank order)", py::arg("slots"),
        py::arg("acc"), py::arg("gscale"), py::arg("accumulate"), py::arg("acquire") = false);
  m.def("copy_acquire", &hipps::copy_acquire, "dst = src after a system-scope acquire (bytes written by a peer GPU)");
  m.def("convert", &hipps::convert, "dst = scale * src with f32/bf16 conversion");
  m.def("gather_flat", &hipps::gather_flat, "multi-tensor gather (+cast) of grads into a flat buffer");
  m.def("transpose_cast", &hipps::transpose_cast, "multi-matrix dst[c,r] = bf16(src[r,c]) (1x1 dgrad weights)");
  m.def("sgd_step", &hipps::sgd_step, "fused decode+sum+SGD (reference ps.py:197-214 math)", pybind11::arg("grads"),
        pybind11::arg("gscale"), pybind11::arg("p"), pybind11::arg("buf"), pybind11::arg("pub"),
        pybind11::arg("zero_src"), pybind11::arg("lr"), pybind11::arg("wd"), pybind11::arg("momentum"),
        pybind11::arg("dampening"), pybind11::arg("nesterov"), pybind11::arg("first"),
        pybind11::arg("mask") = pybind11::none(), pybind11::arg("csteps") = pybind11::none(),
        pybind11::arg("lookahead") = 0.0);
  m.def("adam_step", &hipps::adam_step, "fused decode+sum+Adam (reference ps.py:217-261 math)",
        pybind11::arg("grads"), pybind11::arg("gscale"), pybind11::arg("p"), pybind11::arg("exp_avg"),
        pybind11::arg("exp_avg_sq"), pybind11::arg("max_exp_avg_sq"), pybind11::arg("pub"), pybind11::arg("zero_src"),
        pybind11::arg("lr"), pybind11::arg("beta1"), pybind11::arg("beta2"), pybind11::arg("eps"), pybind11::arg("wd"),
        pybind11::arg("step"), pybind11::arg("amsgrad"), pybind11::arg("torch_mode"),
        pybind11::arg("mask") = pybind11::none(), pybind11::arg("csteps") = pybind11::none());
  m.def("q8_encode", &hipps::q8_encode, "per-256-block absmax int8 quantization (+EF, +stochastic)");
  m.def("q8_aggregate", &hipps::q8_aggregate, "acc (+)= gscale * sum_w dequant(q_w, s_w)", py::arg("qs"), py::arg("ss"),
        py::arg("acc"), py::arg("gscale"), py::arg("accumulate"), py::arg("acquire") = false);
  m.def("topk_encode", &hipps::topk_encode, "exact top-k |g| (radix select) -> idx asc, val");
  m.def("topk_workspace_bytes", &hipps::topk_workspace_bytes, py::arg("n"), py::arg("k") = 0);
  m.def("topk_accumulate", &hipps::topk_accumulate, "acc[idx] += gscale * val", py::arg("idx"), py::arg("val"),
        py::arg("acc"), py::arg("gscale"), py::arg("acquire") = false);
  m.def("topk_q8_accumulate", &hipps::topk_q8_accumulate, "acc[idx] += gscale * deq(q)", py::arg("idx"), py::arg("q"),
        py::arg("scales"), py::arg("acc"), py::arg("gscale"), py::arg("acquire") = false);
  m.def("topk_q8_residual", &hipps::topk_q8_residual, "EF: r[idx] += v - deq(q)");
  m.def("thresh_encode", &hipps::thresh_encode, "variable-size |x|>tau sparsification, device count header");
  m.def("thresh_accumulate", &hipps::thresh_accumulate, "acc[idx[:count]] += gscale * val[:count]", py::arg("count"),
        py::arg("idx"), py::arg("val"), py::arg("acc"), py::arg("gscale"), py::arg("acquire") = false);
  m.def("copy_counted", &hipps::copy_counted, "copy a [count | idx | val] message moving only count entries");
  m.def("bn_forward_train", &hipps::bn_forward_train, "fused channels-last BN train fwd (+res) (+relu)");
  m.def("bn_apply", &hipps::bn_apply, "y = act(x*scale + shift (+res))");
  m.def("bn_backward", &hipps::bn_backward, "fused BN bwd with relu-mask recompute (+dres)");
  m.def("bn_forward_partials", &hipps::bn_forward_partials, "BN fwd finalize+apply from producer-reduced partials");
  m.def("bn_backward_partials", &hipps::bn_backward_partials, "BN bwd finalize+apply from consumer-reduced partials",
        py::arg("part"), py::arg("nrb"), py::arg("dy"), py::arg("x"), py::arg("mask_mode"), py::arg("weight"),
        py::arg("mean"), py::arg("invstd"), py::arg("scale"), py::arg("shift"), py::arg("dx"), py::arg("dres"),
        py::arg("dweight"), py::arg("dbias"), py::arg("C"), py::arg("mask_in"), py::arg("unr") = 0);
  m.def("conv1x1_mtiles", &hipps::conv1x1_mtiles);
  m.def("bn_dual_forward", &hipps::bn_dual_forward,
        "z = relu(bn3(x3) + bnd(xd)) from producer partials: two finalizes + one apply (downsample block)");
  m.def("bn_dual_backward", &hipps::bn_dual_backward,
        "backward of bn_dual_forward: dx3 + the downsample BN's reduction in one pass, then dxd",
        py::arg("part3"), py::arg("nrb3"), py::arg("dz"), py::arg("x3"), py::arg("xd"), py::arg("mask"), py::arg("w3"),
        py::arg("mean3"), py::arg("invstd3"), py::arg("wd"), py::arg("meand"), py::arg("invstdd"), py::arg("dx3"),
        py::arg("dxd"), py::arg("dw3"), py::arg("db3"), py::arg("dwd"), py::arg("dbd"), py::arg("C"),
        py::arg("unr") = 4);
  m.def("gemm2_mtiles", &hipps::gemm2_mtiles, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("bm") = 0);
  m.def("gemm2_conv", &hipps::gemm2_conv, "second-generation MFMA conv GEMM (LDS-DMA staged, 256-row tiles)",
        py::arg("x"), py::arg("w"), py::arg("y"), py::arg("part") = py::none(), py::arg("add") = py::none(),
        py::arg("add_mask") = py::none(), py::arg("Hi"), py::arg("Wi"), py::arg("stride") = 1, py::arg("KH") = 1,
        py::arg("KW") = 1, py::arg("pad") = 0, py::arg("bm") = 0, py::arg("bn") = 0, py::arg("bn_x") = py::none(),
        py::arg("bn_bits") = py::none(), py::arg("bn_mean") = py::none(), py::arg("bn_invstd") = py::none(),
        py::arg("bn_scale") = py::none(), py::arg("bn_shift") = py::none(), py::arg("stages") = 2,
        py::arg("add_s2") = false, py::arg("pro_scale") = py::none(), py::arg("pro_shift") = py::none(),
        py::arg("bias") = py::none(), py::arg("gelu_pre") = py::none(), py::arg("gelu") = 0);
  m.def("gemm2_dgrad_s2", &hipps::gemm2_dgrad_s2,
        "stride-2 3x3 input gradient as four output-parity implicit GEMMs (+ BN-backward reduction)",
        py::arg("dy"), py::arg("wf"), py::arg("dx"), py::arg("bm") = 128, py::arg("bn") = 128,
        py::arg("bn_x") = py::none(), py::arg("bn_bits") = py::none(), py::arg("bn_mean") = py::none(),
        py::arg("bn_invstd") = py::none(), py::arg("bn_scale") = py::none(), py::arg("bn_shift") = py::none());
  m.def("gemm2_wgrad", &hipps::gemm2_wgrad, "conv weight gradient on the LDS-DMA MFMA core (split-M slabs)",
        py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"),
        py::arg("Hi"), py::arg("Wi"), py::arg("cfg") = 0, py::arg("stages") = 2, py::arg("pro_scale") = py::none(),
        py::arg("pro_shift") = py::none(), py::arg("sdiv") = 1);
  m.def("conv1x1_forward", &hipps::conv1x1_forward,
        "MFMA 1x1 conv (NHWC GEMM) with fused BN-stats epilogue and optional (+ add * mask) epilogue",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("part"), pybind11::arg("Hi"),
        pybind11::arg("Wi"), pybind11::arg("stride"), pybind11::arg("add") = pybind11::none(),
        pybind11::arg("add_mask") = pybind11::none(), pybind11::arg("bn_x") = pybind11::none(),
        pybind11::arg("bn_bits") = pybind11::none(), pybind11::arg("bn_mean") = pybind11::none(),
        pybind11::arg("bn_invstd") = pybind11::none(), pybind11::arg("bn_scale") = pybind11::none(),
        pybind11::arg("bn_shift") = pybind11::none(), pybind11::arg("pro_scale") = pybind11::none(),
        pybind11::arg("pro_shift") = pybind11::none());
  m.def("convkxk_forward", &hipps::convkxk_forward,
        "MFMA KxK conv forward (implicit GEMM, channels-last bf16) with optional BN-statistics epilogue",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("part") = pybind11::none(),
        pybind11::arg("stride") = 1, pybind11::arg("pad") = 1);
  m.def("stem_mtiles", &hipps::stem_mtiles, "number of BN partial-statistic columns of stem_forward");
  m.def("stem_forward", &hipps::stem_forward,
        "ResNet stem 7x7/s2/p3 3->64 conv forward on MFMA (channels-last bf16), optional BN-statistics epilogue",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("part") = pybind11::none());
  m.def("stem_bnpool_backward", &hipps::stem_bnpool_backward,
        "backward of maxpool(relu(bn(stem(x)))): BN parameter grads + stem weight grad, no pool gradient "
        "materialised (the BN input gradient only with materialize_dy)",
        py::arg("dp"), py::arg("code"), py::arg("y"), py::arg("x"), py::arg("bn_weight"), py::arg("mean"),
        py::arg("invstd"), py::arg("scale"), py::arg("shift"), py::arg("dbn_w"), py::arg("dbn_b"), py::arg("dw"),
        py::arg("materialize_dy") = false, py::arg("quad") = true);
  m.def("stem_wgrad", &hipps::stem_wgrad, "ResNet stem 7x7/s2/p3 weight gradient on MFMA (fp32 dW, deterministic)");
  m.def("conv_wgrad", &hipps::conv_wgrad, "MFMA KxK conv weight gradient (implicit GEMM, split-M, fp32 dW)");
  m.def("maxpool3s2_forward", &hipps::maxpool3s2_forward,
        "3x3/s2/p1 max pool, channels-last bf16, 4-bit tap codes; optional BN-apply + ReLU prologue",
        pybind11::arg("x"), pybind11::arg("y"), pybind11::arg("code"), pybind11::arg("scale") = pybind11::none(),
        pybind11::arg("shift") = pybind11::none());
  m.def("bn_finalize_partials", &hipps::bn_finalize_partials,
        "BN train-mode finalize from producer partial sums (mean/invstd/scale/shift + running stats)");
  m.def("embed_forward", &hipps::embed_forward, "word + position + type embedding -> bf16 rows (embed.hip)");
  m.def("embed_pos_backward", &hipps::embed_pos_backward, "position-table gradient: fixed-order batch sum");
  m.def("embed_seg_backward", &hipps::embed_seg_backward, "table gradient over id-sorted rows, one wave per id");
  m.def("rms_forward", &hipps::rms_forward,
        "RMSNorm forward: fp32 / bf16 rows -> bf16, fp32 rstd; optional fused residual add (ln.hip)", py::arg("x"),
        py::arg("w"), py::arg("y"), py::arg("rstd"), py::arg("eps"), py::arg("add") = py::none(),
        py::arg("xsum") = py::none());
  m.def("rms_backward", &hipps::rms_backward,
        "RMSNorm backward: dx in x's dtype, fp32 weight gradient; optional residual gradient in, bf16 twin out "
        "(ln.hip)",
        py::arg("dy"), py::arg("x"), py::arg("rstd"), py::arg("w"), py::arg("dx"), py::arg("dw"),
        py::arg("dres") = py::none(), py::arg("dx16") = py::none());
  m.def("ln_forward", &hipps::ln_forward, "LayerNorm forward, bf16 rows, fp32 weight / bias / mean / rstd (ln.hip)");
  m.def("ln_backward", &hipps::ln_backward,
        "LayerNorm backward: bf16 dx, fp32 weight / bias gradients, optional column sum of dx (ln.hip)",
        py::arg("dy"), py::arg("x"), py::arg("mean"), py::arg("rstd"), py::arg("w"), py::arg("dx"), py::arg("dw"),
        py::arg("db"), py::arg("dxsum") = py::none());
  m.def("swiglu_forward", &hipps::swiglu_forward, "c = silu(a) * b, bf16 (act.hip)");
  m.def("swiglu_backward", &hipps::swiglu_backward, "gradients of silu(a) * b w.r.t. a and b, bf16 (act.hip)");
  m.def("rope_apply", &hipps::rope_apply, py::arg("x"), py::arg("y"), py::arg("cos"), py::arg("sin"), py::arg("S"),
        py::arg("hd"), py::arg("sign") = 1.0, "rotary embedding of interleaved pairs, fp32 tables (act.hip)");
  m.def("swiglu_rows_forward", &hipps::swiglu_rows_forward,
        "c = silu(y[:, :F]) * y[:, F:] for a packed [rows, 2F] gate/up projection (act.hip)");
  m.def("swiglu_rows_backward", &hipps::swiglu_rows_backward,
        "packed [rows, 2F] gradient (da | db) of swiglu_rows_forward (act.hip)");
  m.def("colsum_fold", &hipps::colsum_fold, "fixed-order sum of fp32 partial rows [P, N] -> [N]");
  m.def("colsum_bf16", &hipps::colsum_bf16, "fp32 column sums of a bf16 [rows, cols] matrix (bias gradients)");
  m.def("attn_forward", &hipps::attn_forward, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("causal"),
        py::arg("scale"), py::arg("kv_len") = py::none(),
        "flash attention forward on MFMA: q [B,Sq,Hq,D], k/v [B,Sk,Hkv,D] bf16 -> (o, lse) (attn.hip)");
  m.def("attn_backward", &hipps::attn_backward, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"),
        py::arg("o"), py::arg("lse"), py::arg("causal"), py::arg("scale"), py::arg("kv_len") = py::none(),
        py::arg("dq_out") = py::none(), py::arg("dk_out") = py::none(), py::arg("dv_out") = py::none(),
        "flash attention backward (deterministic dQ and dK/dV kernels) -> (dq, dk, dv) (attn.hip)");
  m.def("xent_forward", &hipps::xent_forward,
        "fused softmax cross-entropy over bf16 logits: (mean loss, counted rows, per-row log-sum-exp)");
  m.def("xent_backward", &hipps::xent_backward, py::arg("logits"), py::arg("labels"), py::arg("lse"), py::arg("gout"),
        py::arg("scale"), py::arg("ignore_index"), py::arg("dx"), py::arg("count") = py::none(),
        "cross-entropy gradient (softmax - onehot) * g * scale / count, bf16");
  m.def("bn_finalize_bwd_partials", &hipps::bn_finalize_bwd_partials,
        "BN backward finalize from partial sums (dweight, dbias, dx coefficients [3, C])");
  m.def("maxpool3s2_backward", &hipps::maxpool3s2_backward, "3x3/s2/p1 max pool backward (gather form, no atomics)");
  m.def("conv1x1_wgrad", &hipps::conv1x1_wgrad, "MFMA 1x1 conv weight gradient (tr_b16 LDS reads, split-M)",
        pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("dw"), pybind11::arg("Hi"), pybind11::arg("Wi"),
        pybind11::arg("stride"), pybind11::arg("pro_scale") = pybind11::none(),
        pybind11::arg("pro_shift") = pybind11::none());
  m.def("bn_forward_stats", &hipps::bn_forward_stats,
        "training BatchNorm statistics only (reduce + finalize: mean, invstd, scale, shift, running stats); the "
        "apply is left to a consumer's prologue");
  m.def("pull_params", &hipps::rt::pull_params,
        "GPU-time AsySG-InCon pull: select newest published version, copy it, release the reader word");
  m.def("pull_select", &hipps::rt::pull_select, "GPU-time pull, stage 1: choose the version, announce the reader");
  m.def("emu_sweep", &hipps::rt::emu_sweep, py::arg("wr"), py::arg("rd"), py::arg("sink"), py::arg("stamp"),
        py::arg("blocks") = 8, "emulated remote traffic: write sweep of wr + read sweep of rd from a few workgroups");
  m.def("pull_copy_ptrs", &hipps::rt::pull_copy_ptrs, py::arg("sel"), py::arg("ptrs"), py::arg("npub"),
        py::arg("bf16"), py::arg("dst"), py::arg("lo"), py::arg("hi"), py::arg("shadow") = py::none());
  m.def("pull_copy_b_ptrs", &hipps::rt::pull_copy_b_ptrs, py::arg("selb"), py::arg("boff"), py::arg("ptrs"),
        py::arg("npub"), py::arg("bf16"), py::arg("dst"), py::arg("lo"), py::arg("hi"),
        py::arg("shadow") = py::none(), py::arg("b0") = 0, py::arg("b1") = -1);
  m.def("pull_copy", &hipps::rt::pull_copy, py::arg("sel"), py::arg("pub"), py::arg("stride"), py::arg("npub"),
        py::arg("bf16"), py::arg("dst"), py::arg("lo"), py::arg("hi"), py::arg("shadow") = py::none(),
        "GPU-time pull, stage 2: copy params[lo, hi) of the chosen version (+ their bf16 shadow)");
  m.def("pull_done", &hipps::rt::pull_done, "GPU-time pull, stage 3: release the reader word, record the version");
  m.def("pull_select_b", &hipps::rt::pull_select_b, "bucket-granular pull, stage 1: newest version per bucket");
  m.def("pull_copy_b", &hipps::rt::pull_copy_b, py::arg("selb"), py::arg("boff"), py::arg("pub"), py::arg("stride"),
        py::arg("npub"), py::arg("bf16"), py::arg("dst"), py::arg("lo"), py::arg("hi"), py::arg("shadow") = py::none(),
        "bucket-granular pull, stage 2: copy each bucket's selected slot (+ its bf16 shadow)");
  m.def("pull_done_b", &hipps::rt::pull_done_b, "bucket-granular pull, stage 3: release, record min version");
  hipps::rt::bind_control(m);
  hipps::rt::bind_rccl(m);
  hipps::rt::bind_ipc(m);
  hipps::rt::bind_psloop(m);
  hipps::rt::bind_trace(m);
}
