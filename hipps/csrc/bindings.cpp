// hipps._C — pybind11 bindings for the CDNA4 kernels and the native PS runtime.
#include <torch/extension.h>

namespace hipps {
// flat.hip
void aggregate(const std::vector<at::Tensor>& slots, at::Tensor acc, double gscale, bool accumulate);
void convert(at::Tensor src, at::Tensor dst, double scale);
void sgd_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, c10::optional<at::Tensor> buf,
              c10::optional<at::Tensor> pub, bool zero_src, double lr, double wd, double momentum, double dampening,
              bool nesterov, bool first);
void adam_step(const std::vector<at::Tensor>& grads, double gscale, at::Tensor p, at::Tensor exp_avg,
               at::Tensor exp_avg_sq, c10::optional<at::Tensor> max_exp_avg_sq, c10::optional<at::Tensor> pub,
               bool zero_src, double lr, double beta1, double beta2, double eps, double wd, int64_t step,
               bool amsgrad, bool torch_mode);
}  // namespace hipps

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "hipps native kernels (gfx950) and parameter-server runtime";
  m.def("aggregate", &hipps::aggregate, "acc (+)= gscale * sum_w slots[w] (rank order)");
  m.def("convert", &hipps::convert, "dst = scale * src with f32/bf16 conversion");
  m.def("sgd_step", &hipps::sgd_step, "fused decode+sum+SGD (reference ps.py:197-214 math)");
  m.def("adam_step", &hipps::adam_step, "fused decode+sum+Adam (reference ps.py:217-261 math)");
}
