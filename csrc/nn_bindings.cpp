// Bindings for the model hot-path kernels (fused BN + residual + ReLU; MFMA GEMM).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#include "dla_bindings.h"
#include "dla_kernels.h"
#include "dla_tables.h"

namespace dla {

static void check_act(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, " must be a GPU tensor");
  TORCH_CHECK(t.dim() == 4 || t.dim() == 2, what, " must be NCHW-shaped (channels_last) or [M, C]");
  const bool ok = t.dim() == 4 ? t.is_contiguous(at::MemoryFormat::ChannelsLast) : t.is_contiguous();
  TORCH_CHECK(ok, what, " must be channels_last (4-D) or contiguous (2-D)");
  TORCH_CHECK(t.size(1) % 8 == 0, what, ": channel count must be a multiple of 8");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what, " must be 16-byte aligned");
}

static int64_t rows_of(const at::Tensor& t) { return t.numel() / t.size(1); }

static int64_t partial_floats(int64_t M, int C) {
  int tpr, nrb, nct;
  bn_geometry(M, C, &tpr, &nrb, &nct, 2048);
  return (int64_t)nrb * C * 2;
}

// Returns (y, ws). ws (7C fp32) carries mean/invstd for backward.
std::vector<at::Tensor> bn_act_fwd(at::Tensor x, c10::optional<at::Tensor> residual, c10::optional<at::Tensor> weight,
                                   c10::optional<at::Tensor> bias, c10::optional<at::Tensor> running_mean,
                                   c10::optional<at::Tensor> running_var, bool training, double momentum, double eps,
                                   bool relu) {
  check_act(x, "x");
  const int C = (int)x.size(1);
  const int64_t M = rows_of(x);
  const at::Tensor* res = nullptr;
  if (residual.has_value() && residual->defined()) {
    check_act(*residual, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type(), "residual mismatch");
    res = &residual.value();
  }
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor ws = at::empty({7 * (int64_t)C}, f32);
  auto fptr = [](const c10::optional<at::Tensor>& t) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "BN parameters/stats must be fp32 contiguous");
    return t->data_ptr<float>();
  };
  float* g = fptr(weight);
  float* b = fptr(bias);
  float* rm = fptr(running_mean);
  float* rv = fptr(running_var);
  if (!training) {
    TORCH_CHECK(rm && rv, "eval-mode BN needs running statistics");
    // scale/shift from running stats (tiny per-channel torch ops, C elements)
    auto invstd = (running_var->to(at::kFloat) + eps).rsqrt();
    auto gm = weight.has_value() && weight->defined() ? *weight : at::ones_like(invstd);
    auto bt = bias.has_value() && bias->defined() ? *bias : at::zeros_like(invstd);
    ws.narrow(0, 0, C).copy_(*running_mean);
    ws.narrow(0, C, C).copy_(invstd);
    ws.narrow(0, 2 * C, C).copy_(gm * invstd);
    ws.narrow(0, 3 * C, C).copy_(bt - *running_mean * gm * invstd);
  }
  at::Tensor part = at::empty({training ? partial_floats(M, C) : 1}, f32);
  at::Tensor y = at::empty_like(x);
  launch_bn_fwd(x.data_ptr(), res ? res->data_ptr() : nullptr, y.data_ptr(), M, C, dtype_code(x), g, b, (float)eps,
                (float)momentum, training ? rm : nullptr, training ? rv : nullptr, ws.data_ptr<float>(),
                part.data_ptr<float>(), relu, training, current_stream(x));
  return {y, ws};
}

// Returns (dx, dres-or-undefined, dgamma, dbeta).
std::vector<at::Tensor> bn_act_bwd(at::Tensor dy, at::Tensor y, at::Tensor x, at::Tensor ws,
                                   c10::optional<at::Tensor> weight, bool relu, bool need_dres) {
  dy = dy.dim() == 4 ? dy.contiguous(at::MemoryFormat::ChannelsLast) : dy.contiguous();
  check_act(dy, "dy");
  check_act(x, "x");
  if (relu) check_act(y, "y");
  const int C = (int)x.size(1);
  const int64_t M = rows_of(x);
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "dy dtype must match x");
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor part = at::empty({partial_floats(M, C)}, f32);
  at::Tensor dx = at::empty_like(x);
  at::Tensor dres = need_dres ? at::empty_like(x) : at::Tensor();
  at::Tensor dg = at::empty({C}, f32), db = at::empty({C}, f32);
  const float* g = (weight.has_value() && weight->defined()) ? weight->data_ptr<float>() : nullptr;
  launch_bn_bwd(dy.data_ptr(), relu ? y.data_ptr() : nullptr, x.data_ptr(), dx.data_ptr(),
                need_dres ? dres.data_ptr() : nullptr, M, C, dtype_code(x), g, ws.data_ptr<float>(),
                part.data_ptr<float>(), dg.data_ptr<float>(), db.data_ptr<float>(), relu, current_stream(x));
  return {dx, dres, dg, db};
}

void bind_nn(pybind11::module& m) {
  m.def("bn_act_fwd", &bn_act_fwd, "fused BatchNorm(+residual)(+ReLU) forward, NHWC", pybind11::arg("x"),
        pybind11::arg("residual"), pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("running_mean"),
        pybind11::arg("running_var"), pybind11::arg("training"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("relu"));
  m.def("bn_act_bwd", &bn_act_bwd, "fused BatchNorm(+residual)(+ReLU) backward, NHWC");
}

}  // namespace dla
