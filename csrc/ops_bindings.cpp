// PyTorch bindings for the element-wise / multi-tensor HIP kernels.
// Tensor checks live here; the kernels (csrc/kernels/*.hip) see raw pointers only.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "dla_kernels.h"
#include "dla_bindings.h"
#include "dla_tables.h"

namespace dla {

int dtype_code(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return kF32;
  if (t.scalar_type() == at::kBFloat16) return kBF16;
  TORCH_CHECK(false, "distributed_learning_amd: unsupported dtype ", t.scalar_type(), " (fp32/bf16 only)");
  return -1;
}

hipStream_t current_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_dev(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, " must be a GPU tensor");
  // Elementwise kernels walk raw storage order, so any dense non-overlapping layout works
  // (channels_last conv weights included) as long as all operands share it.
  TORCH_CHECK(t.is_non_overlapping_and_dense(), what, " must be dense (non-overlapping)");
}

// Uploads a host byte blob to a device uint8 tensor (construction time only).
at::Tensor upload(const void* data, size_t bytes, const at::Device& dev) {
  auto host = at::empty({(int64_t)bytes}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), data, bytes);
  return host.to(dev);
}

// ------------------------------------------------------------------------------------------
// SgdTable: one fused multi-tensor SGD launch per step over a fixed parameter set.
// ------------------------------------------------------------------------------------------
class SgdTable {
 public:
  SgdTable(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> moms,
           std::vector<at::Tensor> shadows)
      : params_(std::move(params)), grads_(std::move(grads)), moms_(std::move(moms)), shadows_(std::move(shadows)) {
    TORCH_CHECK(!params_.empty(), "SgdTable: empty parameter list");
    TORCH_CHECK(params_.size() == grads_.size(), "SgdTable: params/grads size mismatch");
    TORCH_CHECK(moms_.empty() || moms_.size() == params_.size(), "SgdTable: momentum list size mismatch");
    TORCH_CHECK(shadows_.empty() || shadows_.size() == params_.size(), "SgdTable: shadow list size mismatch");
    grad_dtype_ = dtype_code(grads_[0]);
    std::vector<SgdEntry> entries;
    std::vector<int32_t> prefix;
    int32_t blocks = 0;
    const int chunk = mt_chunk_elems();
    for (size_t i = 0; i < params_.size(); ++i) {
      auto& p = params_[i];
      check_dev(p, "param");
      check_dev(grads_[i], "grad");
      TORCH_CHECK(p.scalar_type() == at::kFloat, "SgdTable: parameters must be fp32 (master weights)");
      TORCH_CHECK(grads_[i].numel() == p.numel(), "SgdTable: grad numel mismatch");
      TORCH_CHECK(same_layout(grads_[i], p), "SgdTable: grad layout (strides) must match the parameter");
      TORCH_CHECK(dtype_code(grads_[i]) == grad_dtype_, "SgdTable: all grads must share a dtype");
      SgdEntry e{};
      e.param = p.data_ptr<float>();
      e.grad = grads_[i].data_ptr();
      e.momentum = moms_.empty() ? nullptr : moms_[i].data_ptr<float>();
      if (!moms_.empty()) {
        check_dev(moms_[i], "momentum");
        TORCH_CHECK(moms_[i].numel() == p.numel() && moms_[i].scalar_type() == at::kFloat &&
                        same_layout(moms_[i], p),
                    "SgdTable: momentum buffer must be fp32 with the parameter's layout");
      }
      e.param_bf16 = nullptr;
      if (!shadows_.empty()) {
        check_dev(shadows_[i], "bf16 shadow");
        TORCH_CHECK(shadows_[i].scalar_type() == at::kBFloat16 && shadows_[i].numel() == p.numel(), "bad shadow");
        e.param_bf16 = reinterpret_cast<uint16_t*>(shadows_[i].data_ptr());
      }
      e.numel = p.numel();
      if (e.numel == 0) continue;
      entries.push_back(e);
      prefix.push_back(blocks);
      blocks += (int32_t)((e.numel + chunk - 1) / chunk);
    }
    ntensors_ = (int)entries.size();
    nblocks_ = blocks;
    entries_ = upload(entries.data(), entries.size() * sizeof(SgdEntry), params_[0].device());
    prefix_ = upload(prefix.data(), prefix.size() * sizeof(int32_t), params_[0].device());
  }

  void step(double lr, double momentum, double dampening, double weight_decay, bool nesterov, double grad_scale,
            bool first_step) {
    SgdParams hp{(float)lr, (float)momentum, (float)dampening, (float)weight_decay, (float)grad_scale,
                 nesterov ? 1 : 0, first_step ? 1 : 0};
    launch_sgd(reinterpret_cast<const SgdEntry*>(entries_.data_ptr()), reinterpret_cast<const int32_t*>(prefix_.data_ptr()), ntensors_, nblocks_,
               grad_dtype_, !moms_.empty(), hp, current_stream(params_[0]));
  }

  int num_blocks() const { return nblocks_; }

 private:
  std::vector<at::Tensor> params_, grads_, moms_, shadows_;
  at::Tensor entries_, prefix_;
  int ntensors_ = 0, nblocks_ = 0, grad_dtype_ = kF32;
};

// ------------------------------------------------------------------------------------------
// By-value list launches (tensor addresses may change every step).
// ------------------------------------------------------------------------------------------
void sgd_step_list(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> moms,
                   std::vector<at::Tensor> shadows, double lr, double momentum, double dampening, double weight_decay,
                   bool nesterov, double grad_scale, bool first_step) {
  TORCH_CHECK(params.size() == grads.size(), "sgd_step_list: params/grads size mismatch");
  TORCH_CHECK(moms.empty() || moms.size() == params.size(), "sgd_step_list: momentum list size mismatch");
  TORCH_CHECK(shadows.empty() || shadows.size() == params.size(), "sgd_step_list: shadow list size mismatch");
  if (params.empty()) return;
  const int gdt = dtype_code(grads[0]);
  const bool use_m = !moms.empty();
  const SgdParams hp{(float)lr, (float)momentum, (float)dampening, (float)weight_decay, (float)grad_scale,
                     nesterov ? 1 : 0, first_step ? 1 : 0};
  const int chunk = mt_chunk_elems();
  hipStream_t st = current_stream(params[0]);
  SgdList list{};
  int blocks = 0;
  auto flush = [&]() {
    if (list.ntensors == 0) return;
    list.prefix[list.ntensors] = blocks;
    launch_sgd_list(list, blocks, gdt, use_m, hp, st);
    list = SgdList{};
    blocks = 0;
  };
  for (size_t i = 0; i < params.size(); ++i) {
    const at::Tensor& p = params[i];
    check_dev(p, "param");
    check_dev(grads[i], "grad");
    TORCH_CHECK(p.scalar_type() == at::kFloat, "sgd_step_list: parameters/masters must be fp32");
    TORCH_CHECK(dtype_code(grads[i]) == gdt && same_layout(grads[i], p),
                "sgd_step_list: grad ", i, " must match its parameter's layout and the list's grad dtype");
    if (p.numel() == 0) continue;
    SgdEntry e{};
    e.param = p.data_ptr<float>();
    e.grad = grads[i].data_ptr();
    if (use_m) {
      TORCH_CHECK(moms[i].scalar_type() == at::kFloat && same_layout(moms[i], p), "bad momentum buffer");
      e.momentum = moms[i].data_ptr<float>();
    }
    if (!shadows.empty()) {
      TORCH_CHECK(shadows[i].scalar_type() == at::kBFloat16 && same_layout(shadows[i], p), "bad shadow");
      e.param_bf16 = reinterpret_cast<uint16_t*>(shadows[i].data_ptr());
    }
    e.numel = p.numel();
    list.prefix[list.ntensors] = blocks;
    list.e[list.ntensors++] = e;
    blocks += (int)((e.numel + chunk - 1) / chunk);
    if (list.ntensors == kMaxList) flush();
  }
  flush();
}

void pack_tensors_on(const std::vector<at::Tensor>& ts, const std::vector<int64_t>& offs, const at::Tensor& flat,
                     float scale, hipStream_t st) {
  TORCH_CHECK(ts.size() == offs.size(), "pack: tensors/offsets size mismatch");
  const int fdt = dtype_code(flat);
  const int chunk = mt_chunk_elems();
  PackList list{};
  int blocks = 0, sdt = -1;
  auto flush = [&]() {
    if (list.ntensors == 0) return;
    list.prefix[list.ntensors] = blocks;
    launch_pack_list(list, blocks, sdt, fdt, flat.data_ptr(), scale, st);
    list = PackList{};
    blocks = 0;
  };
  for (size_t i = 0; i < ts.size(); ++i) {
    check_dev(ts[i], "pack tensor");
    const int d = dtype_code(ts[i]);
    if (sdt != -1 && d != sdt) flush();
    sdt = d;
    TORCH_CHECK(offs[i] >= 0 && offs[i] + ts[i].numel() <= flat.numel(), "pack: slot out of range");
    if (ts[i].numel() == 0) continue;
    list.prefix[list.ntensors] = blocks;
    list.e[list.ntensors++] = PackEntry{ts[i].data_ptr(), ts[i].numel(), offs[i]};
    blocks += (int)((ts[i].numel() + chunk - 1) / chunk);
    if (list.ntensors == kMaxList) flush();
  }
  flush();
}

void pack_list(std::vector<at::Tensor> ts, std::vector<int64_t> offs, at::Tensor flat, double scale) {
  check_dev(flat, "flat");
  pack_tensors_on(ts, offs, flat, (float)scale, current_stream(flat));
}

// ------------------------------------------------------------------------------------------
// PackTable (declared in dla_tables.h).
// ------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------
// Free functions
// ------------------------------------------------------------------------------------------
void reduce_sum_(at::Tensor dst, std::vector<at::Tensor> srcs, bool accumulate, double scale) {
  check_dev(dst, "dst");
  TORCH_CHECK((int)srcs.size() <= kMaxReduceSrc, "reduce_sum_: at most ", kMaxReduceSrc, " sources");
  ReduceSrcs rs{};
  rs.count = (int)srcs.size();
  for (size_t i = 0; i < srcs.size(); ++i) {
    check_dev(srcs[i], "src");
    TORCH_CHECK(srcs[i].scalar_type() == dst.scalar_type(), "reduce_sum_: dtype mismatch");
    TORCH_CHECK(srcs[i].numel() >= dst.numel(), "reduce_sum_: source shorter than destination");
    rs.ptr[i] = srcs[i].data_ptr();
  }
  launch_reduce_sum(dst.data_ptr(), accumulate, rs, dst.numel(), dtype_code(dst), (float)scale, current_stream(dst));
}

void scale_(at::Tensor t, double scale) {
  check_dev(t, "tensor");
  launch_scale(t.data_ptr(), t.numel(), dtype_code(t), (float)scale, current_stream(t));
}

static const int64_t* step_ptr(const c10::optional<at::Tensor>& step, const at::Tensor& t) {
  if (!step.has_value() || !step->defined()) return nullptr;
  TORCH_CHECK(step->scalar_type() == at::kLong && step->numel() == 1 && step->device() == t.device(),
              "step must be a one-element int64 tensor on the output's device");
  return step->data_ptr<int64_t>();
}

void uniform_(at::Tensor t, int64_t seed, int64_t offset, double lo, double hi, c10::optional<at::Tensor> step,
              int64_t per_step) {
  check_dev(t, "tensor");
  launch_uniform_fill(t.data_ptr(), t.numel(), dtype_code(t), (uint64_t)seed, (uint64_t)offset, (float)lo, (float)hi,
                      current_stream(t), step_ptr(step, t), (uint64_t)per_step);
}

void randint_(at::Tensor t, int64_t high, int64_t seed, int64_t offset, c10::optional<at::Tensor> step,
              int64_t per_step) {
  check_dev(t, "tensor");
  TORCH_CHECK(t.scalar_type() == at::kLong, "randint_: int64 tensor required");
  TORCH_CHECK(high > 0, "randint_: high must be positive");
  launch_randint_fill(t.data_ptr<int64_t>(), t.numel(), high, (uint64_t)seed, (uint64_t)offset, current_stream(t),
                      step_ptr(step, t), (uint64_t)per_step);
}

std::vector<at::Tensor> xent_fwd(at::Tensor logits, at::Tensor target) {
  check_dev(logits, "logits");
  check_dev(target, "target");
  TORCH_CHECK(logits.dim() == 2, "xent_fwd: logits must be [B, C]");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.numel() == logits.size(0), "xent_fwd: bad target");
  const int B = (int)logits.size(0), C = (int)logits.size(1);
  auto f32 = logits.options().dtype(at::kFloat);
  auto ws = at::empty({3 * (int64_t)B}, f32);
  auto loss = at::empty({2}, f32);
  launch_xent_fwd(logits.data_ptr(), target.data_ptr<int64_t>(), ws.data_ptr<float>(), loss.data_ptr<float>(), B, C,
                  dtype_code(logits), current_stream(logits));
  return {loss, ws};
}

at::Tensor xent_bwd(at::Tensor logits, at::Tensor target, at::Tensor ws, at::Tensor loss, at::Tensor gout) {
  check_dev(logits, "logits");
  auto d = at::empty_like(logits);
  const int B = (int)logits.size(0), C = (int)logits.size(1);
  auto g = gout.to(at::kFloat).contiguous();
  launch_xent_bwd(logits.data_ptr(), target.data_ptr<int64_t>(), ws.data_ptr<float>(), loss.data_ptr<float>(),
                  g.data_ptr<float>(), d.data_ptr(), B, C, dtype_code(logits), current_stream(logits));
  return d;
}

void bind_ops(pybind11::module& m) {
  pybind11::class_<SgdTable>(m, "SgdTable")
      .def(pybind11::init<std::vector<at::Tensor>, std::vector<at::Tensor>, std::vector<at::Tensor>,
                          std::vector<at::Tensor>>())
      .def("step", &SgdTable::step)
      .def("num_blocks", &SgdTable::num_blocks);
  pybind11::class_<PackTable>(m, "PackTable")
      .def(pybind11::init<std::vector<at::Tensor>, std::vector<int64_t>>())
      .def("pack", &PackTable::pack)
      .def("unpack", &PackTable::unpack)
      .def("total_numel", &PackTable::total_numel);
  m.def("reduce_sum_", &reduce_sum_, "dst = scale*([dst] + sum(srcs))");
  m.def("sgd_step_list", &sgd_step_list, "fused SGD over a by-value tensor list (<= 32 tensors per launch)");
  m.def("pack_list", &pack_list, "gather tensors into a flat buffer at element offsets (by-value list launch)");
  m.def("scale_", &scale_, "t *= scale");
  m.def("uniform_", &uniform_, "Philox uniform fill (stream position offset [+ *step * per_step])",
        pybind11::arg("t"), pybind11::arg("seed"), pybind11::arg("offset"), pybind11::arg("lo"), pybind11::arg("hi"),
        pybind11::arg("step") = pybind11::none(), pybind11::arg("per_step") = 0);
  m.def("randint_", &randint_, "Philox integer fill in [0, high)", pybind11::arg("t"), pybind11::arg("high"),
        pybind11::arg("seed"), pybind11::arg("offset"), pybind11::arg("step") = pybind11::none(),
        pybind11::arg("per_step") = 0);
  m.def("xent_fwd", &xent_fwd, "fused log-softmax + NLL forward");
  m.def("xent_bwd", &xent_bwd, "fused log-softmax + NLL backward");
}

}  // namespace dla
