// Bindings for the model hot-path kernels (fused BN + residual + ReLU; MFMA GEMM).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#include "dla_bindings.h"
#include "dla_kernels.h"
#include "dla_tables.h"

namespace dla {

// Bytes one operand spans (its last element's offset + 1): the MFMA main loops and the streaming GEMM
// address operands through buffer descriptors whose out-of-range slots use offset 0x80000000 (kOOB,
// dla_mfma.h), so every operand must stay below 2 GiB; beyond it they would read wrapped data.
static void check_span(const at::Tensor& t, const char* what) {
  int64_t last = 0;
  for (int64_t d = 0; d < t.dim(); ++d) last += (t.size(d) - 1) * t.stride(d);
  const int64_t bytes = t.numel() ? (last + 1) * (int64_t)t.element_size() : 0;
  TORCH_CHECK(bytes < (int64_t(1) << 31), what, ": ", bytes,
              " bytes reach the 2 GiB buffer-descriptor range of the native kernels (lower the per-GPU batch)");
}

static void check_act(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, " must be a GPU tensor");
  TORCH_CHECK(t.dim() == 4 || t.dim() == 2, what, " must be NCHW-shaped (channels_last) or [M, C]");
  const bool ok = t.dim() == 4 ? t.is_contiguous(at::MemoryFormat::ChannelsLast) : t.is_contiguous();
  TORCH_CHECK(ok, what, " must be channels_last (4-D) or contiguous (2-D)");
  TORCH_CHECK(t.size(1) % 8 == 0, what, ": channel count must be a multiple of 8");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what, " must be 16-byte aligned");
  check_span(t, what);
}

static int64_t rows_of(const at::Tensor& t) { return t.numel() / t.size(1); }

// Row stride of a bf16 channels_last [N, C, H, W] tensor read as [M, C] rows: 0 when contiguous, the
// wider tensor's channel count when it is a channel slice of one (e.g. one branch of the fused
// Inception fan-in GEMM output).
static int64_t cl_row_stride(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.scalar_type() == at::kBFloat16 && t.size(1) % 8 == 0, what,
              " must be a bf16 [N, C, H, W] GPU tensor with C % 8 == 0");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what, " must be 16-byte aligned");
  if (t.is_contiguous(at::MemoryFormat::ChannelsLast)) return 0;
  const int64_t ld = t.stride(3);
  TORCH_CHECK(t.stride(1) == 1 && ld > t.size(1) && ld % 8 == 0 && t.stride(2) == ld * t.size(3) &&
                  t.stride(0) == t.stride(2) * t.size(2),
              what, " must be channels_last or a channel slice of a channels_last tensor");
  return ld;
}


// launch_bn_fwd scratch for GEMM-epilogue statistics [rows][C][2]: the folded rows (>= 1 float)
static int64_t ext_part_floats(const c10::optional<at::Tensor>& st, int C) {
  return std::max<int64_t>(1, (int64_t)bn_fold_groups((int)st->size(0)) * C * 2);
}

static int64_t partial_floats(int64_t M, int C) { return bn_partial_floats(M, C); }

// Returns (y, ws, mask). ws (7C fp32) carries mean/invstd/scale/shift for backward; mask (uint8,
// one bit per element) is only produced for ReLU after a residual add in training mode.
std::vector<at::Tensor> bn_act_fwd(at::Tensor x, c10::optional<at::Tensor> residual, c10::optional<at::Tensor> weight,
                                   c10::optional<at::Tensor> bias, c10::optional<at::Tensor> running_mean,
                                   c10::optional<at::Tensor> running_var, bool training, double momentum, double eps,
                                   bool relu, c10::optional<at::Tensor> stats, c10::optional<at::Tensor> out,
                                   int64_t out_channel, bool defer) {
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
  const bool ext = stats.has_value() && stats->defined();
  if (ext) {
    TORCH_CHECK(stats->scalar_type() == at::kFloat && stats->is_contiguous() && stats->dim() == 3 &&
                    stats->size(1) == C && stats->size(2) == 2,
                "stats must be fp32 [row_blocks, C, 2] partials");
  }
  at::Tensor part = at::empty({(training && !ext) ? partial_floats(M, C) : ext ? ext_part_floats(stats, C) : 1}, f32);
  // out: write y into channels [out_channel, out_channel + C) of a wider channels_last tensor (the
  // concatenated output of an Inception block) instead of a fresh one
  at::Tensor y;
  int64_t ldy = 0;
  if (out.has_value() && out->defined()) {
    TORCH_CHECK(x.dim() == 4 && out->dim() == 4 && out->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    out->scalar_type() == x.scalar_type() && out->size(0) == x.size(0) && out->size(2) == x.size(2) &&
                    out->size(3) == x.size(3) && out->size(1) % 8 == 0 && out_channel % 8 == 0 && out_channel >= 0 &&
                    out_channel + C <= out->size(1),
                "bn_act_fwd: out must be a channels_last [N, Ctot, H, W] tensor (Ctot, out_channel % 8 == 0) of x's "
                "dtype and spatial size holding channels [out_channel, out_channel + C)");
    y = out->narrow(1, out_channel, C);
    ldy = out->size(1);
  } else {
    y = at::empty_like(x);
  }
  at::Tensor mask;
  if (training && relu && res) mask = at::empty({(M * C + 7) / 8}, x.options().dtype(at::kByte));
  // defer: statistics and coefficients only; y (and the mask) are written later by the consumer's GEMM
  // (gemm_nt_apply) or by bn_apply_deferred
  TORCH_CHECK(!defer || (training && ldy == 0 && x.scalar_type() == at::kBFloat16),
              "bn_act_fwd: defer needs training mode, bf16 and a fresh output");
  launch_bn_fwd(x.data_ptr(), res ? res->data_ptr() : nullptr, defer ? nullptr : y.data_ptr(), M, C, dtype_code(x), g, b, (float)eps,
                (float)momentum, training ? rm : nullptr, training ? rv : nullptr, ws.data_ptr<float>(),
                part.data_ptr<float>(), relu, training, current_stream(x), ext ? stats->data_ptr<float>() : nullptr,
                ext ? (int)stats->size(0) : 0, mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, ldy);
  return {y, ws, mask};
}

// Training-mode act(BN(x) + BN_d(xd)) — a residual block whose shortcut is a downsample conv + BN —
// in one apply pass: the shortcut BN's output is never materialised. Returns (y, ws, wsd, mask);
// mask (ReLU only) is the 1-bit ReLU mask both backward passes read. stats / statsd: optional
// [row_blocks, C, 2] partials from the producing convs' epilogues.
std::vector<at::Tensor> bn_dual_fwd(at::Tensor x, at::Tensor xd, c10::optional<at::Tensor> weight,
                                    c10::optional<at::Tensor> bias, c10::optional<at::Tensor> running_mean,
                                    c10::optional<at::Tensor> running_var, c10::optional<at::Tensor> weight_d,
                                    c10::optional<at::Tensor> bias_d, c10::optional<at::Tensor> running_mean_d,
                                    c10::optional<at::Tensor> running_var_d, double momentum, double momentum_d,
                                    double eps, double eps_d, bool relu, c10::optional<at::Tensor> stats,
                                    c10::optional<at::Tensor> stats_d, bool defer) {
  check_act(x, "x");
  check_act(xd, "xd");
  TORCH_CHECK(xd.sizes() == x.sizes() && xd.scalar_type() == x.scalar_type(), "bn_dual: x / xd mismatch");
  const int C = (int)x.size(1);
  const int64_t M = rows_of(x);
  auto f32 = x.options().dtype(at::kFloat);
  auto fptr = [](const c10::optional<at::Tensor>& t) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "BN parameters/stats must be fp32 contiguous");
    return t->data_ptr<float>();
  };
  auto finalize = [&](const at::Tensor& in, const c10::optional<at::Tensor>& g, const c10::optional<at::Tensor>& b,
                      const c10::optional<at::Tensor>& rm, const c10::optional<at::Tensor>& rv, double mom, double ep,
                      const c10::optional<at::Tensor>& st) {
    at::Tensor ws = at::empty({7 * (int64_t)C}, f32);
    const bool ext = st.has_value() && st->defined();
    if (ext)
      TORCH_CHECK(st->scalar_type() == at::kFloat && st->is_contiguous() && st->dim() == 3 && st->size(1) == C &&
                      st->size(2) == 2,
                  "stats must be fp32 [row_blocks, C, 2] partials");
    at::Tensor part = at::empty({ext ? ext_part_floats(st, C) : partial_floats(M, C)}, f32);
    launch_bn_fwd(in.data_ptr(), nullptr, nullptr, M, C, dtype_code(in), fptr(g), fptr(b), (float)ep, (float)mom,
                  fptr(rm), fptr(rv), ws.data_ptr<float>(), part.data_ptr<float>(), relu, true, current_stream(in),
                  ext ? st->data_ptr<float>() : nullptr, ext ? (int)st->size(0) : 0);
    return ws;
  };
  at::Tensor ws = finalize(x, weight, bias, running_mean, running_var, momentum, eps, stats);
  at::Tensor wsd = finalize(xd, weight_d, bias_d, running_mean_d, running_var_d, momentum_d, eps_d, stats_d);
  at::Tensor y = at::empty_like(x);
  at::Tensor mask;
  if (relu) mask = at::empty({(M * C + 7) / 8}, x.options().dtype(at::kByte));
  if (!defer)
    launch_bn_dual_apply(x.data_ptr(), xd.data_ptr(), y.data_ptr(), ws.data_ptr<float>(), wsd.data_ptr<float>(), M, C,
                         dtype_code(x), relu, relu ? mask.data_ptr<uint8_t>() : nullptr, current_stream(x));
  return {y, ws, wsd, mask};
}

// The apply pass a deferred bn_act_fwd / bn_dual_fwd skipped: y = act(BN(x) + r) (r a BN input too when wsd is
// given), mask = its ReLU bits. For a deferred output whose consumer is not a gemm_nt_apply.
void bn_apply_deferred(at::Tensor x, c10::optional<at::Tensor> r_, at::Tensor ws, c10::optional<at::Tensor> wsd,
                       at::Tensor y, c10::optional<at::Tensor> mask_) {
  check_act(x, "x");
  check_act(y, "y");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 && y.sizes() == x.sizes(),
              "bn_apply_deferred: x, y must be bf16 tensors of one shape");
  const int C = (int)x.size(1);
  const int64_t M = rows_of(x);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() == 7 * (int64_t)C, "ws: 7C fp32");
  if (!(r_.has_value() && r_->defined())) {  // relu(BN(x)), no residual (its backward recomputes the ReLU from x)
    launch_bn_fwd(x.data_ptr(), nullptr, y.data_ptr(), M, C, kBF16, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr,
                  ws.data_ptr<float>(), nullptr, true, false, current_stream(x), nullptr, 0, nullptr, 0);
    return;
  }
  at::Tensor r = *r_;
  check_act(r, "r");
  TORCH_CHECK(r.scalar_type() == at::kBFloat16 && r.sizes() == x.sizes(), "bn_apply_deferred: r like x");
  TORCH_CHECK(mask_.has_value() && mask_->defined(), "bn_apply_deferred: a residual needs the ReLU mask");
  at::Tensor mask = *mask_;
  TORCH_CHECK(mask.scalar_type() == at::kByte && mask.numel() * 8 >= M * C, "mask: one bit per element");
  const bool dual = wsd.has_value() && wsd->defined();
  if (dual) {
    TORCH_CHECK(wsd->scalar_type() == at::kFloat && wsd->is_contiguous() && wsd->numel() == 7 * (int64_t)C, "wsd: 7C fp32");
    launch_bn_dual_apply(x.data_ptr(), r.data_ptr(), y.data_ptr(), ws.data_ptr<float>(), wsd->data_ptr<float>(), M, C,
                         kBF16, true, mask.data_ptr<uint8_t>(), current_stream(x));
  } else {
    launch_bn_fwd(x.data_ptr(), r.data_ptr(), y.data_ptr(), M, C, kBF16, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr,
                  ws.data_ptr<float>(), nullptr, true, false, current_stream(x), nullptr, 0, mask.data_ptr<uint8_t>(), 0);
  }
}

// Backward of bn_dual_fwd: returns (dx, dgamma, dbeta, dxd, dgamma_d, dbeta_d).
std::vector<at::Tensor> bn_dual_bwd(at::Tensor dy, c10::optional<at::Tensor> mask, at::Tensor x, at::Tensor ws,
                                    c10::optional<at::Tensor> weight, at::Tensor xd, at::Tensor wsd,
                                    c10::optional<at::Tensor> weight_d, bool want_dx) {
  dy = dy.dim() == 4 ? dy.contiguous(at::MemoryFormat::ChannelsLast) : dy.contiguous();
  check_act(dy, "dy");
  check_act(x, "x");
  check_act(xd, "xd");
  const int C = (int)x.size(1);
  const int64_t M = rows_of(x);
  TORCH_CHECK(dy.sizes() == x.sizes() && xd.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type() &&
                  xd.scalar_type() == x.scalar_type(),
              "bn_dual_bwd: dy / x / xd mismatch");
  TORCH_CHECK(ws.numel() == 7 * (int64_t)C && wsd.numel() == 7 * (int64_t)C, "bn_dual_bwd: 7C workspaces");
  const uint8_t* mp = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() * 8 >= M * C, "bn_dual_bwd: bit mask size");
    mp = mask->data_ptr<uint8_t>();
  }
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor part = at::empty({partial_floats(M, C)}, f32), partd = at::empty({partial_floats(M, C)}, f32);
  // want_dx = false: reductions + finalizes only (ws / wsd then hold the apply coefficients)
  at::Tensor dx = want_dx ? at::empty_like(x) : at::Tensor(), dxd = want_dx ? at::empty_like(xd) : at::Tensor();
  at::Tensor dg = at::empty({C}, f32), db = at::empty({C}, f32), dgd = at::empty({C}, f32), dbd = at::empty({C}, f32);
  auto gp = [](const c10::optional<at::Tensor>& w) -> const float* {
    return (w.has_value() && w->defined()) ? w->data_ptr<float>() : nullptr;
  };
  launch_bn_dual_bwd(dy.data_ptr(), mp, x.data_ptr(), xd.data_ptr(), want_dx ? dx.data_ptr() : nullptr,
                     want_dx ? dxd.data_ptr() : nullptr, M, C,
                     dtype_code(x), gp(weight), gp(weight_d), ws.data_ptr<float>(), wsd.data_ptr<float>(),
                     part.data_ptr<float>(), partd.data_ptr<float>(), dg.data_ptr<float>(), db.data_ptr<float>(),
                     dgd.data_ptr<float>(), dbd.data_ptr<float>(), current_stream(x));
  return {dx, dg, db, dxd, dgd, dbd};
}

// Returns (dx, dres-or-undefined, dgamma, dbeta). mask_mode (see launch_bn_bwd): 0 no ReLU,
// 1 recompute the ReLU branch from x, 2 use `mask` from bn_act_fwd, 3 use the saved output `y`.
std::vector<at::Tensor> bn_act_bwd(at::Tensor dy, c10::optional<at::Tensor> y, c10::optional<at::Tensor> mask,
                                   at::Tensor x, at::Tensor ws, c10::optional<at::Tensor> weight, int64_t mask_mode,
                                   bool need_dres, c10::optional<at::Tensor> ext_part, bool want_dx) {
  TORCH_CHECK(want_dx || !need_dres, "bn_act_bwd: the residual gradient comes from the apply pass");
  check_act(x, "x");
  const int C = (int)x.size(1);
  const int64_t M = rows_of(x);
  // dy may be a channel slice of a wider channels_last tensor (an Inception branch of the
  // concatenated output gradient): read in place with its row stride
  int64_t ld_dy = 0;
  if (dy.dim() == 4 && x.dim() == 4 && dy.sizes() == x.sizes() && dy.stride(1) == 1 && dy.stride(3) > C &&
      dy.stride(3) % 8 == 0 && dy.stride(2) == dy.stride(3) * dy.size(3) && dy.stride(0) == dy.stride(2) * dy.size(2) &&
      (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0 && !need_dres && mask_mode != 3) {
    ld_dy = dy.stride(3);
  } else {
    dy = dy.dim() == 4 ? dy.contiguous(at::MemoryFormat::ChannelsLast) : dy.contiguous();
    check_act(dy, "dy");
  }
  TORCH_CHECK(mask_mode >= 0 && mask_mode <= 3, "bad mask_mode");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() == 7 * (int64_t)C, "ws must be the 7C fp32 workspace");
  const void* yp = nullptr;
  const uint8_t* mp = nullptr;
  if (mask_mode == 3) {
    TORCH_CHECK(y.has_value() && y->defined(), "mask_mode 3 needs y");
    check_act(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes() && y->scalar_type() == x.scalar_type(), "y mismatch");
    yp = y->data_ptr();
  } else if (mask_mode == 2) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->scalar_type() == at::kByte &&
                    mask->numel() * 8 >= M * C && mask->is_cuda(),
                "mask_mode 2 needs the forward's 1-bit mask");
    mp = mask->data_ptr<uint8_t>();
  }
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "dy dtype must match x");
  auto f32 = x.options().dtype(at::kFloat);
  const bool ext = ext_part.has_value() && ext_part->defined();
  if (ext)
    TORCH_CHECK(ext_part->scalar_type() == at::kFloat && ext_part->is_contiguous() && ext_part->dim() == 3 &&
                    ext_part->size(1) == C && ext_part->size(2) == 2,
                "ext_part must be fp32 [rows, C, 2] (sum dy', sum dy'(x-mean)) partials");
  at::Tensor part = at::empty({ext ? 1 : partial_floats(M, C)}, f32);
  // want_dx = false: reduction + finalize only (ws then holds the apply coefficients for a fused consumer)
  at::Tensor dx = want_dx ? at::empty_like(x) : at::Tensor();
  at::Tensor dres = need_dres ? at::empty_like(x) : at::Tensor();
  at::Tensor dg = at::empty({C}, f32), db = at::empty({C}, f32);
  const float* g = (weight.has_value() && weight->defined()) ? weight->data_ptr<float>() : nullptr;
  launch_bn_bwd(dy.data_ptr(), yp, mp, x.data_ptr(), want_dx ? dx.data_ptr() : nullptr, need_dres ? dres.data_ptr() : nullptr, M, C,
                dtype_code(x), g, ws.data_ptr<float>(), part.data_ptr<float>(), dg.data_ptr<float>(),
                db.data_ptr<float>(), (int)mask_mode, current_stream(x), ext ? ext_part->data_ptr<float>() : nullptr,
                ext ? (int)ext_part->size(0) : 0, ld_dy);
  return {dx, dres, dg, db};
}

// BN-backward epilogue operands (see BnBwdArgs): x_bn is the BN input laid out like the GEMM output.
static BnBwdArgs make_bn_bwd(const at::Tensor& x_bn, const at::Tensor& ws, const c10::optional<at::Tensor>& mask,
                             int64_t mode, int64_t M, int64_t N, int64_t rows, at::Tensor& part) {
  int64_t ldx = 0;
  if (x_bn.dim() == 4 && !x_bn.is_contiguous(at::MemoryFormat::ChannelsLast)) ldx = cl_row_stride(x_bn, "bn epilogue x");
  TORCH_CHECK(x_bn.is_cuda() && x_bn.scalar_type() == at::kBFloat16 && x_bn.numel() == M * N &&
                  (x_bn.dim() == 2 ? x_bn.is_contiguous() : (ldx > 0 || x_bn.is_contiguous(at::MemoryFormat::ChannelsLast))) &&
                  x_bn.size(1) == N,
              "bn epilogue: x must be the bf16 BN input with the GEMM output's shape (channels_last, or a channel "
              "slice of a wider channels_last tensor)");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() == 7 * N, "bn epilogue: ws must be the 7C workspace");
  TORCH_CHECK(mode >= 0 && mode <= 2, "bn epilogue: mode 0 (no ReLU), 1 (recompute) or 2 (bit mask)");
  const uint8_t* mp = nullptr;
  if (mode == 2) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->scalar_type() == at::kByte && mask->numel() * 8 >= M * N,
                "bn epilogue: mode 2 needs the forward's bit mask");
    mp = mask->data_ptr<uint8_t>();
  }
  part = at::empty({rows, N, 2}, ws.options());
  TORCH_CHECK(ldx == 0 || mode != 2, "bn epilogue: the bit mask needs a contiguous x");
  return BnBwdArgs{x_bn.data_ptr(), ws.data_ptr<float>(), mp, (int)mode, part.data_ptr<float>(), ldx};
}

static void check_mat(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2, what, " must be a 2-D GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, what, " must be bf16");
  TORCH_CHECK(t.stride(1) == 1, what, " must have unit stride in its last dim");
  TORCH_CHECK(t.size(1) % 8 == 0 && t.stride(0) % 8 == 0, what, ": rows must be multiples of 8 elements");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what, " must be 16-byte aligned");
  check_span(t, what);
}

// C = A @ B^T (A [M,K], B [N,K]; or C = A @ B with B [K,N] when b_kmajor) in bf16 with fp32 accumulation. Optionally returns per-row-block
// column statistics partials [ceil(M/128), N, 2] (sum, sum of squares of the bf16 outputs).
static const uint8_t* addend_mask_ptr(const c10::optional<at::Tensor>& m, int64_t M, int64_t N, bool add) {
  if (!m.has_value() || !m->defined()) return nullptr;
  TORCH_CHECK(add, "addend_mask needs an addend");
  TORCH_CHECK(m->scalar_type() == at::kByte && m->is_cuda() && m->numel() * 8 >= M * N,
              "addend_mask must be the uint8 1-bit mask of the addend");
  return m->data_ptr<uint8_t>();
}

// addend2: the gradient of the block input's stride-2 subsample, [n, C, H/2, W/2] channels_last,
// added at the even pixels of the [n*H*W, C] output rows (requires even H, W).
static const void* addend2_ptr(const c10::optional<at::Tensor>& a2, int64_t M, int64_t N, int64_t H, int64_t W) {
  if (!a2.has_value() || !a2->defined()) return nullptr;
  TORCH_CHECK(H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0 && M % (H * W) == 0, "addend2: even H, W dividing M");
  TORCH_CHECK(a2->scalar_type() == at::kBFloat16 && a2->dim() == 4 && a2->size(1) == N && a2->size(2) == H / 2 &&
                  a2->size(3) == W / 2 && a2->size(0) == M / (H * W) &&
                  a2->is_contiguous(at::MemoryFormat::ChannelsLast),
              "addend2 must be the bf16 channels_last [n, C, H/2, W/2] gradient");
  return a2->data_ptr();
}

// Grouped training BN+ReLU (launch_bn_group_fwd / _bwd): the BatchNorms of an Inception block's
// branches, one launch per pass. bn_concat_*: outputs are channel slices of the concatenated NHWC
// block output (dy read in place from its gradient); bn_group_*: each output its own tensor.
static void check_bn_param(const at::Tensor& t, int64_t C, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == C, what,
              " must be a contiguous fp32 GPU vector of C elements");
}

static int64_t check_branch(const at::Tensor& y, const at::Tensor& ref, const char* what) {
  const int64_t ld = cl_row_stride(y, what);
  TORCH_CHECK(y.size(0) == ref.size(0) && y.size(2) == ref.size(2) && y.size(3) == ref.size(3), what,
              ": every branch must have the same N, H, W");
  return ld;
}

// [rows, C, 2] fp32 partials, or a channel slice of a wider [rows, Ctot, 2] tensor: row stride in channels
static int partials_row_stride(const at::Tensor& st, int64_t C, const char* what) {
  TORCH_CHECK(st.is_cuda() && st.scalar_type() == at::kFloat && st.dim() == 3 && st.size(1) == C && st.size(2) == 2 &&
                  st.stride(2) == 1 && st.stride(1) == 2 && st.stride(0) % 2 == 0 && st.stride(0) >= 2 * C,
              what, " must be fp32 [row_blocks, C, 2] partials (or a channel slice of wider ones)");
  return st.stride(0) == 2 * C ? 0 : (int)(st.stride(0) / 2);
}

// forward fields shared by both variants; returns the workspaces (keep: scratch kept alive)
static std::vector<at::Tensor> group_fwd_fields(BnGroups& G, const std::vector<at::Tensor>& ys,
                                                const std::vector<at::Tensor>& gammas,
                                                const std::vector<at::Tensor>& betas, const std::vector<at::Tensor>& rms,
                                                const std::vector<at::Tensor>& rvs, const std::vector<double>& moms,
                                                const std::vector<double>& epss, const std::vector<at::Tensor>& stats,
                                                std::vector<at::Tensor>& keep) {
  const int n = (int)ys.size();
  TORCH_CHECK(n >= 1 && n <= kMaxBnGroups && (int)gammas.size() == n && (int)betas.size() == n &&
                  (int)rms.size() == n && (int)rvs.size() == n && (int)moms.size() == n && (int)epss.size() == n &&
                  (int)stats.size() == n,
              "grouped BN: 1..4 branches, one entry per branch in every list");
  G.n = n;
  std::vector<at::Tensor> wss;
  for (int g = 0; g < n; ++g) {
    G.ldx[g] = check_branch(ys[g], ys[0], "y");
    const int C = (int)ys[g].size(1);
    const at::Tensor& st = stats[g];
    G.ldp[g] = partials_row_stride(st, C, "grouped BN stats");
    check_bn_param(gammas[g], C, "weight");
    check_bn_param(betas[g], C, "bias");
    check_bn_param(rms[g], C, "running_mean");
    check_bn_param(rvs[g], C, "running_var");
    auto f32 = ys[g].options().dtype(at::kFloat);
    at::Tensor ws = at::empty({7 * (int64_t)C}, f32);
    keep.push_back(at::empty({std::max<int64_t>(1, (int64_t)bn_fold_groups((int)st.size(0)) * C * 2)}, f32));
    G.x[g] = (const uint16_t*)ys[g].data_ptr();
    G.C[g] = C;
    G.nrb[g] = (int)st.size(0);
    G.part[g] = st.data_ptr<float>();
    G.wpart[g] = keep.back().data_ptr<float>();
    G.gamma[g] = gammas[g].data_ptr<float>();
    G.beta[g] = betas[g].data_ptr<float>();
    G.rm[g] = rms[g].data_ptr<float>();
    G.rv[g] = rvs[g].data_ptr<float>();
    G.ws[g] = ws.data_ptr<float>();
    G.eps[g] = (float)epss[g];
    G.mom[g] = (float)moms[g];
    wss.push_back(ws);
  }
  return wss;
}

// into channels [off_g, off_g + C_g) of out (the concatenated block output); returns the workspaces
std::vector<at::Tensor> bn_concat_fwd(std::vector<at::Tensor> ys, std::vector<at::Tensor> gammas,
                                      std::vector<at::Tensor> betas, std::vector<at::Tensor> rms,
                                      std::vector<at::Tensor> rvs, std::vector<double> moms, std::vector<double> epss,
                                      std::vector<at::Tensor> stats, at::Tensor out) {
  check_act(out, "out");
  TORCH_CHECK(out.dim() == 4 && out.scalar_type() == at::kBFloat16, "bn_concat_fwd: out must be bf16 [N, Ctot, H, W]");
  BnGroups G{};
  std::vector<at::Tensor> keep;
  auto wss = group_fwd_fields(G, ys, gammas, betas, rms, rvs, moms, epss, stats, keep);
  int64_t off = 0;
  for (int g = 0; g < G.n; ++g) {
    (void)check_branch(ys[g], out, "y");
    G.y[g] = (uint16_t*)out.data_ptr() + off;
    G.ldy[g] = out.size(1);
    off += G.C[g];
  }
  TORCH_CHECK(off == out.size(1), "bn_concat_fwd: branch channels must add up to out's channels");
  const int64_t M = rows_of(out);
  if (M > 0) launch_bn_group_fwd(G, M, current_stream(out));
  return wss;
}

// each branch into its own tensor; returns [a_0 .. a_{n-1}, ws_0 .. ws_{n-1}]
std::vector<at::Tensor> bn_group_fwd(std::vector<at::Tensor> ys, std::vector<at::Tensor> gammas,
                                     std::vector<at::Tensor> betas, std::vector<at::Tensor> rms,
                                     std::vector<at::Tensor> rvs, std::vector<double> moms, std::vector<double> epss,
                                     std::vector<at::Tensor> stats) {
  BnGroups G{};
  std::vector<at::Tensor> keep;
  auto wss = group_fwd_fields(G, ys, gammas, betas, rms, rvs, moms, epss, stats, keep);
  std::vector<at::Tensor> res;
  for (int g = 0; g < G.n; ++g) {
    res.push_back(at::empty(ys[g].sizes(), ys[g].options().memory_format(at::MemoryFormat::ChannelsLast)));
    G.y[g] = (uint16_t*)res.back().data_ptr();
    G.ldy[g] = 0;
  }
  const int64_t M = rows_of(ys[0]);
  if (M > 0) launch_bn_group_fwd(G, M, current_stream(ys[0]));
  res.insert(res.end(), wss.begin(), wss.end());
  return res;
}

// backward fields shared by both variants; returns [dx_0, dgamma_0, dbeta_0, dx_1, ...]
static std::vector<at::Tensor> group_bwd_fields(BnGroups& G, const std::vector<at::Tensor>& ys,
                                                const std::vector<at::Tensor>& gammas,
                                                const std::vector<at::Tensor>& wss,
                                                const std::vector<at::Tensor>& dx_out = {}) {
  const int n = (int)ys.size();
  TORCH_CHECK(n >= 1 && n <= kMaxBnGroups && (int)gammas.size() == n && (int)wss.size() == n,
              "grouped BN backward: 1..4 branches, one entry per branch in every list");
  G.n = n;
  std::vector<at::Tensor> res;
  TORCH_CHECK(dx_out.empty() || (int)dx_out.size() == n, "grouped BN backward: one dx output per branch");
  for (int g = 0; g < n; ++g) {
    G.ldx[g] = check_branch(ys[g], ys[0], "y");
    const int C = (int)ys[g].size(1);
    check_bn_param(gammas[g], C, "weight");
    TORCH_CHECK(wss[g].scalar_type() == at::kFloat && wss[g].numel() == 7 * (int64_t)C, "ws must be the 7C workspace");
    auto f32 = ys[g].options().dtype(at::kFloat);
    at::Tensor dx, dg = at::empty({C}, f32), db = at::empty({C}, f32);
    if (!dx_out.empty()) {  // written into a given (possibly strided) slice, e.g. of the fan-in's dY
      dx = dx_out[g];
      G.lddx[g] = check_branch(dx, ys[g], "dx_out");
      TORCH_CHECK(dx.size(1) == C, "dx_out: channel count of its branch");
    } else {
      dx = at::empty(ys[g].sizes(), ys[g].options().memory_format(at::MemoryFormat::ChannelsLast));
    }
    G.x[g] = (const uint16_t*)ys[g].data_ptr();
    G.C[g] = C;
    G.gamma[g] = gammas[g].data_ptr<float>();
    G.ws[g] = wss[g].data_ptr<float>();
    G.dx[g] = (uint16_t*)dx.data_ptr();
    G.dgamma[g] = dg.data_ptr<float>();
    G.dbeta[g] = db.data_ptr<float>();
    res.push_back(dx);
    res.push_back(dg);
    res.push_back(db);
  }
  return res;
}

static void group_reduce_scratch(BnGroups& G, int64_t M, std::vector<at::Tensor>& keep, const at::Tensor& like) {
  int Cs[kMaxBnGroups];
  for (int g = 0; g < G.n; ++g) Cs[g] = G.C[g];
  const int rows = bn_group_bwd_rows(M, Cs, G.n);
  for (int g = 0; g < G.n; ++g) {
    keep.push_back(at::empty({(int64_t)rows * G.C[g] * 2}, like.options().dtype(at::kFloat)));
    G.wpart[g] = keep.back().data_ptr<float>();
  }
}

// dy of branch g read in place from channels [off_g, off_g + C_g) of dout
std::vector<at::Tensor> bn_concat_bwd(at::Tensor dout, std::vector<at::Tensor> ys, std::vector<at::Tensor> gammas,
                                      std::vector<at::Tensor> wss, std::vector<at::Tensor> dx_out) {
  check_act(dout, "dout");
  TORCH_CHECK(dout.dim() == 4 && dout.scalar_type() == at::kBFloat16, "bn_concat_bwd: dout must be bf16 [N, Ctot, H, W]");
  BnGroups G{};
  std::vector<at::Tensor> outs;
  for (size_t g = 0; g < dx_out.size(); ++g) outs.push_back(dx_out[g]);
  auto res = group_bwd_fields(G, ys, gammas, wss, outs);
  int64_t off = 0;
  for (int g = 0; g < G.n; ++g) {
    (void)check_branch(ys[g], dout, "y");
    G.dy[g] = (const uint16_t*)dout.data_ptr() + off;
    G.lddy[g] = dout.size(1);
    off += G.C[g];
  }
  TORCH_CHECK(off == dout.size(1), "bn_concat_bwd: branch channels must add up to dout's channels");
  const int64_t M = rows_of(dout);
  std::vector<at::Tensor> keep;
  group_reduce_scratch(G, M, keep, dout);
  if (M > 0) launch_bn_group_bwd(G, false, M, current_stream(dout));
  return res;
}

// dys: one gradient per branch; exts: the consumer dgrad epilogues' reduction partials for every
// branch, or empty (then a grouped reduce pass runs)
std::vector<at::Tensor> bn_group_bwd(std::vector<at::Tensor> dys, std::vector<at::Tensor> ys,
                                     std::vector<at::Tensor> gammas, std::vector<at::Tensor> wss,
                                     std::vector<at::Tensor> exts, std::vector<at::Tensor> dx_out) {
  BnGroups G{};
  auto res = group_bwd_fields(G, ys, gammas, wss, dx_out);
  TORCH_CHECK((int)dys.size() == G.n && (exts.empty() || (int)exts.size() == G.n),
              "bn_group_bwd: one dy (and optionally one partials tensor) per branch");
  std::vector<at::Tensor> keep;
  for (int g = 0; g < G.n; ++g) {
    check_act(dys[g], "dy");
    TORCH_CHECK(dys[g].sizes() == ys[g].sizes() && dys[g].scalar_type() == at::kBFloat16, "bn_group_bwd: dy must match y");
    G.dy[g] = (const uint16_t*)dys[g].data_ptr();
    G.lddy[g] = 0;
    if (!exts.empty()) {
      const at::Tensor& e = exts[g];
      TORCH_CHECK(e.is_cuda() && e.scalar_type() == at::kFloat && e.is_contiguous() && e.dim() == 3 &&
                      e.size(1) == G.C[g] && e.size(2) == 2,
                  "bn_group_bwd: partials must be fp32 [rows, C, 2]");
      G.part[g] = e.data_ptr<float>();
      G.nrb[g] = (int)e.size(0);
      keep.push_back(at::empty({std::max<int64_t>(1, (int64_t)bn_fold_groups((int)e.size(0)) * G.C[g] * 2)},
                               e.options()));
      G.wpart[g] = keep.back().data_ptr<float>();
    }
  }
  const int64_t M = rows_of(ys[0]);
  if (exts.empty()) group_reduce_scratch(G, M, keep, ys[0]);
  if (M > 0) launch_bn_group_bwd(G, !exts.empty(), M, current_stream(ys[0]));
  return res;
}

// DLA_GEMM_SPLITK=0 keeps every gemm_nt on the tile kernel (A/B runs)
static bool split_k_nt() {
  static const bool v = [] {
    const char* e = std::getenv("DLA_GEMM_SPLITK");
    return !(e && e[0] == '0');
  }();
  return v;
}

std::vector<at::Tensor> gemm_nt(at::Tensor A, at::Tensor B, bool stats, c10::optional<at::Tensor> addend,
                                bool b_kmajor, int64_t tile, c10::optional<at::Tensor> addend_mask,
                                c10::optional<at::Tensor> addend2, int64_t H, int64_t W) {
  TORCH_CHECK(tile >= 0 && tile <= kTile256x256, "gemm_nt: tile config 0..8");
  check_mat(A, "A");
  check_mat(B, "B");
  TORCH_CHECK(A.size(1) == B.size(b_kmajor ? 0 : 1), "gemm_nt: K mismatch");
  const int M = (int)A.size(0), N = (int)B.size(b_kmajor ? 1 : 0), K = (int)A.size(1);
  const bool add = addend.has_value() && addend->defined();
  if (add) {
    check_mat(*addend, "addend");
    TORCH_CHECK(addend->size(0) == M && addend->size(1) == N, "gemm_nt: addend must be [M, N]");
  }
  at::Tensor C = at::empty({M, N}, A.options());
  check_span(C, "gemm_nt output");
  at::Tensor S;
  // memory-bound short-K shapes: the persistent streaming kernel (forward with statistics, data gradient
  // with the fused identity-gradient addend + ReLU-bit mask; not the stride-2 second addend)
  const bool add2 = addend2.has_value() && addend2->defined();
  const bool mask = addend_mask.has_value() && addend_mask->defined();
  const bool stream_ok = tile == kTileAuto && !add2 && (!mask || add) &&
                         (!add || (b_kmajor && !stats && addend->stride(0) > 0 && addend->stride(0) % 8 == 0 &&
                                   (int64_t)M * addend->stride(0) * 2 < (int64_t(1) << 31)));
  const int srows = stream_ok ? gemm_stream_rows(M, N, K, A.stride(0), C.stride(0), b_kmajor, add) : 0;
  if (srows > 0) {
    if (stats) S = at::empty({srows, N, 2}, A.options().dtype(at::kFloat));
    TORCH_CHECK(launch_gemm_stream(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), b_kmajor, C.data_ptr(),
                                   C.stride(0), M, N, K, stats ? S.data_ptr<float>() : nullptr, current_stream(A),
                                   add ? addend->data_ptr() : nullptr, add ? addend->stride(0) : 0,
                                   addend_mask_ptr(addend_mask, M, N, add)),
                "gemm_nt: streaming kernel refused a shape it planned");
    return {C, S};
  }
  if (stats) S = at::empty({gemm_nt_stats_rows(M, N, (int)tile, K, !add), N, 2},
                           A.options().dtype(at::kFloat));
  // split-K only for the fully connected heads' shape class: no epilogue features beyond a bias row
  // (a full addend is a conv dgrad's residual sum, whose bitwise result must not depend on which
  // path — tile or split-K — the same sum takes, tests/test_gpu_bn_epilogue.py)
  const bool plain = !stats && tile == kTileAuto && !(addend_mask.has_value() && addend_mask->defined()) &&
                     !(addend2.has_value() && addend2->defined()) && (!add || addend->stride(0) == 0);
  const int splits = plain && M > 0 && N > 0 && split_k_nt() ? gemm_nt_splitk_splits(M, N, K) : 1;
  if (splits > 1) {  // few output tiles, long K (fully connected heads): split-K + fp32 slab reduce
    at::Tensor P = at::empty({(int64_t)splits * M * N}, A.options().dtype(at::kFloat));
    launch_gemm_nt_splitk(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), b_kmajor, P.data_ptr<float>(), splits,
                          C.data_ptr(), M, N, K, add ? addend->data_ptr() : nullptr, add ? addend->stride(0) : 0,
                          current_stream(A));
    return {C, S};
  }
  if (M > 0 && N > 0)
    launch_gemm_nt(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0), M, N, K,
                   stats ? S.data_ptr<float>() : nullptr, current_stream(A), add ? addend->data_ptr() : nullptr,
                   add ? addend->stride(0) : 0, b_kmajor, (int)tile, nullptr, addend_mask_ptr(addend_mask, M, N, add),
                   addend2_ptr(addend2, M, N, H, W), (int)H, (int)W);
  return {C, S};
}

// 1x1-conv forward over a deferred act(BN(y) + r) (gemm_apply.hip): writes out (the BN's output) and its ReLU
// mask, returns (C = out @ B^T, statistics [gemm_apply_rows][N][2] or undefined). y, r, out: bf16 [M, K]
// contiguous rows; B [N, K]; ws / wsd the 7K workspaces (wsd: r is the shortcut BN's input).
std::vector<at::Tensor> gemm_nt_apply(at::Tensor y, at::Tensor r, at::Tensor ws, c10::optional<at::Tensor> wsd,
                                      at::Tensor B, bool stats, at::Tensor out, at::Tensor mask,
                                      c10::optional<at::Tensor> xs, int64_t H, int64_t W) {
  check_mat(y, "y");
  check_mat(r, "r");
  check_mat(out, "out");
  check_mat(B, "B");
  const int64_t M = y.size(0);
  const int K = (int)y.size(1), N = (int)B.size(0);
  TORCH_CHECK(y.is_contiguous() && r.is_contiguous() && out.is_contiguous() && B.is_contiguous() &&
                  r.sizes() == y.sizes() && out.sizes() == y.sizes() && B.size(1) == K,
              "gemm_nt_apply: y, r, out contiguous [M, K], B contiguous [N, K]");
  TORCH_CHECK(gemm_apply_ok(M, N, K), "gemm_nt_apply: shape not served (check gemm_apply_ok)");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() == 7 * (int64_t)K, "ws: 7K fp32");
  const bool dual = wsd.has_value() && wsd->defined();
  if (dual)
    TORCH_CHECK(wsd->scalar_type() == at::kFloat && wsd->is_contiguous() && wsd->numel() == 7 * (int64_t)K, "wsd: 7K fp32");
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.numel() * 8 >= M * K, "mask: one bit per element");
  const bool sub = xs.has_value() && xs->defined();
  if (sub) {
    TORCH_CHECK(H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0 && M % (H * W) == 0, "gemm_nt_apply: xs needs even H, W");
    TORCH_CHECK(xs->is_cuda() && xs->scalar_type() == at::kBFloat16 && xs->dim() == 4 &&
                    xs->is_contiguous(at::MemoryFormat::ChannelsLast) && xs->size(0) == M / (H * W) &&
                    xs->size(1) == K && xs->size(2) == H / 2 && xs->size(3) == W / 2 &&
                    (reinterpret_cast<uintptr_t>(xs->data_ptr()) & 15) == 0,
                "gemm_nt_apply: xs must be a channels_last bf16 [n, K, H/2, W/2] tensor");
  }
  at::Tensor C = at::empty({M, N}, y.options());
  at::Tensor S;
  if (stats) S = at::empty({gemm_apply_rows(M), N, 2}, y.options().dtype(at::kFloat));
  launch_gemm_apply(y.data_ptr(), r.data_ptr(), ws.data_ptr<float>(), dual ? wsd->data_ptr<float>() : nullptr,
                    out.data_ptr(), mask.data_ptr<uint8_t>(), B.data_ptr(), B.stride(0), C.data_ptr(), (int)M, N, K,
                    stats ? S.data_ptr<float>() : nullptr, current_stream(y), sub ? xs->data_ptr() : nullptr, (int)H,
                    (int)W);
  return {C, S};
}

bool gemm_nt_apply_ok(int64_t M, int64_t N, int64_t K) { return gemm_apply_ok(M, (int)N, (int)K); }

// 1x1-conv forward with statistics over a deferred BN+ReLU output on the streaming GEMM (gemm_stream.hip kAp):
// y the BN input [M, K] (contiguous), ws its 7K workspace; writes out = relu(BN(y)) and returns (C, statistics
// [gemm_stream_rows][N][2]). Only shapes the streaming kernel plans (gemm_stream_rows(M, N, K, K, N, false) > 0).
std::vector<at::Tensor> gemm_nt_stream_apply(at::Tensor y, at::Tensor ws, at::Tensor B, at::Tensor out) {
  check_mat(y, "y");
  check_mat(B, "B");
  check_mat(out, "out");
  const int64_t M = y.size(0);
  const int K = (int)y.size(1), N = (int)B.size(0);
  TORCH_CHECK(y.is_contiguous() && out.is_contiguous() && out.sizes() == y.sizes() && B.size(1) == K,
              "gemm_nt_stream_apply: y, out contiguous [M, K], B [N, K]");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() == 7 * (int64_t)K, "ws: 7K fp32");
  const int rows = gemm_stream_rows(M, N, K, K, N, false, false, false);
  TORCH_CHECK(rows > 0, "gemm_nt_stream_apply: shape not served by the streaming kernel");
  at::Tensor C = at::empty({M, N}, y.options());
  at::Tensor S = at::empty({rows, N, 2}, y.options().dtype(at::kFloat));
  TORCH_CHECK(launch_gemm_stream(y.data_ptr(), K, B.data_ptr(), B.stride(0), false, C.data_ptr(), N, (int)M, N, K,
                                 S.data_ptr<float>(), current_stream(y), nullptr, 0, nullptr, nullptr,
                                 ws.data_ptr<float>(), out.data_ptr()),
              "gemm_nt_stream_apply: the streaming kernel refused a shape it planned");
  return {C, S};
}

bool gemm_nt_stream_apply_ok(int64_t M, int64_t N, int64_t K) {
  return M > 0 && K % 8 == 0 && gemm_stream_rows(M, (int)N, (int)K, K, N, false, false, false) > 0;
}

// gemm_nt whose output is the dy of a fused BN: also returns that BN's backward-reduction partials.
std::vector<at::Tensor> gemm_nt_bn(at::Tensor A, at::Tensor B, c10::optional<at::Tensor> addend, bool b_kmajor,
                                   at::Tensor x_bn, at::Tensor ws, c10::optional<at::Tensor> mask, int64_t mode,
                                   c10::optional<at::Tensor> addend_mask, c10::optional<at::Tensor> addend2, int64_t H,
                                   int64_t W) {
  check_mat(A, "A");
  check_mat(B, "B");
  TORCH_CHECK(A.size(1) == B.size(b_kmajor ? 0 : 1), "gemm_nt_bn: K mismatch");
  const int M = (int)A.size(0), N = (int)B.size(b_kmajor ? 1 : 0), K = (int)A.size(1);
  const bool add = addend.has_value() && addend->defined();
  if (add) {
    check_mat(*addend, "addend");
    TORCH_CHECK(addend->size(0) == M && addend->size(1) == N, "gemm_nt_bn: addend must be [M, N]");
  }
  at::Tensor C = at::empty({M, N}, A.options());
  check_span(C, "gemm_nt_bn output");
  at::Tensor part;
  // short-K data gradients: the persistent streaming kernel, whose epilogue loads x while the next tile's
  // rows are already in flight (the tile kernel's epilogue loads stall its block)
  const bool add2 = addend2.has_value() && addend2->defined();
  const bool amask = addend_mask.has_value() && addend_mask->defined();
  const bool stream_ok = b_kmajor && !add2 && (!amask || add) &&
                         (!add || (addend->stride(0) > 0 && addend->stride(0) % 8 == 0 &&
                                   (int64_t)M * addend->stride(0) * 2 < (int64_t(1) << 31)));
  const int srows = stream_ok ? gemm_stream_rows(M, N, K, A.stride(0), C.stride(0), b_kmajor, add, true) : 0;
  if (srows > 0) {
    const BnBwdArgs sb = make_bn_bwd(x_bn, ws, mask, mode, M, N, srows, part);
    if (launch_gemm_stream(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), b_kmajor, C.data_ptr(), C.stride(0), M,
                           N, K, nullptr, current_stream(A), add ? addend->data_ptr() : nullptr,
                           add ? addend->stride(0) : 0, addend_mask_ptr(addend_mask, M, N, add), &sb))
      return {C, part};
  }
  const BnBwdArgs bnb = make_bn_bwd(x_bn, ws, mask, mode, M, N, gemm_nt_stats_rows(M, N, kTileAuto, K, false), part);
  launch_gemm_nt(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0), M, N, K, nullptr,
                 current_stream(A), add ? addend->data_ptr() : nullptr, add ? addend->stride(0) : 0, b_kmajor,
                 kTileAuto, &bnb, addend_mask_ptr(addend_mask, M, N, add), addend2_ptr(addend2, M, N, H, W), (int)H,
                 (int)W);
  return {C, part};
}

// ---- fp32 convolutions (conv_f32.hip) ------------------------------------------------------------------------
// x: [N, C, H, W] in channels_last memory (NHWC) or a channel slice of such a tensor, fp32; w: [Cout, R, S, C]
// contiguous fp32 (OHWI). Returns y [N, Cout,
// OH, OW] channels_last, or adds into `out` (same shape / layout) when given.
static void check_nhwc_f32(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.scalar_type() == at::kFloat, what, ": 4-D fp32 CUDA tensor");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), what, ": channels_last memory");
  check_span(t, what);
}

// channels_last, or a channel slice of a channels_last tensor: unit channel stride, pixel stride ldp >= C (a multiple of
// 4, 16-byte aligned base); returns ldp
static int64_t check_nhwc_f32_slice(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.scalar_type() == at::kFloat, what, ": 4-D fp32 CUDA tensor");
  const int64_t ldp = t.stride(3);
  const bool ok = t.stride(1) == 1 && ldp >= t.size(1) && t.stride(2) == ldp * t.size(3) &&
                  t.stride(0) == t.stride(2) * t.size(2) && ldp % 4 == 0 && (uintptr_t)t.data_ptr() % 16 == 0;
  TORCH_CHECK(ok || t.is_contiguous(at::MemoryFormat::ChannelsLast), what,
              ": channels_last memory or a 16-byte aligned channel slice of it");
  check_span(t, what);
  return t.is_contiguous(at::MemoryFormat::ChannelsLast) ? t.size(1) : ldp;
}

at::Tensor conv_f32_fwd(at::Tensor x, at::Tensor w, int64_t pad, int64_t stride, c10::optional<at::Tensor> out) {
  const int64_t ldx = check_nhwc_f32_slice(x, "conv_f32_fwd x");
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kFloat && w.is_contiguous(),
              "conv_f32_fwd: w must be a contiguous fp32 [Cout, R, S, C] tensor");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int Cout = (int)w.size(0), R = (int)w.size(1), S = (int)w.size(2);
  TORCH_CHECK(w.size(3) == C, "conv_f32_fwd: weight channels ", w.size(3), " != input channels ", C);
  TORCH_CHECK(stride >= 1 && pad >= 0, "conv_f32_fwd: bad stride / padding");
  const int OH = (H + 2 * (int)pad - R) / (int)stride + 1, OW = (W + 2 * (int)pad - S) / (int)stride + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "conv_f32_fwd: empty output");
  TORCH_CHECK(conv_f32_supported(C, Cout, (int64_t)N * OH * OW, R * S * C),
              "conv_f32_fwd: needs C % 4 == 0, Cout % 4 == 0 and fewer than 2^24 output pixels");
  at::Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    check_nhwc_f32(y, "conv_f32_fwd out");
    TORCH_CHECK(y.size(0) == N && y.size(1) == Cout && y.size(2) == OH && y.size(3) == OW, "conv_f32_fwd: out shape");
  } else {
    y = at::empty({N, Cout, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  launch_conv_f32_fwd(x.data_ptr<float>(), ldx, N, H, W, C, w.data_ptr<float>(), Cout, R, S, (int)pad, (int)stride,
                      y.data_ptr<float>(), out.has_value() && out->defined(), current_stream(x));
  return y;
}

// dw [Cout, R, S, C] of a conv with input x (channels_last fp32) and output gradient dy (channels_last fp32)
at::Tensor conv_f32_wgrad(at::Tensor dy, at::Tensor x, int64_t R, int64_t S, int64_t pad, int64_t stride) {
  check_nhwc_f32(dy, "conv_f32_wgrad dy");
  const int64_t ldx = check_nhwc_f32_slice(x, "conv_f32_wgrad x");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), Cout = (int)dy.size(1);
  const int OH = (H + 2 * (int)pad - (int)R) / (int)stride + 1, OW = (W + 2 * (int)pad - (int)S) / (int)stride + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == OH && dy.size(3) == OW, "conv_f32_wgrad: dy shape does not match x");
  const int64_t M = (int64_t)N * OH * OW;
  const int K = (int)(R * S * C);
  TORCH_CHECK(conv_f32_supported(C, Cout, M, K), "conv_f32_wgrad: needs C % 4 == 0, Cout % 4 == 0, M < 2^24");
  at::Tensor dw = at::empty({Cout, R, S, C}, x.options());
  const int splits = conv_f32_wgrad_splits(M, Cout, K);
  at::Tensor part = at::empty({(int64_t)splits * Cout * K}, x.options());
  launch_conv_f32_wgrad(dy.data_ptr<float>(), x.data_ptr<float>(), ldx, N, H, W, C, Cout, (int)R, (int)S, (int)pad,
                        (int)stride, part.data_ptr<float>(), splits, dw.data_ptr<float>(), false, current_stream(x));
  return dw;
}

// out = scale * A^T @ B with A [K, Mo], B [K, No] (reduction over the long row dim, split-K).
at::Tensor gemm_tn(at::Tensor A, at::Tensor B, c10::ScalarType out_dtype, double scale) {
  check_mat(A, "A");
  check_mat(B, "B");
  TORCH_CHECK(A.size(0) == B.size(0), "gemm_tn: K mismatch");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "gemm_tn: fp32/bf16 output");
  const int K = (int)A.size(0), Mo = (int)A.size(1), No = (int)B.size(1);
  at::Tensor out = at::empty({Mo, No}, A.options().dtype(out_dtype));
  const int splits = gemm_tn_splits(Mo, No, K);
  at::Tensor part = at::empty({(int64_t)splits * Mo * No}, A.options().dtype(at::kFloat));
  launch_gemm_tn(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), part.data_ptr<float>(), splits, Mo, No, K,
                 out.data_ptr(), out_dtype == at::kFloat ? kF32 : kBF16, (float)scale, false, current_stream(A));
  return out;
}

// Data and weight gradient of a stride-1 1x1 conv in one pass over dy (gemm_dual.hip): dy [M, Cout], x [M, Cin]
// rows, w [Cout, Cin]. Returns (dx [M, Cin] bf16, dw [Cout, Cin] out_dtype), or an empty list when the shape
// is not served (the caller then runs gemm_nt + gemm_tn).
// With y_bn (+ ws, mask): dy is the incoming gradient of the BN(+residual)+ReLU whose input y_bn is this conv's
// output; its backward apply (bit-mask ReLU, finalized ws) runs inside the kernel.
std::vector<at::Tensor> conv1x1_dual(at::Tensor dy, at::Tensor x, at::Tensor w, c10::ScalarType out_dtype,
                                     c10::optional<at::Tensor> y_bn, c10::optional<at::Tensor> ws,
                                     c10::optional<at::Tensor> mask) {
  check_mat(dy, "dy");
  check_mat(x, "x");
  TORCH_CHECK(w.is_cuda() && w.dim() == 2 && w.scalar_type() == at::kBFloat16 && w.is_contiguous(),
              "conv1x1_dual: w must be a contiguous bf16 [Cout, Cin] matrix");
  TORCH_CHECK(dy.size(0) == x.size(0) && w.size(0) == dy.size(1) && w.size(1) == x.size(1), "conv1x1_dual: shapes");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "conv1x1_dual: fp32/bf16 weight gradient");
  const int64_t M = dy.size(0);
  const int Cout = (int)dy.size(1), Cin = (int)x.size(1);
  const int groups = conv1x1_dual_groups(M, Cin, Cout);
  if (!groups || dy.stride(0) != Cout || x.stride(0) != Cin) return {};
  const bool bn = y_bn.has_value() && y_bn->defined();
  if (bn) {
    if (!conv1x1_dual_bn_ok(M, Cin, Cout)) return {};
    check_mat(*y_bn, "y_bn");
    TORCH_CHECK(y_bn->sizes() == dy.sizes() && y_bn->stride(0) == Cout, "conv1x1_dual: y_bn must be laid out like dy");
    TORCH_CHECK(ws.has_value() && ws->scalar_type() == at::kFloat && ws->is_contiguous() && ws->numel() == 7 * Cout,
                "conv1x1_dual: ws must be the BN's finalized 7C workspace");
    TORCH_CHECK(mask.has_value() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() * 8 >= M * Cout,
                "conv1x1_dual: the BN's 1-bit ReLU mask");
  }
  at::Tensor dx = at::empty({M, Cin}, dy.options());
  at::Tensor part = at::empty({(int64_t)groups * Cout * Cin}, dy.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({Cout, Cin}, dy.options().dtype(out_dtype));
  hipStream_t st = current_stream(dy);
  TORCH_CHECK(launch_conv1x1_dual(dy.data_ptr(), x.data_ptr(), w.data_ptr(), dx.data_ptr(), part.data_ptr<float>(), M,
                                  Cin, Cout, st, bn ? y_bn->data_ptr() : nullptr,
                                  bn ? mask->data_ptr<uint8_t>() : nullptr, bn ? ws->data_ptr<float>() : nullptr),
              "conv1x1_dual: kernel refused a shape it planned");
  launch_splitk_reduce(part.data_ptr<float>(), groups, (int64_t)Cout * Cin, dw.data_ptr(),
                       out_dtype == at::kFloat ? kF32 : kBF16, 1.f, false, st);
  return {dx, dw};
}

static int pool_out(int in, int k, int s, int p, bool ceil_mode);

// Stem BatchNorm (training) + ReLU + max-pool: returns (y_pool, ws, pos). x is the BN input
// (channels_last bf16); y_pool/pos [N, C, OH, OW] channels_last.
std::vector<at::Tensor> bn_relu_maxpool_fwd(at::Tensor x, c10::optional<at::Tensor> weight,
                                            c10::optional<at::Tensor> bias, c10::optional<at::Tensor> running_mean,
                                            c10::optional<at::Tensor> running_var, double momentum, double eps,
                                            int64_t k, int64_t s, int64_t p, c10::optional<at::Tensor> stats,
                                            bool ceil_mode) {
  check_act(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.scalar_type() == at::kBFloat16, "bn_relu_maxpool: bf16 4-D input");
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && p >= 0 && 2 * p <= k, "bn_relu_maxpool: unsupported window");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int64_t M = (int64_t)N * H * W;
  TORCH_CHECK(M < (1 << 24), "bn_relu_maxpool: too many pixels for 24-bit index math");
  // ceil mode (GoogLeNet) only adds trailing windows that start inside the input; the kernels skip
  // their out-of-range taps and the backward gather clamps to OH/OW
  const int OH = pool_out(H, (int)k, (int)s, (int)p, ceil_mode), OW = pool_out(W, (int)k, (int)s, (int)p, ceil_mode);
  auto f32 = x.options().dtype(at::kFloat);
  auto fptr = [](const c10::optional<at::Tensor>& t) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "BN parameters/stats must be fp32 contiguous");
    return t->data_ptr<float>();
  };
  at::Tensor ws = at::empty({7 * (int64_t)C}, f32);
  const bool ext = stats.has_value() && stats->defined();
  if (ext) {
    TORCH_CHECK(stats->scalar_type() == at::kFloat && stats->is_contiguous() && stats->dim() == 3 &&
                    stats->size(1) == C && stats->size(2) == 2,
                "stats must be fp32 [row_blocks, C, 2] partials");
  }
  at::Tensor part = at::empty({ext ? ext_part_floats(stats, C) : partial_floats(M, C)}, f32);
  launch_bn_fwd(x.data_ptr(), nullptr, nullptr, M, C, kBF16, fptr(weight), fptr(bias), (float)eps, (float)momentum,
                fptr(running_mean), fptr(running_var), ws.data_ptr<float>(), part.data_ptr<float>(), true, true,
                current_stream(x), ext ? stats->data_ptr<float>() : nullptr, ext ? (int)stats->size(0) : 0);
  auto opts = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  at::Tensor y = at::empty({N, C, OH, OW}, opts);
  at::Tensor pos = at::empty({N, C, OH, OW}, opts.dtype(at::kByte));
  launch_bn_relu_maxpool_fwd(x.data_ptr(), ws.data_ptr<float>(), y.data_ptr(), pos.data_ptr<uint8_t>(), N, H, W, C, OH,
                             OW, (int)k, (int)s, (int)p, current_stream(x));
  return {y, ws, pos};
}

// Returns (dx, dgamma, dbeta) of the fused stem op, gathering dy from the pooled gradient.
std::vector<at::Tensor> bn_relu_maxpool_bwd(at::Tensor dy_pool, at::Tensor pos, at::Tensor x, at::Tensor ws,
                                            c10::optional<at::Tensor> weight, int64_t k, int64_t s, int64_t p,
                                            bool want_dx) {
  dy_pool = dy_pool.contiguous(at::MemoryFormat::ChannelsLast).to(at::kBFloat16);
  check_act(x, "x");
  TORCH_CHECK(pos.scalar_type() == at::kByte && pos.sizes() == dy_pool.sizes() &&
                  pos.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_relu_maxpool_bwd: pos must be the forward's positions");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int OH = (int)dy_pool.size(2), OW = (int)dy_pool.size(3);
  const int64_t M = (int64_t)N * H * W;
  auto f32 = x.options().dtype(at::kFloat);
  at::Tensor part = at::empty({bn_relu_maxpool_part_floats(M, C)}, f32);
  // want_dx false: the quad reduce + finalize only (ws then holds the backward coefficients); the stem weight
  // gradient applies them itself (stem_wgrad_bn). Only the quad form (3x3 / s2, even input, OH = H / 2) stops there.
  TORCH_CHECK(want_dx || (k == 3 && s == 2 && (p == 0 || p == 1) && H % 2 == 0 && W % 2 == 0 && OH == H / 2 &&
                          OW == W / 2),
              "bn_relu_maxpool_bwd: want_dx=False needs the quad form (3x3 / stride 2, even input)");
  at::Tensor dx = want_dx ? at::empty_like(x) : at::Tensor();
  at::Tensor dg = at::empty({C}, f32), db = at::empty({C}, f32);
  const float* g = (weight.has_value() && weight->defined()) ? weight->data_ptr<float>() : nullptr;
  launch_bn_relu_maxpool_bwd(dy_pool.data_ptr(), pos.data_ptr<uint8_t>(), x.data_ptr(),
                             want_dx ? dx.data_ptr() : nullptr, N, H, W, C, OH,
                             OW, (int)k, (int)s, (int)p, g, ws.data_ptr<float>(), part.data_ptr<float>(),
                             dg.data_ptr<float>(), db.data_ptr<float>(), current_stream(x));
  return {dx, dg, db};
}

static int pool_out(int in, int k, int s, int p, bool ceil_mode) {
  int o = (in + 2 * p - k + (ceil_mode ? s - 1 : 0)) / s + 1;
  if (ceil_mode && (int64_t)(o - 1) * s >= in + p) --o;  // last window must start inside the input
  return o;
}

// NHWC max pooling. Returns (y, pos); pos (uint8, same shape as y) is the window position of each
// maximum and is only produced when `need_pos` (training).
std::vector<at::Tensor> maxpool_fwd(at::Tensor x, int64_t k, int64_t s, int64_t p, bool ceil_mode, bool need_pos) {
  check_act(x, "x");
  TORCH_CHECK(x.dim() == 4, "maxpool: 4-D input");
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && p >= 0 && 2 * p <= k, "maxpool: unsupported window");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int OH = pool_out(H, (int)k, (int)s, (int)p, ceil_mode), OW = pool_out(W, (int)k, (int)s, (int)p, ceil_mode);
  TORCH_CHECK(OH > 0 && OW > 0, "maxpool: empty output");
  TORCH_CHECK((int64_t)N * H * W * (C / 8) < (1LL << 31), "maxpool: tensor too large for 32-bit indexing");
  auto opts = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  at::Tensor y = at::empty({N, C, OH, OW}, opts);
  at::Tensor pos;
  if (need_pos) pos = at::empty({N, C, OH, OW}, opts.dtype(at::kByte));
  launch_maxpool_fwd(x.data_ptr(), y.data_ptr(), need_pos ? pos.data_ptr<uint8_t>() : nullptr, N, H, W, C, OH, OW,
                     (int)k, (int)s, (int)p, dtype_code(x), current_stream(x));
  return {y, pos};
}

at::Tensor maxpool_bwd(at::Tensor dy, at::Tensor pos, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_act(dy, "dy");
  TORCH_CHECK(pos.scalar_type() == at::kByte && pos.sizes() == dy.sizes() &&
                  pos.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_bwd: pos must be the forward's uint8 positions");
  const int N = (int)dy.size(0), C = (int)dy.size(1), OH = (int)dy.size(2), OW = (int)dy.size(3);
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_maxpool_bwd(dy.data_ptr(), pos.data_ptr<uint8_t>(), dx.data_ptr(), N, (int)H, (int)W, C, OH, OW, (int)k,
                     (int)s, (int)p, dtype_code(dy), current_stream(dy));
  return dx;
}

// ResNet stem conv (7x7/s2/p3, 3 input channels). Returns (y, stats-or-undefined, xs) with xs the
// space-to-depth folded input the weight gradient reads.
std::vector<at::Tensor> stem_fwd(at::Tensor x, at::Tensor wpk, bool want_stats) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.size(1) == 3 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_fwd: x must be a bf16 channels_last [N, 3, H, W] GPU tensor");
  TORCH_CHECK(wpk.is_cuda() && wpk.dim() == 2 && wpk.size(1) == 256 && wpk.size(0) % 8 == 0 &&
                  wpk.scalar_type() == at::kBFloat16 && wpk.is_contiguous() &&
                  (reinterpret_cast<uintptr_t>(wpk.data_ptr()) & 15) == 0,
              "stem_fwd: wpk must be the packed bf16 [Cout, 256] weight");
  const int N = (int)x.size(0), H = (int)x.size(2), W = (int)x.size(3), Cout = (int)wpk.size(0);
  const int OH = (H + 1) / 2, OW = (W + 1) / 2;  // 7x7 / s2 / p3
  const int64_t P = (int64_t)N * OH * OW;
  TORCH_CHECK(P < (1 << 24), "stem_fwd: too many output pixels for 24-bit index math");
  at::Tensor xs = at::empty({N, OH, OW, 16}, x.options().memory_format(at::MemoryFormat::Contiguous));
  launch_stem_fold(x.data_ptr(), xs.data_ptr(), N, H, W, current_stream(x));
  at::Tensor y = at::empty({N, Cout, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor stats;
  if (want_stats) stats = at::empty({stem_stats_rows(P, Cout), Cout, 2}, x.options().dtype(at::kFloat));
  launch_stem_fwd(xs.data_ptr(), wpk.data_ptr(), y.data_ptr(), N, H, W, Cout,
                  want_stats ? stats.data_ptr<float>() : nullptr, current_stream(x));
  return {y, stats, xs};
}

// The stem weight gradient with the stem BN+ReLU+max-pool backward apply fused (stem.hip stem_wgrad_bn_kernel):
// dy_pool / pos from the pooled op, x = the conv output (the BN input), ws = the coefficients a
// bn_relu_maxpool_bwd(..., want_dx=False) finalized. The conv output's gradient is never materialised.
at::Tensor stem_wgrad_bn(at::Tensor dy_pool, at::Tensor pos, at::Tensor x, at::Tensor ws, at::Tensor xs, int64_t H,
                         int64_t W, c10::ScalarType out_dtype) {
  dy_pool = dy_pool.contiguous(at::MemoryFormat::ChannelsLast).to(at::kBFloat16);
  check_act(x, "x");
  check_act(dy_pool, "dy_pool");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 4, "stem_wgrad_bn: x must be the bf16 conv output");
  TORCH_CHECK(pos.scalar_type() == at::kByte && pos.sizes() == dy_pool.sizes() &&
                  pos.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_wgrad_bn: pos must be the pooled op's positions");
  TORCH_CHECK(xs.is_cuda() && xs.dim() == 4 && xs.size(3) == 16 && xs.scalar_type() == at::kBFloat16 &&
                  xs.is_contiguous(),
              "stem_wgrad_bn: xs must be the forward's folded [N, OH, OW, 16] input");
  const int N = (int)x.size(0), Cout = (int)x.size(1), OH = (int)dy_pool.size(2), OW = (int)dy_pool.size(3);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() == 7 * (int64_t)Cout,
              "stem_wgrad_bn: ws must be the 7C workspace");
  TORCH_CHECK(xs.size(0) == N && xs.size(1) == (H + 1) / 2 && xs.size(2) == (W + 1) / 2 && x.size(2) == xs.size(1) &&
                  x.size(3) == xs.size(2) && dy_pool.size(0) == N && dy_pool.size(1) == Cout,
              "stem_wgrad_bn: x / xs / dy_pool / image size mismatch");
  TORCH_CHECK(stem_wgrad_bn_eligible(N, (int)H, (int)W, Cout, OH, OW),
              "stem_wgrad_bn: needs 64 channels, an even conv output and a 3x3 / s2 / p1 pool");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "stem_wgrad_bn: fp32/bf16 output");
  const int splits = stem_wgrad_bn_splits(N, (int)H, (int)W);
  at::Tensor part = at::empty({(int64_t)splits * Cout * 256}, xs.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({Cout, 256}, xs.options().dtype(out_dtype));
  launch_stem_wgrad_bn(dy_pool.data_ptr(), pos.data_ptr<uint8_t>(), x.data_ptr(), ws.data_ptr<float>(), xs.data_ptr(),
                       part.data_ptr<float>(), splits, dw.data_ptr(), out_dtype == at::kFloat ? kF32 : kBF16, N,
                       (int)H, (int)W, OH, OW, current_stream(xs));
  return dw;
}

at::Tensor stem_wgrad(at::Tensor dy, at::Tensor xs, int64_t H, int64_t W, c10::ScalarType out_dtype) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(xs.is_cuda() && xs.dim() == 4 && xs.size(3) == 16 && xs.scalar_type() == at::kBFloat16 &&
                  xs.is_contiguous(),
              "stem_wgrad: xs must be the forward's folded [N, OH, OW, 16] input");
  check_act(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.size(1) % 64 == 0, "stem_wgrad: dy must be bf16, Cout % 64");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "stem_wgrad: fp32/bf16 output");
  const int N = (int)xs.size(0), Cout = (int)dy.size(1);
  TORCH_CHECK(xs.size(1) == (H + 1) / 2 && xs.size(2) == (W + 1) / 2, "stem_wgrad: xs / image size mismatch");
  TORCH_CHECK((int64_t)N * xs.size(1) * xs.size(2) < (1 << 24), "stem_wgrad: too many output pixels");
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == xs.size(1) && dy.size(3) == xs.size(2), "stem_wgrad: dy shape");
  const int splits = stem_wgrad_splits(N, (int)H, (int)W, Cout);
  at::Tensor part = at::empty({(int64_t)splits * Cout * 256}, xs.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({Cout, 256}, xs.options().dtype(out_dtype));
  launch_stem_wgrad(dy.data_ptr(), xs.data_ptr(), part.data_ptr<float>(), splits, dw.data_ptr(),
                    out_dtype == at::kFloat ? kF32 : kBF16, N, (int)H, (int)W, Cout, current_stream(xs));
  return dw;
}

// x[:, :, ::2, ::2] of a channels_last bf16 activation as a compact channels_last tensor (the
// stride-2 downsample conv's input)
at::Tensor subsample2(at::Tensor x) {
  check_act(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.scalar_type() == at::kBFloat16 && x.size(1) % 8 == 0 && x.size(2) % 2 == 0 &&
                  x.size(3) % 2 == 0,
              "subsample2: bf16 [N, C % 8, even H, even W]");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  TORCH_CHECK((int64_t)N * (H / 2) * (W / 2) * (C / 8) < (1ll << 32), "subsample2: too large");
  at::Tensor y = at::empty({N, C, H / 2, W / 2}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_subsample2(x.data_ptr(), y.data_ptr(), N, H, W, C, current_stream(x));
  return y;
}

// Global average pooling: x [N, C, H, W] channels_last -> y [N, C] (the flattened head input).
at::Tensor gap_fwd(at::Tensor x) {
  check_act(x, "x");
  TORCH_CHECK(x.dim() == 4, "global_avg_pool: 4-D input");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "global_avg_pool: bf16 or fp32");
  const int N = (int)x.size(0), C = (int)x.size(1), HW = (int)(x.size(2) * x.size(3));
  at::Tensor y = at::empty({N, C}, x.options().memory_format(at::MemoryFormat::Contiguous));
  if (N > 0 && HW > 0) launch_gap_fwd(x.data_ptr(), y.data_ptr(), N, HW, C, dtype_code(x), current_stream(x));
  return y;
}

at::Tensor gap_bwd(at::Tensor dy, int64_t H, int64_t W) {
  dy = dy.contiguous();
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 2 && dy.size(1) % 8 == 0, "global_avg_pool_bwd: dy [N, C], C % 8 == 0");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kFloat, "global_avg_pool_bwd: bf16 or fp32");
  const int N = (int)dy.size(0), C = (int)dy.size(1);
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_gap_bwd(dy.data_ptr(), dx.data_ptr(), N, (int)(H * W), C, dtype_code(dy), current_stream(dy));
  return dx;
}

static void check_conv3(const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3: x must be a bf16 channels_last 4-D GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.scalar_type() == at::kBFloat16 && w.size(2) == 3 && w.size(3) == 3 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3: w must be a bf16 channels_last [Cout, Cin, 3, 3] tensor");
  TORCH_CHECK(w.size(1) == x.size(1), "conv3x3: channel mismatch");
  TORCH_CHECK(x.size(1) % 8 == 0 && w.size(0) % 8 == 0, "conv3x3: Cin and Cout must be multiples of 8");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(w.data_ptr()) & 15) == 0,
              "conv3x3: 16-byte aligned operands required");
  TORCH_CHECK(x.numel() / x.size(1) < (1 << 24), "conv3x3: too many pixels for 24-bit index math");
  check_span(x, "conv3x3 input");
  TORCH_CHECK(x.numel() / x.size(1) * w.size(0) * 2 < (int64_t(1) << 31),
              "conv3x3: the output reaches the 2 GiB buffer-descriptor range (lower the per-GPU batch)");
}

// 3x3 / pad 1 convolution forward (stride 1 or 2). Returns (y, stats-or-undefined).
std::vector<at::Tensor> conv3x3_fwd(at::Tensor x, at::Tensor w, int64_t stride, bool stats, int64_t tile) {
  TORCH_CHECK(tile >= 0 && tile <= kTile512x128, "conv3x3: tile config 0..9");
  check_conv3(x, w);
  TORCH_CHECK(stride == 1 || stride == 2, "conv3x3: stride 1 or 2");
  TORCH_CHECK(x.size(1) % 64 == 0 || tile_bm(tile) * tile_bn(tile) <= 128 * 128,
              "conv3x3: Cin % 64 != 0 needs a tile of at most 128x128");
  const int N = (int)x.size(0), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), Cout = (int)w.size(0);
  const int OH = (H - 1) / (int)stride + 1, OW = (W - 1) / (int)stride + 1;
  at::Tensor y = at::empty({N, Cout, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor S;
  const int64_t P = (int64_t)N * OH * OW;
  if (stats) S = at::empty({conv3x3_stats_rows(P, Cout, (int)tile, 9 * Cin, Cin % 64 == 0), Cout, 2}, x.options().dtype(at::kFloat));
  launch_conv3x3_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), N, H, W, Cin, Cout, (int)stride,
                     stats ? S.data_ptr<float>() : nullptr, current_stream(x), (int)tile);
  return {y, S};
}

// stride-1 data gradient (+ optional fused addend, same shape as dx)
at::Tensor conv3x3_dgrad(at::Tensor dy, at::Tensor w, c10::optional<at::Tensor> addend, int64_t tile) {
  TORCH_CHECK(tile >= 0 && tile <= kTile512x128, "conv3x3: tile config 0..9");
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(dy.dim() == 4 && dy.size(1) == w.size(0), "conv3x3_dgrad: dy/w mismatch");
  const int N = (int)dy.size(0), Cout = (int)w.size(0), Cin = (int)w.size(1), H = (int)dy.size(2), W = (int)dy.size(3);
  at::Tensor dx = at::empty({N, Cin, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_conv3(dx, w);
  TORCH_CHECK(Cout % 64 == 0 || tile_bm(tile) * tile_bn(tile) <= 128 * 128,
              "conv3x3_dgrad: Cout % 64 != 0 needs a tile of at most 128x128");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0,
              "conv3x3_dgrad: bf16 aligned dy");
  const void* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->sizes() == dx.sizes() && addend->scalar_type() == at::kBFloat16 &&
                    addend->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv3x3_dgrad: addend must match dx");
    add = addend->data_ptr();
  }
  if (tile == 0 && halo_conv_eligible(Cout, Cin, W, 1, false)) {
    // stride-1 data gradient = the forward conv of dy with W'[ci][kh][kw][co] = W[co][2-kh][2-kw][ci]
    const at::Tensor wt = w.flip({2, 3}).transpose(0, 1).contiguous(at::MemoryFormat::ChannelsLast);
    launch_conv3x3_halo(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), N, H, W, nullptr, current_stream(dy), add);
    return dx;
  }
  launch_conv3x3_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, add, current_stream(dy),
                       (int)tile);
  return dx;
}

// stride-2 3x3 data gradient for an input of even size H x W
at::Tensor conv3x3s2_dgrad(at::Tensor dy, at::Tensor w, int64_t H, int64_t W) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(dy.dim() == 4 && dy.size(1) == w.size(0), "conv3x3s2_dgrad: dy/w mismatch");
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0 && dy.size(2) == H / 2 && dy.size(3) == W / 2,
              "conv3x3s2_dgrad: needs even H, W and dy = [N, Cout, H/2, W/2]");
  const int N = (int)dy.size(0), Cout = (int)w.size(0), Cin = (int)w.size(1);
  at::Tensor dx = at::empty({N, Cin, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_conv3(dx, w);
  TORCH_CHECK(Cin % 64 == 0 && Cout % 64 == 0, "conv3x3s2_dgrad: Cin and Cout must be multiples of 64");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0,
              "conv3x3s2_dgrad: bf16 aligned dy");
  launch_conv3x3s2_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, (int)H, (int)W, Cin, Cout,
                         current_stream(dy));
  return dx;
}

// stride-1 3x3 data gradient that is the dy of a fused BN: returns (dx, BN-backward partials)
std::vector<at::Tensor> conv3x3_dgrad_bn(at::Tensor dy, at::Tensor w, c10::optional<at::Tensor> addend,
                                         at::Tensor x_bn, at::Tensor ws, c10::optional<at::Tensor> mask, int64_t mode) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(dy.dim() == 4 && dy.size(1) == w.size(0), "conv3x3_dgrad_bn: dy/w mismatch");
  const int N = (int)dy.size(0), Cout = (int)w.size(0), Cin = (int)w.size(1), H = (int)dy.size(2), W = (int)dy.size(3);
  at::Tensor dx = at::empty({N, Cin, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_conv3(dx, w);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0,
              "conv3x3_dgrad_bn: bf16 aligned dy");
  const void* add = nullptr;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->sizes() == dx.sizes() && addend->scalar_type() == at::kBFloat16 &&
                    addend->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv3x3_dgrad_bn: addend must match dx");
    add = addend->data_ptr();
  }
  const int64_t P = (int64_t)N * H * W;
  at::Tensor part;
  const BnBwdArgs bnb = make_bn_bwd(x_bn, ws, mask, mode, P, Cin, conv3x3_stats_rows(P, Cin, kTileAuto, 9 * Cout, Cout % 64 == 0), part);
  launch_conv3x3_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), N, H, W, Cin, Cout, add, current_stream(dy),
                       kTileAuto, &bnb);
  return {dx, part};
}

// weight gradient, returned as a channels_last [Cout, Cin, 3, 3] tensor of out_dtype
at::Tensor conv3x3_wgrad(at::Tensor dy, at::Tensor x, int64_t stride, c10::ScalarType out_dtype) {
  dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.scalar_type() == at::kBFloat16 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0,
              "conv3x3_wgrad: x must be bf16 channels_last with Cin % 8 == 0");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.size(1) % 8 == 0, "conv3x3_wgrad: dy must be bf16, Cout % 8");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "conv3x3_wgrad: fp32/bf16 output");
  TORCH_CHECK(x.numel() / x.size(1) < (1 << 24), "conv3x3_wgrad: too many pixels");
  const int N = (int)x.size(0), Cin = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), Cout = (int)dy.size(1);
  TORCH_CHECK(dy.size(2) == (H - 1) / stride + 1 && dy.size(3) == (W - 1) / stride + 1, "conv3x3_wgrad: dy shape");
  at::Tensor dw = at::empty({Cout, Cin, 3, 3}, x.options().dtype(out_dtype).memory_format(at::MemoryFormat::ChannelsLast));
  if (halo_wgrad_eligible(Cin, Cout, W, (int)stride) && (int64_t)N * (H + 2) * (W + 2) < (1 << 30)) {
    const int hs = halo_wgrad_splits(N, H, W);
    at::Tensor hpart = at::empty({(int64_t)hs * Cout * 9 * Cin}, x.options().dtype(at::kFloat));
    launch_conv3x3_halo_wgrad(dy.data_ptr(), x.data_ptr(), hpart.data_ptr<float>(), hs, dw.data_ptr(),
                              out_dtype == at::kFloat ? kF32 : kBF16, N, H, W, current_stream(x));
    return dw;
  }
  const int splits = conv3x3_wgrad_splits(N, H, W, Cin, Cout, (int)stride);
  at::Tensor part = at::empty({(int64_t)splits * Cout * 9 * Cin}, x.options().dtype(at::kFloat));
  launch_conv3x3_wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr<float>(), splits, dw.data_ptr(),
                       out_dtype == at::kFloat ? kF32 : kBF16, N, H, W, Cin, Cout, (int)stride, current_stream(x));
  return dw;
}

void bind_nn(pybind11::module& m) {
  m.def("gemm_nt_bn", &gemm_nt_bn, "gemm_nt producing a fused BN's dy plus its backward-reduction partials",
        pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("addend"), pybind11::arg("b_kmajor"),
        pybind11::arg("x_bn"), pybind11::arg("ws"), pybind11::arg("mask"), pybind11::arg("mode"),
        pybind11::arg("addend_mask") = pybind11::none(), pybind11::arg("addend2") = pybind11::none(),
        pybind11::arg("H") = 0, pybind11::arg("W") = 0);
  m.def("conv3x3_dgrad_bn", &conv3x3_dgrad_bn, "3x3 dgrad producing a fused BN's dy plus its backward partials",
        pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("addend"), pybind11::arg("x_bn"), pybind11::arg("ws"),
        pybind11::arg("mask"), pybind11::arg("mode"));
  m.def("set_mfma_pipeline", &set_mfma_pipeline, "MFMA main loop: 0 register staging, 2/3 LDS-DMA stages, -1 per-shape auto");
  m.def("set_gemm_stream", &set_gemm_stream, "persistent streaming 1x1 GEMM: -1 environment (default on), 0 off, 1 on");
  m.def("set_gemm_persist", &set_gemm_persist, "persistent register-stored 1x1 GEMM: blocks per CU (0 off, -1 env)");
  m.def("set_gemm_direct", &set_gemm_direct, "register-stored 128x128 1x1 GEMM tiles: -1 environment (default off), 0 / 1");
  m.def("gemm_stream_rows", &gemm_stream_rows, "BN-statistics partial rows of the streaming GEMM (0: shape not served)",
        pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("K"), pybind11::arg("lda"), pybind11::arg("ldc"), pybind11::arg("b_kmajor") = false,
        pybind11::arg("add") = false, pybind11::arg("bnb") = false);
  m.def("mfma_pipeline", &mfma_pipeline);
  m.def("set_tile256_min_k_stats", &set_tile256_min_k_stats, "smallest K of the auto 256x256 tiles of statistics forwards (A/B)");
  m.def("set_tile256_min_k", &set_tile256_min_k, "smallest K of the auto 256x256 gemm_nt / conv tiles (A/B; <= 0 default 1024)");
  m.def("set_tn256", &set_tn256, "256x256 weight-gradient tiles: -1 environment (DLA_TN256, default on), 0 off, 1 on");
  m.def("set_splitk_blocks", &set_splitk_blocks, "split-K weight-gradient block target (0 = default / DLA_SPLITK_BLOCKS)");
  m.def("splitk_target_blocks", &splitk_target_blocks);
  m.def("set_bn_red_blocks", &set_bn_red_blocks, "BN reduction-pass block target (0 = default / DLA_BN_RED_BLOCKS)");
  m.def("bn_red_blocks", &bn_red_blocks);
  m.def("conv3x3_fwd", &conv3x3_fwd, "implicit-GEMM 3x3/pad-1 conv forward (NHWC bf16, MFMA)", pybind11::arg("x"),
        pybind11::arg("w"), pybind11::arg("stride") = 1, pybind11::arg("stats") = false, pybind11::arg("tile") = 0);
  m.def("conv3x3_dgrad", &conv3x3_dgrad, "implicit-GEMM 3x3 conv data gradient (stride 1)", pybind11::arg("dy"),
        pybind11::arg("w"), pybind11::arg("addend") = pybind11::none(), pybind11::arg("tile") = 0);
  m.def("conv3x3s2_dgrad", &conv3x3s2_dgrad, "implicit-GEMM 3x3 / stride-2 conv data gradient (parity classes)",
        pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("H"), pybind11::arg("W"));
  m.def("conv3x3_wgrad", &conv3x3_wgrad, "implicit-GEMM 3x3 conv weight gradient (split-K)", pybind11::arg("dy"),
        pybind11::arg("x"), pybind11::arg("stride") = 1, pybind11::arg("out_dtype") = at::kFloat);
  m.def("bn_relu_maxpool_fwd", &bn_relu_maxpool_fwd, "stem BN(train)+ReLU+max-pool forward (pooled output only)",
        pybind11::arg("x"), pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("running_mean"),
        pybind11::arg("running_var"), pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("k"),
        pybind11::arg("s"), pybind11::arg("p"), pybind11::arg("stats") = pybind11::none(),
        pybind11::arg("ceil_mode") = false);
  m.def("bn_relu_maxpool_bwd", &bn_relu_maxpool_bwd, "stem BN+ReLU+max-pool backward (dy gathered from the pool)",
        pybind11::arg("dy_pool"), pybind11::arg("pos"), pybind11::arg("x"), pybind11::arg("ws"), pybind11::arg("weight"),
        pybind11::arg("k"), pybind11::arg("s"), pybind11::arg("p"), pybind11::arg("want_dx") = true);
  m.def("maxpool_fwd", &maxpool_fwd, "NHWC max pooling forward (+ argmax window positions)", pybind11::arg("x"),
        pybind11::arg("k"), pybind11::arg("s"), pybind11::arg("p"), pybind11::arg("ceil_mode") = false,
        pybind11::arg("need_pos") = true);
  m.def("maxpool_bwd", &maxpool_bwd, "NHWC max pooling backward (gather form)");
  m.def("bn_dual_fwd", &bn_dual_fwd, "training act(BN(x) + BN_d(xd)) in one apply pass (downsample residual)",
        pybind11::arg("x"), pybind11::arg("xd"), pybind11::arg("weight"), pybind11::arg("bias"),
        pybind11::arg("running_mean"), pybind11::arg("running_var"), pybind11::arg("weight_d"), pybind11::arg("bias_d"),
        pybind11::arg("running_mean_d"), pybind11::arg("running_var_d"), pybind11::arg("momentum"),
        pybind11::arg("momentum_d"), pybind11::arg("eps"), pybind11::arg("eps_d"), pybind11::arg("relu"),
        pybind11::arg("stats"), pybind11::arg("stats_d"), pybind11::arg("defer") = false);
  m.def("bn_apply_deferred", &bn_apply_deferred, "the apply pass of a deferred bn_act_fwd / bn_dual_fwd (ReLU, residual)",
        pybind11::arg("x"), pybind11::arg("r"), pybind11::arg("ws"), pybind11::arg("wsd"), pybind11::arg("y"),
        pybind11::arg("mask"));
  m.def("gemm_nt_apply", &gemm_nt_apply,
        "1x1-conv forward over a deferred act(BN(y) + r): writes the BN output + mask and returns (C, stats)",
        pybind11::arg("y"), pybind11::arg("r"), pybind11::arg("ws"), pybind11::arg("wsd"), pybind11::arg("B"),
        pybind11::arg("stats"), pybind11::arg("out"), pybind11::arg("mask"), pybind11::arg("xs") = pybind11::none(),
        pybind11::arg("H") = 0, pybind11::arg("W") = 0);
  m.def("gemm_nt_apply_ok", &gemm_nt_apply_ok, "shapes gemm_nt_apply serves (M rows, N outputs, K channels)");
  m.def("gemm_nt_stream_apply", &gemm_nt_stream_apply,
        "streaming 1x1-conv forward over a deferred BN+ReLU output: writes relu(BN(y)) and returns (C, stats)",
        pybind11::arg("y"), pybind11::arg("ws"), pybind11::arg("B"), pybind11::arg("out"));
  m.def("gemm_nt_stream_apply_ok", &gemm_nt_stream_apply_ok, "shapes gemm_nt_stream_apply serves (M, N, K)");
  m.def("set_gemm256_direct", &set_gemm256_direct, "256x256 statistics forwards stored from registers (-1 env, 0, 1)");
  m.def("set_stem_stream", &set_stem_stream, "stem forward on the persistent streaming GEMM (-1 env, 0, 1)");
  m.def("set_wgrad_w4", &set_wgrad_w4, "128x256 tiles for the Cout-128 3x3 weight gradients (-1 env, 0, 1)");
  m.def("set_gemm_apply_max_k", &set_gemm_apply_max_k, "largest K gemm_nt_apply serves (<= 0: environment / 512)");
  m.def("bn_dual_bwd", &bn_dual_bwd, "backward of bn_dual_fwd (one dy read for both BatchNorms)", pybind11::arg("dy"),
        pybind11::arg("mask"), pybind11::arg("x"), pybind11::arg("ws"), pybind11::arg("weight"), pybind11::arg("xd"),
        pybind11::arg("wsd"), pybind11::arg("weight_d"), pybind11::arg("want_dx") = true);
  m.def("gap_fwd", &gap_fwd, "NHWC global average pooling -> [N, C]");
  m.def("subsample2", &subsample2, "x[:, :, ::2, ::2] of a channels_last bf16 tensor, compact channels_last");
  m.def("stem_fwd", &stem_fwd, "7x7/s2/p3 stem conv, 3 input channels (space-to-depth + MFMA implicit GEMM, BN-statistics epilogue)");
  m.def("stem_wgrad_bn", &stem_wgrad_bn,
        "stem weight gradient with the BN+ReLU+max-pool backward apply fused (the conv-output gradient never stored)");
  m.def("stem_wgrad", &stem_wgrad, "7x7/s2/p3 stem conv weight gradient from the folded input (packed [Cout, 256] layout)");
  m.def("gap_bwd", &gap_bwd, "NHWC global average pooling backward (channels_last dx)");
  m.def("gemm_nt", &gemm_nt, "C = A @ B^T (bf16 MFMA), optional fused column statistics", pybind11::arg("A"),
        pybind11::arg("B"), pybind11::arg("stats") = false, pybind11::arg("addend") = pybind11::none(),
        pybind11::arg("b_kmajor") = false, pybind11::arg("tile") = 0,
        pybind11::arg("addend_mask") = pybind11::none(), pybind11::arg("addend2") = pybind11::none(),
        pybind11::arg("H") = 0, pybind11::arg("W") = 0);
  m.def("gemm_nt_splitk_splits", [](int64_t M, int64_t N, int64_t K) { return gemm_nt_splitk_splits((int)M, (int)N, (int)K); },
        "split count gemm_nt uses for this shape (1 = tile kernel)");
  m.def("pick_tile", [](int64_t M, int64_t N, int64_t K, bool wide_ok) { return pick_tile(M, (int)N, kTileAuto, (int)K, wide_ok); },
        "tile config the auto policy picks for an M x N GEMM with reduction K (TileCfg: 1 = 128x128, 2 = 128x64, 8 = 256x256)");
  m.def("pick_conv_tile", [](int64_t P, int64_t N, int64_t K, bool wide_ok) { return pick_conv_tile(P, (int)N, kTileAuto, (int)K, wide_ok); },
        "tile of a 3x3 forward / data-gradient launch (pick_tile + the conv-only 512x128 tile)");
  m.def("gemm_tn_splits", [](int64_t Mo, int64_t No, int64_t K) { return gemm_tn_splits((int)Mo, (int)No, (int)K); },
        "split-K count of a weight-gradient gemm_tn launch");
  m.def("set_halo_wgrad", &set_halo_wgrad, "halo 64-channel 3x3 weight gradient: -1 environment (default on), 0 off, 1 on");
  m.def("halo_wgrad_eligible", [](int64_t Cin, int64_t Cout, int64_t W, int64_t stride) {
        return halo_wgrad_eligible((int)Cin, (int)Cout, (int)W, (int)stride); });
  m.def("halo_conv_eligible", [](int64_t Cin, int64_t Cout, int64_t W, int64_t stride, bool fwd) {
        return halo_conv_eligible((int)Cin, (int)Cout, (int)W, (int)stride, fwd); },
        "whether a 3x3 conv pass runs on the halo-tiled kernel (conv_halo.hip) under the current DLA_HALO mode");
  m.def("conv1x1_dual_blocks", [](int64_t M, int64_t Cin, int64_t Cout) { return conv1x1_dual_blocks(M, (int)Cin, (int)Cout); },
        "blocks of the one-pass dgrad + wgrad 1x1 kernel for this shape (0: not served)");
  m.def("conv1x1_dual", &conv1x1_dual, "stride-1 1x1 conv data + weight gradient in one pass over dy",
        pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("out_dtype") = at::kFloat,
        pybind11::arg("y_bn") = pybind11::none(), pybind11::arg("ws") = pybind11::none(),
        pybind11::arg("mask") = pybind11::none());
  m.def("conv1x1_dual_bn_ok", [](int64_t M, int64_t Cin, int64_t Cout) { return conv1x1_dual_bn_ok(M, (int)Cin, (int)Cout); },
        "the one-pass 1x1 gradient kernel can also apply the consuming BN's backward for this shape");
  m.def("conv_f32_fwd", &conv_f32_fwd, "fp32 implicit-GEMM convolution (v_mfma_f32_16x16x4_f32), NHWC / OHWI",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("pad"), pybind11::arg("stride") = 1,
        pybind11::arg("out") = c10::nullopt);
  m.def("set_conv_f32_buffers", &set_conv_f32_buffers, "fp32 conv main loop: 1 or 2 (default) LDS buffers");
  m.def("conv_f32_wgrad", &conv_f32_wgrad, "fp32 convolution weight gradient [Cout, R, S, C] (split over pixels)",
        pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("R"), pybind11::arg("S"), pybind11::arg("pad"),
        pybind11::arg("stride") = 1);
  m.def("gemm_tn", &gemm_tn, "A^T @ B (bf16 MFMA, split-K over rows)", pybind11::arg("A"), pybind11::arg("B"),
        pybind11::arg("out_dtype") = at::kFloat, pybind11::arg("scale") = 1.0);
  m.def("bn_act_fwd", &bn_act_fwd, "fused BatchNorm(+residual)(+ReLU) forward, NHWC", pybind11::arg("x"),
        pybind11::arg("residual"), pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("running_mean"),
        pybind11::arg("running_var"), pybind11::arg("training"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("relu"), pybind11::arg("stats") = pybind11::none(), pybind11::arg("out") = pybind11::none(),
        pybind11::arg("out_channel") = 0, pybind11::arg("defer") = false);
  m.def("bn_concat_fwd", &bn_concat_fwd, "grouped training BN+ReLU of concatenated branches into one NHWC output");
  m.def("bn_concat_bwd", &bn_concat_bwd, "backward of bn_concat_fwd (dy slices read in place)", pybind11::arg("dout"),
        pybind11::arg("ys"), pybind11::arg("weights"), pybind11::arg("wss"),
        pybind11::arg("dx_out") = std::vector<at::Tensor>{});
  m.def("bn_group_fwd", &bn_group_fwd, "grouped training BN+ReLU of same-size tensors, one output each");
  m.def("bn_group_bwd", &bn_group_bwd, "backward of bn_group_fwd (optionally from dgrad-epilogue partials)",
        pybind11::arg("dys"), pybind11::arg("ys"), pybind11::arg("weights"), pybind11::arg("wss"),
        pybind11::arg("exts") = std::vector<at::Tensor>{}, pybind11::arg("dx_out") = std::vector<at::Tensor>{});
  m.def("bn_act_bwd", &bn_act_bwd, "fused BatchNorm(+residual)(+ReLU) backward, NHWC", pybind11::arg("dy"),
        pybind11::arg("y"), pybind11::arg("mask"), pybind11::arg("x"), pybind11::arg("ws"), pybind11::arg("weight"),
        pybind11::arg("mask_mode"), pybind11::arg("need_dres"), pybind11::arg("ext_part") = pybind11::none(),
        pybind11::arg("want_dx") = true);
}

}  // namespace dla
