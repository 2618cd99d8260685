// Python bindings for the fused network-layer kernels (csrc/kernels/bnact.hip).  Kept out of
// bindings.cpp so the codec bindings do not recompile when these change.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "grace_kernels.h"

namespace {

using at::Tensor;
inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

// [M, C] row-major view of an NHWC (channels_last) or 2-D activation
void check_rows(const Tensor& t, const char* what, int64_t* M, int64_t* C) {
  TORCH_CHECK(t.is_cuda() && (t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat), what,
              " must be a bf16 or fp32 GPU tensor");
  if (t.dim() == 4) {
    TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), what, " must be channels_last");
    *C = t.size(1);
  } else {
    TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), what, " must be [M, C] contiguous or NHWC");
    *C = t.size(1);
  }
  *M = t.numel() / std::max<int64_t>(*C, 1);
  TORCH_CHECK(grace::bn_supported((int)*C), what, ": channels must be a multiple of 8, <= 2048, and a multiple of 256 above 256");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what, " must be 16-byte aligned");
}

void same_layout(const Tensor& a, const Tensor& b, const char* what) {
  TORCH_CHECK(a.sizes() == b.sizes() && a.strides() == b.strides() && b.scalar_type() == a.scalar_type() &&
                  (reinterpret_cast<uintptr_t>(b.data_ptr()) & 15) == 0,
              what, " must match the input's shape, strides and dtype");
}

const float* opt_f32(const c10::optional<Tensor>& t, int64_t C, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C, what,
              " must be a contiguous fp32 [C] GPU tensor");
  return t->data_ptr<float>();
}

// returns (y, save[6C] = mean, invstd, scale, shift, backward totals [2C] (zeroed), relu mask [M*C/8] uint8 (undefined without relu))
bool bn_supported(int64_t C) { return grace::bn_supported((int)C); }

std::vector<Tensor> bn_act_fwd(const Tensor& x, const c10::optional<Tensor>& res, const c10::optional<Tensor>& weight,
                               const c10::optional<Tensor>& bias, const c10::optional<Tensor>& running_mean,
                               const c10::optional<Tensor>& running_var, const c10::optional<Tensor>& nbt,
                               double momentum, double eps, bool relu) {
  int64_t M, C;
  check_rows(x, "x", &M, &C);
  const bool has_res = res.has_value() && res->defined();
  if (has_res) same_layout(x, *res, "residual");
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean / running_var: both or neither");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "num_batches_tracked");
    nb = nbt->data_ptr<int64_t>();
  }
  DevGuard guard(x.device());
  Tensor y = at::empty_like(x);
  auto f32 = x.options().dtype(at::kFloat);
  Tensor save = at::empty({6 * C}, f32);  // + the backward's atomic totals [2C]
  // ReLU: 1 bit per element (bit j of byte i = output element 8i+j > 0), read by the backward
  Tensor mask = relu ? at::empty({M * C / 8}, x.options().dtype(at::kByte)) : Tensor();
  Tensor ws = at::empty({grace::bn_workspace_floats(M, (int)C)}, f32);
  grace::bn_act_forward(x.data_ptr(), has_res ? res->data_ptr() : nullptr, x.scalar_type() == at::kFloat, M, (int)C,
                        opt_f32(weight, C, "weight"), opt_f32(bias, C, "bias"), rm, rv, nb, (float)momentum,
                        (float)eps, relu, save.data_ptr<float>(), ws.data_ptr<float>(),
                        y.data_ptr(), relu ? mask.data_ptr<uint8_t>() : nullptr, cur_stream());
  return {y, save, mask};
}

// fp32 forward from the conv GEMM's epilogue statistics ([tiles][2][C] partial sums)
std::vector<Tensor> bn_act_fwd_partials(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& part,
                                        int64_t tiles, const c10::optional<Tensor>& weight,
                                        const c10::optional<Tensor>& bias, const c10::optional<Tensor>& running_mean,
                                        const c10::optional<Tensor>& running_var, const c10::optional<Tensor>& nbt,
                                        double momentum, double eps, bool relu) {
  int64_t M, C;
  check_rows(x, "x", &M, &C);
  TORCH_CHECK(x.scalar_type() == at::kFloat, "bn_act_fwd_partials: fp32 activations");
  const bool has_res = res.has_value() && res->defined();
  if (has_res) same_layout(x, *res, "residual");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  tiles >= 1 && part.numel() >= tiles * 2 * C, "partials: fp32 [tiles][2][C]");
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean / running_var: both or neither");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "num_batches_tracked");
    nb = nbt->data_ptr<int64_t>();
  }
  DevGuard guard(x.device());
  Tensor y = at::empty_like(x);
  Tensor save = at::empty({6 * C}, x.options());
  Tensor mask = relu ? at::empty({M * C / 8}, x.options().dtype(at::kByte)) : Tensor();
  Tensor fws = at::empty({grace::bn_fold_ws_doubles(tiles, C)}, x.options().dtype(at::kDouble));
  grace::bn_act_forward_from_partials(x.data_ptr<float>(), has_res ? res->data_ptr<float>() : nullptr,
                                      part.data_ptr<float>(), (int)tiles, M, (int)C, opt_f32(weight, C, "weight"),
                                      opt_f32(bias, C, "bias"), rm, rv, nb, (float)momentum, (float)eps, relu,
                                      save.data_ptr<float>(), y.data_ptr<float>(),
                                      relu ? mask.data_ptr<uint8_t>() : nullptr, cur_stream(), fws.data_ptr<double>());
  return {y, save, mask};
}

// BN statistics pass only (no apply) over an fp32 channels_last activation: save [6C], running
// statistics updated; the apply runs in the consumer GEMM's prologue
Tensor bn_stats_only(const Tensor& x, const c10::optional<Tensor>& weight, const c10::optional<Tensor>& bias,
                     const c10::optional<Tensor>& running_mean, const c10::optional<Tensor>& running_var,
                     const c10::optional<Tensor>& nbt, double momentum, double eps) {
  int64_t M, C;
  check_rows(x, "x", &M, &C);
  TORCH_CHECK(x.scalar_type() == at::kFloat, "bn_stats_only: fp32 activations");
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean / running_var: both or neither");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "num_batches_tracked");
    nb = nbt->data_ptr<int64_t>();
  }
  DevGuard guard(x.device());
  Tensor save = at::empty({6 * C}, x.options());
  Tensor ws = at::empty({grace::bn_workspace_floats(M, (int)C)}, x.options());
  grace::bn_stats_only(x.data_ptr<float>(), M, (int)C, opt_f32(weight, C, "weight"), opt_f32(bias, C, "bias"), rm, rv,
                       nb, (float)momentum, (float)eps, save.data_ptr<float>(), ws.data_ptr<float>(), cur_stream());
  return save;
}

// BN statistics from GEMM partials only: save [6C] (mean, invstd, scale, shift, 0, 0), running
// statistics and num_batches_tracked updated; the apply runs in the consumer GEMM's prologue
Tensor bn_fold_partials(const Tensor& part, int64_t tiles, int64_t M, int64_t C, const c10::optional<Tensor>& weight,
                        const c10::optional<Tensor>& bias, const c10::optional<Tensor>& running_mean,
                        const c10::optional<Tensor>& running_var, const c10::optional<Tensor>& nbt, double momentum,
                        double eps) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && tiles >= 1 &&
                  part.numel() >= tiles * 2 * C && M >= 1 && C >= 1, "partials: fp32 [tiles][2][C]");
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean / running_var: both or neither");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "num_batches_tracked");
    nb = nbt->data_ptr<int64_t>();
  }
  DevGuard guard(part.device());
  Tensor save = at::empty({6 * C}, part.options());
  Tensor fws = at::empty({grace::bn_fold_ws_doubles(tiles, C)}, part.options().dtype(at::kDouble));
  grace::bn_fold_partials(part.data_ptr<float>(), (int)tiles, M, (int)C, opt_f32(weight, C, "weight"),
                          opt_f32(bias, C, "bias"), rm, rv, nb, (float)momentum, (float)eps, save.data_ptr<float>(),
                          cur_stream(), fws.data_ptr<double>());
  return save;
}

// returns (dx, dres (undefined unless want_dres), dweight, dbias)
std::vector<Tensor> bn_act_bwd(const Tensor& dy, const c10::optional<Tensor>& dy2, const Tensor& x,
                               const c10::optional<Tensor>& mask, const c10::optional<Tensor>& weight,
                               const Tensor& save, bool relu, bool want_dres, bool want_dweight,
                               bool deterministic, const c10::optional<Tensor>& dweight_out,
                               const c10::optional<Tensor>& dbias_out) {
  int64_t M, C;
  check_rows(x, "x", &M, &C);
  same_layout(x, dy, "grad_output");
  const bool two = dy2.has_value() && dy2->defined();
  if (two) same_layout(x, *dy2, "second grad_output");
  const bool has_mask = mask.has_value() && mask->defined();
  if (relu && has_mask) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == M * C / 8,
                "relu backward: the forward's mask must be [M*C/8] uint8");
  }
  // relu without a mask: recomputed from x and save (scale, shift); one dy only
  TORCH_CHECK(!(relu && !has_mask && dy2.has_value() && dy2->defined()), "maskless relu backward takes one dy");
  TORCH_CHECK(save.is_cuda() && save.scalar_type() == at::kFloat && save.numel() == 6 * C, "save");
  DevGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor dx = at::empty_like(x);
  Tensor dres = want_dres ? at::empty_like(x) : Tensor();
  // dweight_out / dbias_out: the parameters' gradient buffers (a GRACE / DDP bucket view), written
  // in place so no copy into the bucket follows
  auto out_or = [&](const c10::optional<Tensor>& o) {
    if (o.has_value() && o->defined()) {
      TORCH_CHECK(o->is_cuda() && o->scalar_type() == at::kFloat && o->is_contiguous() && o->numel() == C &&
                      o->get_device() == x.get_device(), "bn_act_bwd: gradient output must be contiguous fp32 [C]");
      return *o;
    }
    return at::empty({C}, f32);
  };
  Tensor dg = want_dweight ? out_or(dweight_out) : Tensor();
  Tensor db = want_dweight ? out_or(dbias_out) : Tensor();
  Tensor coef = at::empty({3 * C}, f32);
  Tensor ws = at::empty({grace::bn_workspace_floats(M, (int)C)}, f32);
  grace::bn_act_backward(dy.data_ptr(), two ? dy2->data_ptr() : nullptr, x.data_ptr(), x.scalar_type() == at::kFloat,
                         relu && has_mask ? mask->data_ptr<uint8_t>() : nullptr, M, (int)C,
                         opt_f32(weight, C, "weight"), save.data_ptr<float>(), relu,
                         want_dweight ? dg.data_ptr<float>() : nullptr, want_dweight ? db.data_ptr<float>() : nullptr,
                         coef.data_ptr<float>(), ws.data_ptr<float>(), dx.data_ptr(),
                         want_dres ? dres.data_ptr() : nullptr, deterministic, cur_stream());
  return {dx, dres, dg, db};
}

// BN backward whose reduction came from the consumer conv's data-grad GEMM epilogue (part:
// [tiles][2][C] = [sum dz | sum dz (x - mean)]); dy is that GEMM's output (unmasked).
std::vector<Tensor> bn_act_bwd_partials(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& mask,
                                        const c10::optional<Tensor>& weight, const Tensor& save, const Tensor& part,
                                        int64_t tiles, bool relu, bool want_dweight,
                                        const c10::optional<Tensor>& dweight_out,
                                        const c10::optional<Tensor>& dbias_out) {
  int64_t M, C;
  check_rows(x, "x", &M, &C);
  same_layout(x, dy, "grad_output");
  TORCH_CHECK(x.scalar_type() == at::kFloat, "bn_act_bwd_partials: fp32 activations");
  const bool has_mask = mask.has_value() && mask->defined();
  if (has_mask)
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() && mask->numel() == M * C / 8,
                "mask [M*C/8] uint8");
  TORCH_CHECK(save.is_cuda() && save.scalar_type() == at::kFloat && save.numel() == 6 * C, "save");
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && tiles >= 1 &&
                  part.numel() >= tiles * 2 * C, "part [tiles][2][C]");
  DevGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  auto out_or = [&](const c10::optional<Tensor>& o) {
    if (o.has_value() && o->defined()) {
      TORCH_CHECK(o->is_cuda() && o->scalar_type() == at::kFloat && o->is_contiguous() && o->numel() == C &&
                      o->get_device() == x.get_device(), "bn_act_bwd_partials: gradient output must be contiguous fp32 [C]");
      return *o;
    }
    return at::empty({C}, f32);
  };
  Tensor dg = want_dweight ? out_or(dweight_out) : Tensor();
  Tensor db = want_dweight ? out_or(dbias_out) : Tensor();
  Tensor coef = at::empty({3 * C}, f32);
  Tensor dx = at::empty_like(x);
  Tensor fws = at::empty({grace::bn_fold_ws_doubles(tiles, C)}, x.options().dtype(at::kDouble));
  grace::bn_act_backward_from_partials(dy.data_ptr<float>(), x.data_ptr<float>(),
                                       relu && has_mask ? mask->data_ptr<uint8_t>() : nullptr, part.data_ptr<float>(),
                                       (int)tiles,
                                       M, (int)C, opt_f32(weight, C, "weight"), save.data_ptr<float>(), relu,
                                       want_dweight ? dg.data_ptr<float>() : nullptr,
                                       want_dweight ? db.data_ptr<float>() : nullptr, coef.data_ptr<float>(),
                                       dx.data_ptr<float>(), cur_stream(), fws.data_ptr<double>());
  return {dx, dg, db};
}

// Fused SGD over a list of fp32 parameters (dense, grads / momentum buffers / bf16 working copies
// with the parameter's strides).  bufs / w16 entries may be None.
void sgd_step(const std::vector<Tensor>& params, const std::vector<Tensor>& grads,
              const std::vector<c10::optional<Tensor>>& bufs, const std::vector<c10::optional<Tensor>>& w16,
              double lr, double momentum, double dampening, double wd, bool nesterov, bool maximize, bool first) {
  const size_t n = params.size();
  TORCH_CHECK(grads.size() == n && bufs.size() == n && w16.size() == n, "sgd_step: list lengths");
  if (n == 0) return;
  std::vector<float*> p(n), b(n);
  std::vector<const float*> g(n);
  std::vector<uint16_t*> w(n);
  std::vector<int64_t> len(n);
  for (size_t i = 0; i < n; ++i) {
    const Tensor& t = params[i];
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_non_overlapping_and_dense(),
                "sgd_step: parameters must be dense fp32 GPU tensors");
    TORCH_CHECK(t.device() == params[0].device(), "sgd_step: every parameter on one device");
    auto same = [&](const Tensor& u, at::ScalarType dt, const char* what) {
      bool ok = u.is_cuda() && u.scalar_type() == dt && u.sizes() == t.sizes();
      for (int64_t d = 0; ok && d < t.dim(); ++d)  // strides of size-1 dims do not move memory
        ok = t.size(d) == 1 || u.stride(d) == t.stride(d);
      TORCH_CHECK(ok, "sgd_step: ", what, " must match its parameter's shape, strides and expected dtype");
    };
    same(grads[i], at::kFloat, "grad");
    p[i] = t.data_ptr<float>();
    g[i] = grads[i].data_ptr<float>();
    b[i] = nullptr;
    if (bufs[i].has_value() && bufs[i]->defined()) {
      same(*bufs[i], at::kFloat, "momentum buffer");
      b[i] = bufs[i]->data_ptr<float>();
    }
    w[i] = nullptr;
    if (w16[i].has_value() && w16[i]->defined()) {
      same(*w16[i], at::kBFloat16, "bf16 working copy");
      w[i] = reinterpret_cast<uint16_t*>(w16[i]->data_ptr());
    }
    len[i] = t.numel();
  }
  DevGuard guard(params[0].device());
  grace::sgd_step(p.data(), g.data(), b.data(), w.data(), len.data(), (int)n, (float)lr, (float)momentum,
                  (float)dampening, (float)wd, nesterov, maximize, first, cur_stream());
}
// conv bias (+ ReLU): y = act(x + bias) for channels_last [N, C, H, W] x
Tensor bias_act_fwd(const Tensor& x, const Tensor& bias, bool relu) {
  int64_t M, C;
  check_rows(x, "x", &M, &C);
  const float* b = opt_f32(bias, C, "bias");
  TORCH_CHECK(b != nullptr, "bias required");
  DevGuard guard(x.device());
  Tensor y = at::empty_like(x);
  grace::bias_act_forward(x.data_ptr(), b, x.scalar_type() == at::kFloat, M, (int)C, relu, y.data_ptr(), cur_stream());
  return y;
}

// returns (dz = dy * [y > 0], dbias = sum over N, H, W of dz) in one pass
std::vector<Tensor> bias_act_bwd(const Tensor& dy, const Tensor& y, bool relu) {
  int64_t M, C;
  check_rows(y, "y", &M, &C);
  same_layout(y, dy, "grad_output");
  DevGuard guard(y.device());
  auto f32 = y.options().dtype(at::kFloat);
  Tensor dz = at::empty_like(y);
  Tensor db = at::empty({C}, f32);
  Tensor ws = at::empty({grace::bn_workspace_floats(M, (int)C)}, f32);
  grace::bias_act_backward(dy.data_ptr(), y.data_ptr(), y.scalar_type() == at::kFloat, M, (int)C, relu,
                           db.data_ptr<float>(), ws.data_ptr<float>(), dz.data_ptr(), cur_stream());
  return {dz, db};
}

// BN (training statistics, running stats) + ReLU + k x k max pool over channels_last x.
// returns (pooled y, save[6C], code)
std::vector<Tensor> bn_act_pool_fwd(const Tensor& x, const c10::optional<Tensor>& weight,
                                    const c10::optional<Tensor>& bias, const c10::optional<Tensor>& running_mean,
                                    const c10::optional<Tensor>& running_var, const c10::optional<Tensor>& nbt,
                                    double momentum, double eps, int64_t k, int64_t s, int64_t pad) {
  int64_t M, C;
  check_rows(x, "x", &M, &C);
  TORCH_CHECK(x.dim() == 4 && k >= 1 && k <= 15 && s >= 1 && pad >= 0 && 2 * pad <= k, "bn+pool: NHWC x, k <= 15");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 * pad - k) / s + 1, OW = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "bn+pool: empty output");
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean / running_var: both or neither");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "num_batches_tracked");
    nb = nbt->data_ptr<int64_t>();
  }
  DevGuard guard(x.device());
  auto f32 = x.options().dtype(at::kFloat);
  Tensor y = at::empty({N, C, OH, OW}, x.options(), at::MemoryFormat::ChannelsLast);
  Tensor code = at::empty({N, C, OH, OW}, x.options().dtype(at::kByte), at::MemoryFormat::ChannelsLast);
  Tensor save = at::empty({6 * C}, f32);  // + the backward's atomic totals [2C]
  Tensor ws = at::empty({grace::bn_workspace_floats(M, (int)C)}, f32);
  grace::bn_act_pool_forward(x.data_ptr(), x.scalar_type() == at::kFloat, (int)N, (int)H, (int)W, (int)C,
                             opt_f32(weight, C, "weight"), opt_f32(bias, C, "bias"), rm, rv, nb, (float)momentum,
                             (float)eps, (int)k, (int)s, (int)pad, (int)OH, (int)OW, save.data_ptr<float>(),
                             ws.data_ptr<float>(), y.data_ptr(), code.data_ptr<uint8_t>(), cur_stream());
  return {y, save, code};
}

// global average pool backward: dy [N, C] -> dx [N, C, H, W] channels_last
Tensor gap_bwd(const Tensor& dy, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 2 && dy.is_contiguous() &&
                  (dy.scalar_type() == at::kFloat || dy.scalar_type() == at::kBFloat16) && dy.size(1) % 8 == 0 &&
                  (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0,
              "gap backward: contiguous [N, C % 8 == 0] fp32/bf16 GPU grad");
  DevGuard guard(dy.device());
  Tensor dx = at::empty({dy.size(0), dy.size(1), H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  grace::global_avgpool_backward(dy.data_ptr(), dy.scalar_type() == at::kFloat, (int)dy.size(0), (int)(H * W),
                                 (int)dy.size(1), dx.data_ptr(), cur_stream());
  return dx;
}

// NHWC max pooling: returns (y, code) -- code = uint8 in-window argmax per output element
std::vector<Tensor> maxpool_fwd(const Tensor& x, int64_t k, int64_t s, int64_t pad) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "maxpool: channels_last fp32/bf16 GPU tensor");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0 && k >= 1 && k <= 15 && s >= 1 && pad >= 0 && 2 * pad <= k, "maxpool: unsupported shape");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0, "maxpool: 16-B aligned input");
  const int64_t OH = (H + 2 * pad - k) / s + 1, OW = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "maxpool: empty output");
  DevGuard guard(x.device());
  Tensor y = at::empty({N, C, OH, OW}, x.options(), at::MemoryFormat::ChannelsLast);
  Tensor code = at::empty({N, C, OH, OW}, x.options().dtype(at::kByte), at::MemoryFormat::ChannelsLast);
  grace::maxpool_forward(x.data_ptr(), x.scalar_type() == at::kFloat, (int)N, (int)H, (int)W, (int)C, (int)OH,
                         (int)OW, (int)k, (int)s, (int)pad, y.data_ptr(), code.data_ptr<uint8_t>(), cur_stream());
  return {y, code};
}

Tensor maxpool_bwd(const Tensor& dy, const Tensor& code, int64_t H, int64_t W, int64_t k, int64_t s, int64_t pad,
                   const c10::optional<Tensor>& dy2) {
  if (dy2.has_value())
    TORCH_CHECK(dy2->sizes() == dy.sizes() && dy2->scalar_type() == dy.scalar_type() &&
                    dy2->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    (reinterpret_cast<uintptr_t>(dy2->data_ptr()) & 15) == 0,
                "maxpool backward: dy2 like dy (channels_last, 16-B aligned)");
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0,
              "maxpool backward: channels_last 16-B aligned grad");
  TORCH_CHECK(code.sizes() == dy.sizes() && code.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  code.scalar_type() == at::kByte, "maxpool backward: code");
  const int64_t N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  DevGuard guard(dy.device());
  Tensor dx = at::empty({N, C, H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  grace::maxpool_backward(dy.data_ptr(), code.data_ptr<uint8_t>(), dy.scalar_type() == at::kFloat, (int)N, (int)H,
                          (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)pad, dx.data_ptr(), cur_stream(),
                          dy2.has_value() ? dy2->data_ptr() : nullptr);
  return dx;
}

}  // namespace

void grace_bind_nn(py::module& m) {
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("gap_bwd", &gap_bwd);
  m.def("bn_act_pool_fwd", &bn_act_pool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd, py::arg("dy"), py::arg("code"), py::arg("H"), py::arg("W"), py::arg("k"),
        py::arg("s"), py::arg("pad"), py::arg("dy2") = py::none());
  m.def("bias_act_fwd", &bias_act_fwd);
  m.def("bias_act_bwd", &bias_act_bwd);
  m.def("sgd_step", &sgd_step);
  m.def("bn_supported", &bn_supported);
  m.def("bn_fused_v", [](int64_t M, int64_t C, bool bwd) { return grace::bn_fused_v(M, (int)C, bwd); });
  m.def("bn_set_fused", &grace::bn_set_fused);
  m.def("bn_fused_v_f32", [](int64_t M, int64_t C, bool bwd) { return grace::bn_fused_v_f32(M, (int)C, bwd); });
  m.def("bn_set_fused_f32", &grace::bn_set_fused_f32);
  m.def("bn_spin_timeouts", []() { return (int64_t)grace::bn_spin_timeouts(); });
  m.def("bn_act_fwd", &bn_act_fwd);
  m.def("bn_act_bwd", &bn_act_bwd, py::arg("dy"), py::arg("dy2"), py::arg("x"), py::arg("mask"), py::arg("weight"),
        py::arg("save"), py::arg("relu"), py::arg("want_dres"), py::arg("want_dweight"), py::arg("deterministic"),
        py::arg("dweight_out") = py::none(), py::arg("dbias_out") = py::none());
  m.def("bn_set_deterministic", [](bool on) { grace::bn_set_deterministic(on); });
  m.def("bn_set_atomic_chunks", [](int64_t n) { grace::bn_set_atomic_chunks((int)n); });
  m.def("bn_atomic_chunks", []() { return (int64_t)grace::bn_atomic_chunks(); });
  m.def("bn_act_fwd_partials", &bn_act_fwd_partials);
  m.def("bn_fold_partials", &bn_fold_partials);
  m.def("bn_stats_only", &bn_stats_only);
  m.def("bn_act_bwd_partials", &bn_act_bwd_partials, py::arg("dy"), py::arg("x"), py::arg("mask"), py::arg("weight"),
        py::arg("save"), py::arg("part"), py::arg("tiles"), py::arg("relu"), py::arg("want_dweight"),
        py::arg("dweight_out") = py::none(), py::arg("dbias_out") = py::none());
}
