// Python bindings for the grace_amd native library (module grace_amd._C).
//
// Every op validates device/dtype/contiguity on the host, then calls the raw-pointer launcher
// on PyTorch's *current* HIP stream so it orders correctly with surrounding torch work and
// can be captured into a HIP graph.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "grace_kernels.h"

namespace {

using at::Tensor;

// On ROCm PyTorch exposes GPUs as device type "cuda"; the *MasqueradingAsCUDA* guard/stream
// are the HIP implementations registered for that device type.
inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " must be " #dt)
#define CHECK_F32(t) \
  CHECK_DEV(t);      \
  CHECK_CONTIG(t);   \
  CHECK_DT(t, at::kFloat)
#define CHECK_I32(t) \
  CHECK_DEV(t);      \
  CHECK_CONTIG(t);   \
  CHECK_DT(t, at::kInt)
#define CHECK_I64(t) \
  CHECK_DEV(t);      \
  CHECK_CONTIG(t);   \
  CHECK_DT(t, at::kLong)

grace::ChunkTable make_ct(const Tensor& seg, const Tensor& cb, const Tensor& ce) {
  CHECK_I32(seg);
  CHECK_I64(cb);
  CHECK_I64(ce);
  TORCH_CHECK(seg.numel() == cb.numel() && cb.numel() == ce.numel(), "chunk table size mismatch");
  grace::ChunkTable ct;
  ct.seg = seg.data_ptr<int32_t>();
  ct.begin = cb.data_ptr<int64_t>();
  ct.end = ce.data_ptr<int64_t>();
  ct.n_chunks = (int32_t)seg.numel();
  return ct;
}

// ------------------------------------------------------------------------------ top-k
void topk_select(const Tensor& g, const c10::optional<Tensor>& r, const Tensor& x, double beta,
                 double gamma, int64_t mode, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                 const Tensor& kseg, const Tensor& state, const Tensor& hist) {
  CHECK_F32(g);
  CHECK_F32(x);
  CHECK_I32(kseg);
  CHECK_I32(state);
  CHECK_I32(hist);
  const int n_seg = (int)kseg.numel();
  TORCH_CHECK(state.numel() >= 2 * n_seg, "state too small");
  TORCH_CHECK(hist.numel() >= (int64_t)n_seg * 2048, "hist too small");
  TORCH_CHECK(x.numel() == g.numel(), "x/g size mismatch");
  const float* rp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(r.has_value(), "mode 1 needs a residual");
    CHECK_F32((*r));
    TORCH_CHECK(r->numel() == g.numel(), "r/g size mismatch");
    rp = r->data_ptr<float>();
  }
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(g.device());
  grace::topk_select_bucket(ct, n_seg, g.data_ptr<float>(), rp, x.data_ptr<float>(), (float)beta,
                            (float)gamma, (int)mode, kseg.data_ptr<int32_t>(),
                            reinterpret_cast<grace::TopkState*>(state.data_ptr<int32_t>()),
                            hist.data_ptr<int32_t>(), cur_stream());
}

void topk_compact(const Tensor& x, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                  const Tensor& state, const Tensor& out_off, const Tensor& counters,
                  const Tensor& out_val, const Tensor& out_idx, const c10::optional<Tensor>& resid,
                  int64_t idx_base) {
  CHECK_F32(x);
  CHECK_I32(state);
  CHECK_I64(out_off);
  CHECK_I32(counters);
  CHECK_F32(out_val);
  CHECK_I32(out_idx);
  const int n_seg = (int)out_off.numel() - 1;
  TORCH_CHECK(n_seg >= 1, "out_off must have n_seg+1 entries");
  TORCH_CHECK(counters.numel() >= 2 * n_seg, "counters too small");
  float* rp = nullptr;
  if (resid.has_value()) {
    CHECK_F32((*resid));
    TORCH_CHECK(resid->numel() == x.numel(), "resid size mismatch");
    rp = resid->data_ptr<float>();
  }
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::topk_compact_bucket(ct, n_seg, x.data_ptr<float>(),
                             reinterpret_cast<const grace::TopkState*>(state.data_ptr<int32_t>()),
                             out_off.data_ptr<int64_t>(), counters.data_ptr<int32_t>(),
                             out_val.data_ptr<float>(), out_idx.data_ptr<int32_t>(), rp, idx_base,
                             cur_stream());
}

void sparse_scatter_add(const Tensor& val, const Tensor& idx, const Tensor& out, double scale,
                        bool accumulate) {
  CHECK_F32(val);
  CHECK_I32(idx);
  CHECK_F32(out);
  TORCH_CHECK(val.numel() == idx.numel(), "val/idx size mismatch");
  DevGuard guard(out.device());
  grace::sparse_scatter_add(val.data_ptr<float>(), idx.data_ptr<int32_t>(), val.numel(),
                            out.data_ptr<float>(), (float)scale, accumulate, cur_stream());
}

// ------------------------------------------------------------------------------ elementwise
void axpby(const Tensor& x, const Tensor& y, const Tensor& out, double a, double b) {
  CHECK_F32(x);
  CHECK_F32(y);
  CHECK_F32(out);
  TORCH_CHECK(x.numel() == y.numel() && y.numel() == out.numel(), "size mismatch");
  DevGuard guard(out.device());
  grace::axpby(x.data_ptr<float>(), y.data_ptr<float>(), out.data_ptr<float>(), x.numel(), (float)a,
               (float)b, cur_stream());
}

void scale_(const Tensor& x, double s) {
  CHECK_F32(x);
  DevGuard guard(x.device());
  grace::scale_inplace(x.data_ptr<float>(), x.numel(), (float)s, cur_stream());
}

std::string build_info() {
  return std::string("grace_amd native: HIP ") + std::to_string(HIP_VERSION_MAJOR) + "." +
         std::to_string(HIP_VERSION_MINOR) + " gfx950";
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "grace_amd native CDNA4 kernels and RCCL runtime";
  m.def("build_info", &build_info);
  m.def("topk_select", &topk_select);
  m.def("topk_compact", &topk_compact);
  m.def("sparse_scatter_add", &sparse_scatter_add);
  m.def("axpby", &axpby);
  m.def("scale_", &scale_);
}
