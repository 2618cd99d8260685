// Dispatcher registration of the GRACE codec primitives: the ``grace`` operator namespace.
//
// The bucketed engine drives the native kernels through pybind (bindings.cpp: segmented, table-
// driven launches on the current stream).  This file exposes the per-tensor GRACE contract --
// compress(tensor) -> payload, decompress(payloads of W ranks) -> tensor, the semantics of
// /root/reference/grace_dl/dist/compressor/{topk,randomk,signsgd,qsgd,natural}.py -- as
// dispatcher operators, so they are visible to torch.ops / torch.library, trace through fake
// tensors (the Meta kernels below give every output's shape and dtype without touching data) and
// appear as opaque nodes under torch.compile:
//
//     vals, idx, resid = torch.ops.grace.topk_compress(g, resid, 0.01, 1.0, 1.0)
//     g_hat = torch.ops.grace.sparse_decompress(all_vals, all_idx, g.shape, 1.0 / W)
//
// The schemas and the Meta kernels live here; the device kernels are registered for the CUDA
// (HIP) and CPU keys by grace_amd/ops/library.py, which routes each op to the same native
// launchers the engine uses on a GPU tensor and to the PyTorch reference path on CPU.
#include <torch/library.h>
#include <ATen/ATen.h>

#include <algorithm>
#include <cstdint>
#include <tuple>
#include <vector>

namespace {

using at::Tensor;

int64_t numel_of(c10::IntArrayRef shape) {
  int64_t n = 1;
  for (auto d : shape) n *= d;
  return n;
}

// k = max(1, int(n * ratio)), at most n (reference topk.py:7, randomk.py:9)
int64_t k_of(int64_t n, double ratio) {
  if (n <= 0) return 0;
  int64_t k = (int64_t)((double)n * ratio);
  return std::min<int64_t>(n, std::max<int64_t>(1, k));
}

std::tuple<Tensor, Tensor, Tensor> topk_compress_meta(const Tensor& grad, const c10::optional<Tensor>& residual,
                                                      double ratio, double beta, double gamma) {
  TORCH_CHECK(grad.scalar_type() == at::kFloat, "grace::topk_compress: fp32 gradients");
  const int64_t k = k_of(grad.numel(), ratio);
  auto o = grad.options();
  return {at::empty({k}, o), at::empty({k}, o.dtype(at::kInt)), at::empty_like(grad)};
}

Tensor sparse_decompress_meta(const Tensor& values, const Tensor& indices, c10::IntArrayRef shape, double scale) {
  TORCH_CHECK(values.numel() == indices.numel(), "grace::sparse_decompress: values / indices size mismatch");
  return at::empty(shape, values.options());
}

Tensor randomk_compress_meta(const Tensor& grad, double ratio, int64_t seed) {
  return at::empty({k_of(grad.numel(), ratio)}, grad.options());
}

Tensor randomk_decompress_meta(const Tensor& values, c10::IntArrayRef shape, double ratio, int64_t seed, double scale) {
  const int64_t k = k_of(numel_of(shape), ratio);
  TORCH_CHECK(values.numel() % std::max<int64_t>(k, 1) == 0, "grace::randomk_decompress: values must be W x k");
  return at::empty(shape, values.options());
}

Tensor sign_compress_meta(const Tensor& grad) {
  return at::empty({(grad.numel() + 63) / 64}, grad.options().dtype(at::kLong));
}

Tensor sign_decompress_meta(const Tensor& words, c10::IntArrayRef shape) {
  const int64_t nw = (numel_of(shape) + 63) / 64;
  TORCH_CHECK(words.numel() % std::max<int64_t>(nw, 1) == 0, "grace::sign_decompress: words must be W x ceil(n/64)");
  return at::empty(shape, words.options().dtype(at::kFloat));
}

std::tuple<Tensor, Tensor> qsgd_compress_meta(const Tensor& grad, int64_t levels, int64_t seed) {
  TORCH_CHECK(levels >= 1 && levels <= 32767, "grace::qsgd_compress: 1 <= levels <= 32767");
  auto o = grad.options();
  return {at::empty({grad.numel()}, o.dtype(levels < 128 ? at::kChar : at::kShort)), at::empty({1}, o)};
}

Tensor qsgd_decompress_meta(const Tensor& codes, const Tensor& norms, int64_t levels, c10::IntArrayRef shape) {
  TORCH_CHECK(codes.numel() == norms.numel() * numel_of(shape), "grace::qsgd_decompress: codes must be W x n, norms W");
  return at::empty(shape, norms.options());
}

Tensor natural_compress_meta(const Tensor& grad, int64_t seed) {
  return at::empty({grad.numel()}, grad.options().dtype(at::kByte));
}

Tensor natural_decompress_meta(const Tensor& codes, c10::IntArrayRef shape) {
  TORCH_CHECK(codes.numel() % std::max<int64_t>(numel_of(shape), 1) == 0, "grace::natural_decompress: codes must be W x n");
  return at::empty(shape, codes.options().dtype(at::kFloat));
}

}  // namespace

TORCH_LIBRARY(grace, m) {
  // Top-K with fused error feedback: x = beta * residual + gamma * grad (x = grad without a
  // residual); the k = max(1, int(n * ratio)) largest |x| leave as (fp32 values, int32 flat
  // indices); residual_out = x with them zeroed (ResidualMemory.update)
  m.def("topk_compress(Tensor grad, Tensor? residual, float ratio, float beta=1.0, float gamma=1.0)"
        " -> (Tensor values, Tensor indices, Tensor residual_out)");
  // sum over every (value, index) pair -- all W ranks' payloads concatenated -- times scale
  m.def("sparse_decompress(Tensor values, Tensor indices, int[] shape, float scale=1.0) -> Tensor");
  // Random-K: the same k indices on every rank from (seed, n) -- keyed Feistel permutation
  m.def("randomk_compress(Tensor grad, float ratio, int seed) -> Tensor");
  m.def("randomk_decompress(Tensor values, int[] shape, float ratio, int seed, float scale=1.0) -> Tensor");
  // SignSGD: one bit per element (x >= 0), 64 per int64 word; decompress = majority vote of W rows
  m.def("sign_compress(Tensor grad) -> Tensor");
  m.def("sign_decompress(Tensor words, int[] shape) -> Tensor");
  // QSGD: stochastic rounding to ``levels`` levels of |x| / ||x||_2 (int8 codes below 128 levels,
  // int16 above); decompress = sum_r norm_r / levels * codes_r
  m.def("qsgd_compress(Tensor grad, int levels, int seed) -> (Tensor codes, Tensor norm)");
  m.def("qsgd_decompress(Tensor codes, Tensor norms, int levels, int[] shape) -> Tensor");
  // Natural compression: stochastic power-of-two rounding, one byte per element
  m.def("natural_compress(Tensor grad, int seed) -> Tensor");
  m.def("natural_decompress(Tensor codes, int[] shape) -> Tensor");
}

TORCH_LIBRARY_IMPL(grace, Meta, m) {
  m.impl("topk_compress", &topk_compress_meta);
  m.impl("sparse_decompress", &sparse_decompress_meta);
  m.impl("randomk_compress", &randomk_compress_meta);
  m.impl("randomk_decompress", &randomk_decompress_meta);
  m.impl("sign_compress", &sign_compress_meta);
  m.impl("sign_decompress", &sign_decompress_meta);
  m.impl("qsgd_compress", &qsgd_compress_meta);
  m.impl("qsgd_decompress", &qsgd_decompress_meta);
  m.impl("natural_compress", &natural_compress_meta);
  m.impl("natural_decompress", &natural_decompress_meta);
}
