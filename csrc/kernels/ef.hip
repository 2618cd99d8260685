// Elementwise error-feedback helpers (ResidualMemory / EFSignSGDMemory compensate when not
// fused into a compressor kernel).  float4-vectorised grid-stride loops, sized for the chip
// (<= 256 CUs x 8 blocks).
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n_vec) {
  int64_t b = (n_vec + kBlock - 1) / kBlock;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

// out = a*x + b*y
__global__ __launch_bounds__(kBlock) void axpby_kernel(const float* x, const float* y, float* out,
                                                       int64_t n, float a, float b) {
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const bool aligned = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
                         reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  int64_t tail = 0;
  if (aligned) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* y4 = reinterpret_cast<const float4*>(y);
    float4* o4 = reinterpret_cast<float4*>(out);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += stride) {
      const float4 u = x4[i], v = y4[i];
      o4[i] = make_float4(fmaf(a, u.x, b * v.x), fmaf(a, u.y, b * v.y), fmaf(a, u.z, b * v.z),
                          fmaf(a, u.w, b * v.w));
    }
    tail = nv << 2;
  }
  for (int64_t i = tail + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    out[i] = fmaf(a, x[i], b * y[i]);
}

__global__ __launch_bounds__(kBlock) void scale_kernel(float* x, int64_t n, float s) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t nv = n >> 2;
  int64_t tail = 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    float4* x4 = reinterpret_cast<float4*>(x);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += stride) {
      float4 u = x4[i];
      u.x *= s; u.y *= s; u.z *= s; u.w *= s;
      x4[i] = u;
    }
    tail = nv << 2;
  }
  for (int64_t i = tail + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) x[i] *= s;
}

}  // namespace

void axpby(const float* x, const float* y, float* out, int64_t n, float a, float b, hipStream_t stream) {
  if (n <= 0) return;
  axpby_kernel<<<grid_for((n + 3) >> 2), kBlock, 0, stream>>>(x, y, out, n, a, b);
}

void scale_inplace(float* x, int64_t n, float s, hipStream_t stream) {
  if (n <= 0) return;
  scale_kernel<<<grid_for((n + 3) >> 2), kBlock, 0, stream>>>(x, n, s);
}

}  // namespace grace
