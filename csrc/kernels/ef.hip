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

// Bucket gather: copy the memory image of up to kGatherSegs parameter gradients into their
// segments of the flat fp32 bucket in ONE launch (pointer table passed by value in the kernel
// arguments, so a captured HIP graph replays it with no host work).  Replaces a bucket memset +
// one AccumulateGrad add kernel per parameter (~4.5 us of device time each for the many small
// tensors of a CNN/transformer).  BF16 sources (gradients of bf16 working weights) are widened
// on the fly.  blockIdx.y = segment, blockIdx.x strides its elements.
struct GatherTable {
  const void* src[kGatherSegs];
  int64_t dst_off[kGatherSegs];  // segment start in the destination
  int64_t len[kGatherSegs];
};

template <bool BF16>
__global__ __launch_bounds__(kBlock) void gather_segments_kernel(GatherTable t, float* __restrict__ dst) {
  const int s = blockIdx.y;
  const int64_t n = t.len[s];
  float* __restrict__ d = dst + t.dst_off[s];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t tail = 0;
  if constexpr (BF16) {
    const uint16_t* __restrict__ src = static_cast<const uint16_t*>(t.src[s]);
    if (((reinterpret_cast<uintptr_t>(src) & 7) | (reinterpret_cast<uintptr_t>(d) & 15)) == 0) {
      const int64_t nv = n >> 2;
      const ushort4* s4 = reinterpret_cast<const ushort4*>(src);
      float4* d4 = reinterpret_cast<float4*>(d);
      for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += stride) {
        const ushort4 h = s4[i];
        d4[i] = make_float4(bf16_to_f32(h.x), bf16_to_f32(h.y), bf16_to_f32(h.z), bf16_to_f32(h.w));
      }
      tail = nv << 2;
    }
    for (int64_t i = tail + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) d[i] = bf16_to_f32(src[i]);
  } else {
    const float* __restrict__ src = static_cast<const float*>(t.src[s]);
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
      const int64_t nv = n >> 2;
      const float4* s4 = reinterpret_cast<const float4*>(src);
      float4* d4 = reinterpret_cast<float4*>(d);
      for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += stride) d4[i] = s4[i];
      tail = nv << 2;
    }
    for (int64_t i = tail + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) d[i] = src[i];
  }
}

// Working-weight refresh: bf16 copies of up to kGatherSegs fp32 master tensors in one launch
// (instead of one cast kernel per weight per forward under autocast).
struct CastTable {
  const float* src[kGatherSegs];
  uint16_t* dst[kGatherSegs];
  int64_t len[kGatherSegs];
};

__global__ __launch_bounds__(kBlock) void cast_segments_kernel(CastTable t) {
  const int s = blockIdx.y;
  const int64_t n = t.len[s];
  const float* __restrict__ src = t.src[s];
  uint16_t* __restrict__ d = t.dst[s];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t tail = 0;
  if (((reinterpret_cast<uintptr_t>(src) & 15) | (reinterpret_cast<uintptr_t>(d) & 7)) == 0) {
    const int64_t nv = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    ushort4* d4 = reinterpret_cast<ushort4*>(d);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += stride) {
      const float4 v = s4[i];
      d4[i] = make_ushort4(f32_to_bf16_rne(v.x), f32_to_bf16_rne(v.y), f32_to_bf16_rne(v.z), f32_to_bf16_rne(v.w));
    }
    tail = nv << 2;
  }
  for (int64_t i = tail + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) d[i] = f32_to_bf16_rne(src[i]);
}

inline unsigned seg_grid(int64_t maxn) {
  int64_t gx = (maxn / 4 + kBlock - 1) / kBlock;
  if (gx > 512) gx = 512;
  if (gx < 1) gx = 1;
  return (unsigned)gx;
}

}  // namespace

void gather_segments(const void* const* src, bool bf16, const int64_t* dst_off, const int64_t* len, int n_seg,
                     float* dst, hipStream_t stream) {
  for (int g0 = 0; g0 < n_seg; g0 += kGatherSegs) {
    const int ng = n_seg - g0 < kGatherSegs ? n_seg - g0 : kGatherSegs;
    GatherTable t;
    int64_t maxn = 0;
    for (int i = 0; i < ng; ++i) {
      t.src[i] = src[g0 + i];
      t.dst_off[i] = dst_off[g0 + i];
      t.len[i] = len[g0 + i];
      if (len[g0 + i] > maxn) maxn = len[g0 + i];
    }
    if (maxn == 0) continue;
    if (bf16)
      gather_segments_kernel<true><<<dim3(seg_grid(maxn), (unsigned)ng), kBlock, 0, stream>>>(t, dst);
    else
      gather_segments_kernel<false><<<dim3(seg_grid(maxn), (unsigned)ng), kBlock, 0, stream>>>(t, dst);
  }
}


void cast_segments_bf16(const float* const* src, uint16_t* const* dst, const int64_t* len, int n_seg,
                        hipStream_t stream) {
  for (int g0 = 0; g0 < n_seg; g0 += kGatherSegs) {
    const int ng = n_seg - g0 < kGatherSegs ? n_seg - g0 : kGatherSegs;
    CastTable t;
    int64_t maxn = 0;
    for (int i = 0; i < ng; ++i) {
      t.src[i] = src[g0 + i];
      t.dst[i] = dst[g0 + i];
      t.len[i] = len[g0 + i];
      if (len[g0 + i] > maxn) maxn = len[g0 + i];
    }
    if (maxn == 0) continue;
    cast_segments_kernel<<<dim3(seg_grid(maxn), (unsigned)ng), kBlock, 0, stream>>>(t);
  }
}

void axpby(const float* x, const float* y, float* out, int64_t n, float a, float b, hipStream_t stream) {
  if (n <= 0) return;
  axpby_kernel<<<grid_for((n + 3) >> 2), kBlock, 0, stream>>>(x, y, out, n, a, b);
}

void scale_inplace(float* x, int64_t n, float s, hipStream_t stream) {
  if (n <= 0) return;
  scale_kernel<<<grid_for((n + 3) >> 2), kBlock, 0, stream>>>(x, n, s);
}

}  // namespace grace
