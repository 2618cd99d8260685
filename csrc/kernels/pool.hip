// Max pooling over channels_last (NHWC) activations with 1-byte window codes.
//
// Why: PyTorch's max_pool2d_with_indices saves an int64 index per OUTPUT element (for the
// ResNet-50 stem: 26 M outputs -> 205 MB written in forward and read back in backward, 8x the
// pooled tensor itself) and its backward scatters into a zero-filled input gradient.  Here the
// forward writes the position of the max inside its k x k window as one byte (k <= 15), and
// the backward GATHERS: every input element enumerates the (at most ceil(k/s)^2) windows that
// contain it and sums the gradients of those whose code points at it -- no zero fill, no
// atomics, deterministic, every byte of the input gradient written once.
//
// Semantics follow PyTorch (aten/src/ATen/native/cuda/DilatedMaxPool2d.cu): padding is
// implicit -inf, the FIRST maximum in row-major window order wins (strict >), a NaN wins and
// propagates.  Each thread owns 8 consecutive channels of one output (forward) or input
// (backward) pixel: 16-B (bf16) or 2 x 16-B (fp32) vector accesses.
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kPB = 256;

struct V8 {
  float v[8];
};

__device__ __forceinline__ V8 ldv(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  return V8{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}};
}
__device__ __forceinline__ V8 ldv(const uint16_t* p) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  V8 r;
  r.v[0] = __uint_as_float(u.x << 16);
  r.v[1] = __uint_as_float(u.x & 0xffff0000u);
  r.v[2] = __uint_as_float(u.y << 16);
  r.v[3] = __uint_as_float(u.y & 0xffff0000u);
  r.v[4] = __uint_as_float(u.z << 16);
  r.v[5] = __uint_as_float(u.z & 0xffff0000u);
  r.v[6] = __uint_as_float(u.w << 16);
  r.v[7] = __uint_as_float(u.w & 0xffff0000u);
  return r;
}
__device__ __forceinline__ void stv(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void stv(uint16_t* p, const float* v) {
  // values are copies of bf16 inputs (max) or sums of bf16 gradients: round to nearest even
  uint4 u;
  u.x = (uint32_t)f32_to_bf16_rne(v[0]) | ((uint32_t)f32_to_bf16_rne(v[1]) << 16);
  u.y = (uint32_t)f32_to_bf16_rne(v[2]) | ((uint32_t)f32_to_bf16_rne(v[3]) << 16);
  u.z = (uint32_t)f32_to_bf16_rne(v[4]) | ((uint32_t)f32_to_bf16_rne(v[5]) << 16);
  u.w = (uint32_t)f32_to_bf16_rne(v[6]) | ((uint32_t)f32_to_bf16_rne(v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = u;
}

struct PoolGeom {
  int N, H, W, C, OH, OW, k, s, pad;
};

template <typename T>
__global__ __launch_bounds__(kPB) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ code, PoolGeom g, int64_t n_vec) {
  const int cv = g.C >> 3;
  for (int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x; i < n_vec; i += (int64_t)gridDim.x * kPB) {
    const int c8 = (int)(i % cv);
    const int64_t pix = i / cv;
    const int ow = (int)(pix % g.OW);
    const int oh = (int)((pix / g.OW) % g.OH);
    const int n = (int)(pix / ((int64_t)g.OW * g.OH));
    const int h0 = oh * g.s - g.pad, w0 = ow * g.s - g.pad;
    // an all -inf window keeps PyTorch's initial index: its first in-range element
    const uint32_t first = (uint32_t)(max(0, -h0) * g.k + max(0, -w0));
    float m[8];
    uint32_t arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      arg[j] = first;
    }
    for (int kh = 0; kh < g.k; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= g.W) continue;
        const V8 v = ldv(x + ((((int64_t)n * g.H + h) * g.W + w) * g.C + c8 * 8));
        const uint32_t pos = (uint32_t)(kh * g.k + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // as PyTorch: the first maximum wins, every NaN takes over
          const bool take = (v.v[j] > m[j]) || (v.v[j] != v.v[j]);
          m[j] = take ? v.v[j] : m[j];
          arg[j] = take ? pos : arg[j];
        }
      }
    }
    stv(y + i * 8, m);
    uint2 packed;
    packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    *reinterpret_cast<uint2*>(code + i * 8) = packed;
  }
}

// q = m / d, r = m % d for m < 2^24 (a float multiply and one correction)
__device__ __forceinline__ int fdiv(int m, int d, float inv, int* r) {
  int q = (int)((float)m * inv);
  int rr = m - q * d;
  if (rr < 0) {
    --q;
    rr += d;
  } else if (rr >= d) {
    ++q;
    rr -= d;
  }
  *r = rr;
  return q;
}

// SMALL: n_vec < 2^24 -- the index decomposition in 32-bit float-reciprocal divmods instead of
// four 64-bit integer divisions per element (the ResNet-50 stem's backward: 101 us -> see
// profiles/r4_final_headline_graph_kernels.txt)
template <typename T, bool SMALL>
__global__ __launch_bounds__(kPB) void maxpool_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                          const uint8_t* __restrict__ code, T* __restrict__ dx,
                                                          PoolGeom g, int64_t n_vec) {
  // dy2 (may be null): a second gradient of the same pooled output (two consumers: the first
  // bottleneck's main path and shortcut), summed here as autograd's add would -- dy + dy2 per
  // element, then the window accumulation -- without that add kernel's extra pass
  const int cv = g.C >> 3;
  const float inv_cv = 1.f / (float)cv, inv_w = 1.f / (float)g.W, inv_h = 1.f / (float)g.H;
  for (int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x; i < n_vec; i += (int64_t)gridDim.x * kPB) {
    int c8, w, h, n;
    if constexpr (SMALL) {
      const int pix = fdiv((int)i, cv, inv_cv, &c8);
      const int q = fdiv(pix, g.W, inv_w, &w);
      n = fdiv(q, g.H, inv_h, &h);
    } else {
      c8 = (int)(i % cv);
      const int64_t pix = i / cv;
      w = (int)(pix % g.W);
      h = (int)((pix / g.W) % g.H);
      n = (int)(pix / ((int64_t)g.W * g.H));
    }
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // windows oh with oh*s - pad <= h <= oh*s - pad + k - 1
    const int hp = h + g.pad, wp = w + g.pad;
    const int oh_lo = hp - g.k + 1 > 0 ? (hp - g.k + 1 + g.s - 1) / g.s : 0;
    const int oh_hi = min(hp / g.s, g.OH - 1);
    const int ow_lo = wp - g.k + 1 > 0 ? (wp - g.k + 1 + g.s - 1) / g.s : 0;
    const int ow_hi = min(wp / g.s, g.OW - 1);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const uint32_t pos = (uint32_t)((hp - oh * g.s) * g.k + (wp - ow * g.s));
        const int64_t o = ((((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + c8 * 8);
        const uint2 pk = *reinterpret_cast<const uint2*>(code + o);
        const uint32_t cw[2] = {pk.x, pk.y};
        bool any = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) any |= ((cw[j >> 2] >> (8 * (j & 3))) & 0xffu) == pos;
        if (!any) continue;
        V8 d = ldv(dy + o);
        if (dy2 != nullptr) {
          const V8 d2 = ldv(dy2 + o);
#pragma unroll
          for (int j = 0; j < 8; ++j) d.v[j] = d.v[j] + d2.v[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((cw[j >> 2] >> (8 * (j & 3))) & 0xffu) == pos) acc[j] += d.v[j];
      }
    }
    stv(dx + i * 8, acc);
  }
}

// global average pool backward: dx[n, h, w, c] = dy[n, c] * inv_hw (channels_last x)
template <typename T>
__global__ __launch_bounds__(kPB) void gap_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int HW, int C,
                                                      float inv_hw, int64_t n_vec) {
  const int cv = C >> 3;
  for (int64_t i = (int64_t)blockIdx.x * kPB + threadIdx.x; i < n_vec; i += (int64_t)gridDim.x * kPB) {
    const int c8 = (int)(i % cv);
    const int64_t n = i / ((int64_t)cv * HW);
    const V8 d = ldv(dy + n * C + c8 * 8);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = d.v[j] * inv_hw;
    stv(dx + i * 8, o);
  }
}

int pool_grid(int64_t n_vec) {
  int64_t b = (n_vec + kPB - 1) / kPB;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

void maxpool_forward(const void* x, bool fp32, int N, int H, int W, int C, int OH, int OW, int k, int s, int pad,
                     void* y, uint8_t* code, hipStream_t stream) {
  const PoolGeom g{N, H, W, C, OH, OW, k, s, pad};
  const int64_t n_vec = (int64_t)N * OH * OW * (C / 8);
  if (n_vec == 0) return;
  if (fp32)
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(pool_grid(n_vec)), dim3(kPB), 0, stream,
                       static_cast<const float*>(x), static_cast<float*>(y), code, g, n_vec);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<uint16_t>, dim3(pool_grid(n_vec)), dim3(kPB), 0, stream,
                       static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), code, g, n_vec);
}

void global_avgpool_backward(const void* dy, bool fp32, int N, int HW, int C, void* dx, hipStream_t stream) {
  const int64_t n_vec = (int64_t)N * HW * (C / 8);
  if (n_vec == 0) return;
  const float inv = 1.f / (float)HW;
  if (fp32)
    hipLaunchKernelGGL(gap_bwd_kernel<float>, dim3(pool_grid(n_vec)), dim3(kPB), 0, stream,
                       static_cast<const float*>(dy), static_cast<float*>(dx), HW, C, inv, n_vec);
  else
    hipLaunchKernelGGL(gap_bwd_kernel<uint16_t>, dim3(pool_grid(n_vec)), dim3(kPB), 0, stream,
                       static_cast<const uint16_t*>(dy), static_cast<uint16_t*>(dx), HW, C, inv, n_vec);
}

void maxpool_backward(const void* dy, const uint8_t* code, bool fp32, int N, int H, int W, int C, int OH, int OW,
                      int k, int s, int pad, void* dx, hipStream_t stream, const void* dy2) {
  const PoolGeom g{N, H, W, C, OH, OW, k, s, pad};
  const int64_t n_vec = (int64_t)N * H * W * (C / 8);
  if (n_vec == 0) return;
  const bool small = n_vec < (int64_t(1) << 24);
#define GRACE_POOL_BWD(T, S)                                                                             \
  hipLaunchKernelGGL((maxpool_bwd_kernel<T, S>), dim3(pool_grid(n_vec)), dim3(kPB), 0, stream,          \
                     static_cast<const T*>(dy), static_cast<const T*>(dy2), code, static_cast<T*>(dx), g, n_vec)
  if (fp32 && small) GRACE_POOL_BWD(float, true);
  else if (fp32) GRACE_POOL_BWD(float, false);
  else if (small) GRACE_POOL_BWD(uint16_t, true);
  else GRACE_POOL_BWD(uint16_t, false);
#undef GRACE_POOL_BWD
}

}  // namespace grace
