// Random-K and Threshold sparsifiers for CDNA4 (gfx950).
//
// Random-K  (reference /root/reference/grace_dl/dist/compressor/randomk.py:6-40):
//   indices are NOT sent; every rank regenerates them from (seed, segment) with the Feistel
//   permutation in grace_rand.h, so only the K fp32 values move.  One thread per selected
//   element (binary search of its segment in the output offsets).
//     randk_gather   : vals[j] = x[idx_j]  (+ optional residual zeroing r[idx_j] = 0)
//     randk_scatter  : out[idx_j] (+)= scale * sum_{r<W} vals_r[j]   (rank-ordered sum -> every
//                      rank gets bit-identical results; serves Allgather AND Allreduce)
//
// Threshold (reference threshold.py:6-27): |x| > thr  -> (value, flat index), compacted with one
//   64-lane ballot + one atomic per wave; fused error feedback (x = beta*r + gamma*g, residual =
//   x with the sent entries zeroed) in the same pass.
#include "grace_common.h"
#include "grace_kernels.h"
#include "grace_rand.h"

namespace grace {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ int find_seg(const int64_t* __restrict__ out_off, int n_seg, int64_t j) {
  int lo = 0, hi = n_seg;  // out_off[lo] <= j < out_off[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (out_off[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kBlock) void randk_gather_kernel(const float* x, int n_seg,
                                                              const int64_t* __restrict__ seg_off,
                                                              const int64_t* __restrict__ out_off,
                                                              const int64_t* __restrict__ seeds,
                                                              float* __restrict__ vals, float* resid) {
  const int64_t K = out_off[n_seg];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < K; j += stride) {
    const int s = find_seg(out_off, n_seg, j);
    const uint64_t n = (uint64_t)(seg_off[s + 1] - seg_off[s]);
    const FeistelKey fk = feistel_key((uint64_t)seeds[s], n);
    const int64_t i = seg_off[s] + (int64_t)feistel_perm((uint64_t)(j - out_off[s]), n, fk);
    vals[j] = x[i];
    if (resid) resid[i] = 0.f;
  }
}

__global__ __launch_bounds__(kBlock) void randk_scatter_kernel(const float* __restrict__ vals, int64_t rank_stride,
                                                               int n_ranks, int n_seg,
                                                               const int64_t* __restrict__ seg_off,
                                                               const int64_t* __restrict__ out_off,
                                                               const int64_t* __restrict__ seeds,
                                                               float* __restrict__ out, float scale,
                                                               int accumulate) {
  const int64_t K = out_off[n_seg];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < K; j += stride) {
    const int s = find_seg(out_off, n_seg, j);
    const uint64_t n = (uint64_t)(seg_off[s + 1] - seg_off[s]);
    const FeistelKey fk = feistel_key((uint64_t)seeds[s], n);
    const int64_t i = seg_off[s] + (int64_t)feistel_perm((uint64_t)(j - out_off[s]), n, fk);
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) acc += vals[(int64_t)r * rank_stride + j];
    acc *= scale;
    out[i] = accumulate ? out[i] + acc : acc;
  }
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int l = lane_id();
  return (l == 0) ? 0ull : (~0ull >> (64 - l));
}

// mode 0: x = g ; mode 1: x = beta*r + gamma*g (and residual written when resid != nullptr)
__global__ __launch_bounds__(kBlock) void threshold_compact_kernel(const float* g, const float* r, int mode,
                                                                   float beta, float gamma, int64_t n,
                                                                   float thr, float* __restrict__ out_val,
                                                                   int32_t* __restrict__ out_idx,
                                                                   int32_t* __restrict__ counter,
                                                                   float* resid) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t steps = (n + stride - 1) / stride;
  for (int64_t s = 0; s < steps; ++s) {
    const int64_t i = s * stride + (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool valid = i < n;
    float v = 0.f;
    if (valid) {
      v = g[i];
      if (mode == 1) v = fmaf(beta, r[i], gamma * v);
    }
    const bool take = valid && fabsf(v) > thr;
    const unsigned long long m = __ballot(take);
    if (m) {
      int32_t base = 0;
      const int leader = __ffsll((long long)m) - 1;
      if (lane_id() == leader) base = atomicAdd(counter, __popcll(m));
      base = __shfl(base, leader, kWave);
      if (take) {
        const int32_t p = base + __popcll(m & lanemask_lt());
        out_val[p] = v;
        out_idx[p] = (int32_t)i;
      }
    }
    if (resid != nullptr && valid) resid[i] = take ? 0.f : v;
  }
}

inline int grid_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

void randk_gather(const float* x, int n_seg, const int64_t* seg_off, const int64_t* out_off,
                  const int64_t* seeds, int64_t K, float* vals, float* resid, hipStream_t stream) {
  if (K <= 0) return;
  randk_gather_kernel<<<grid_for(K), kBlock, 0, stream>>>(x, n_seg, seg_off, out_off, seeds, vals, resid);
}

void randk_scatter(const float* vals, int64_t rank_stride, int n_ranks, int n_seg, const int64_t* seg_off,
                   const int64_t* out_off, const int64_t* seeds, int64_t K, float* out, float scale,
                   bool accumulate, hipStream_t stream) {
  if (K <= 0) return;
  randk_scatter_kernel<<<grid_for(K), kBlock, 0, stream>>>(vals, rank_stride, n_ranks, n_seg, seg_off, out_off,
                                                           seeds, out, scale, accumulate ? 1 : 0);
}

void threshold_compact(const float* g, const float* r, int mode, float beta, float gamma, int64_t n, float thr,
                       float* out_val, int32_t* out_idx, int32_t* counter, float* resid, hipStream_t stream) {
  GRACE_HIP_CHECK(hipMemsetAsync(counter, 0, sizeof(int32_t), stream));
  if (n <= 0) return;
  threshold_compact_kernel<<<grid_for(n), kBlock, 0, stream>>>(g, r, mode, beta, gamma, n, thr, out_val, out_idx,
                                                               counter, resid);
}

}  // namespace grace
