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
//   workgroup prefix sum + one atomic per 8192-element tile; fused error feedback (x = beta*r + gamma*g, residual =
//   x with the sent entries zeroed) in the same pass.
#include "grace_common.h"
#include "grace_kernels.h"
#include "grace_rand.h"
#include "grace_scan.h"

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
                                                              const int64_t* __restrict__ step,
                                                              float* __restrict__ vals, float* resid) {
  const int64_t K = out_off[n_seg];
  const uint64_t mix = step ? (uint64_t)(*step) * 0x9E3779B97F4A7C15ull : 0ull;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < K; j += stride) {
    const int s = find_seg(out_off, n_seg, j);
    const uint64_t n = (uint64_t)(seg_off[s + 1] - seg_off[s]);
    const FeistelKey fk = feistel_key((uint64_t)seeds[s] ^ mix, n);
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
                                                               const int64_t* __restrict__ step,
                                                               float* __restrict__ out, float scale,
                                                               int accumulate) {
  const int64_t K = out_off[n_seg];
  const uint64_t mix = step ? (uint64_t)(*step) * 0x9E3779B97F4A7C15ull : 0ull;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < K; j += stride) {
    const int s = find_seg(out_off, n_seg, j);
    const uint64_t n = (uint64_t)(seg_off[s + 1] - seg_off[s]);
    const FeistelKey fk = feistel_key((uint64_t)seeds[s] ^ mix, n);
    const int64_t i = seg_off[s] + (int64_t)feistel_perm((uint64_t)(j - out_off[s]), n, fk);
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) acc += vals[(int64_t)r * rank_stride + j];
    acc *= scale;
    out[i] = accumulate ? out[i] + acc : acc;
  }
}

// mode 0: x = g ; mode 1: x = beta*r + gamma*g (and residual written when resid != nullptr)
// Tiles of 256 x 32 elements; ONE atomic per tile reserves the output (grace_scan.h).
constexpr int kPer = 32;
constexpr int kTile = kBlock * kPer;

__global__ __launch_bounds__(kBlock) void threshold_compact_kernel(const float* g, const float* r, int mode,
                                                                   float beta, float gamma, int64_t n,
                                                                   float thr, float* __restrict__ out_val,
                                                                   int32_t* __restrict__ out_idx, int64_t cap,
                                                                   int32_t* __restrict__ counter,
                                                                   float* resid) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int bcast;
  for (int64_t tb = (int64_t)blockIdx.x * kTile; tb < n; tb += (int64_t)gridDim.x * kTile) {
    float v[kPer];
    uint32_t take = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = tb + (int64_t)j * kBlock + threadIdx.x;
      v[j] = 0.f;
      if (i < n) {
        float x = g[i];
        if (mode == 1) x = fmaf(beta, r[i], gamma * x);
        v[j] = x;
        take |= (fabsf(x) > thr ? 1u : 0u) << j;
      }
    }
    int tot = 0;
    const int pre = block_exclusive_scan<kBlock>(__popc(take), lds, &tot);
    uint32_t sent = 0;  // selected AND inside the payload capacity
    if (tot > 0) {
      if (threadIdx.x == 0) bcast = atomicAdd(counter, tot);
      __syncthreads();
      int64_t p = (int64_t)bcast + pre;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if ((take >> j) & 1u) {
          if (p < cap) {
            out_val[p] = v[j];
            out_idx[p] = (int32_t)(tb + (int64_t)j * kBlock + threadIdx.x);
            sent |= 1u << j;
          }
          ++p;
        }
      }
    }
    if (resid != nullptr) {  // spilled (selected past the capacity) entries stay in the residual
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int64_t i = tb + (int64_t)j * kBlock + threadIdx.x;
        if (i < n) resid[i] = ((sent >> j) & 1u) ? 0.f : v[j];
      }
    }
    __syncthreads();
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
                  const int64_t* seeds, const int64_t* step, int64_t K, float* vals, float* resid,
                  hipStream_t stream) {
  if (K <= 0) return;
  randk_gather_kernel<<<grid_for(K), kBlock, 0, stream>>>(x, n_seg, seg_off, out_off, seeds, step, vals, resid);
}

void randk_scatter(const float* vals, int64_t rank_stride, int n_ranks, int n_seg, const int64_t* seg_off,
                   const int64_t* out_off, const int64_t* seeds, const int64_t* step, int64_t K, float* out,
                   float scale, bool accumulate, hipStream_t stream) {
  if (K <= 0) return;
  randk_scatter_kernel<<<grid_for(K), kBlock, 0, stream>>>(vals, rank_stride, n_ranks, n_seg, seg_off, out_off,
                                                           seeds, step, out, scale, accumulate ? 1 : 0);
}

void threshold_compact(const float* g, const float* r, int mode, float beta, float gamma, int64_t n, float thr,
                       float* out_val, int32_t* out_idx, int64_t cap, int32_t* counter, float* resid,
                       hipStream_t stream, int header_bytes) {
  GRACE_HIP_CHECK(hipMemsetAsync(counter, 0, header_bytes, stream));
  if (n <= 0) return;
  int64_t tiles = (n + kTile - 1) / kTile;
  if (tiles > 2048) tiles = 2048;
  threshold_compact_kernel<<<(int)tiles, kBlock, 0, stream>>>(g, r, mode, beta, gamma, n, thr, out_val, out_idx,
                                                              cap, counter, resid);
}

}  // namespace grace
