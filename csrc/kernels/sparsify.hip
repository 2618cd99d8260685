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

// The same with float4 loads / stores (g, r and resid 16-B aligned: the host checks), 8 float4 per
// thread per 8192-element tile; the <= 3 trailing elements ride along with block 0's first tile.
// (The 4-B form moved a ResNet-50 bucket at ~1.5 TB/s: 32 dword loads per thread per tile.)
constexpr int kV = 8;
constexpr int kTileV = kBlock * kV * 4;

__global__ __launch_bounds__(kBlock) void threshold_compact_v4_kernel(const float* g, const float* r, int mode,
                                                                      float beta, float gamma, int64_t n,
                                                                      float thr, float* __restrict__ out_val,
                                                                      int32_t* __restrict__ out_idx, int64_t cap,
                                                                      int32_t* __restrict__ counter,
                                                                      float* resid) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int bcast;
  const int64_t n4 = n & ~(int64_t)3;
  const int nt = (int)(n - n4);
  bool first = blockIdx.x == 0;
  for (int64_t tb = (int64_t)blockIdx.x * kTileV; first || tb < n4; tb += (int64_t)gridDim.x * kTileV) {
    float4 v[kV];
    uint32_t take = 0;
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      const int64_t i = tb + 4 * ((int64_t)j * kBlock + threadIdx.x);
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < n4) {
        float4 x = *reinterpret_cast<const float4*>(g + i);
        if (mode == 1) {
          const float4 rr = *reinterpret_cast<const float4*>(r + i);
          x = make_float4(fmaf(beta, rr.x, gamma * x.x), fmaf(beta, rr.y, gamma * x.y), fmaf(beta, rr.z, gamma * x.z),
                          fmaf(beta, rr.w, gamma * x.w));
        }
        v[j] = x;
        take |= ((fabsf(x.x) > thr ? 1u : 0u) | (fabsf(x.y) > thr ? 2u : 0u) | (fabsf(x.z) > thr ? 4u : 0u) |
                 (fabsf(x.w) > thr ? 8u : 0u)) << (4 * j);
      }
    }
    float xe = 0.f;
    int64_t ie = -1;
    bool te = false;
    if (first && (int)threadIdx.x < nt) {
      ie = n4 + threadIdx.x;
      xe = g[ie];
      if (mode == 1) xe = fmaf(beta, r[ie], gamma * xe);
      te = fabsf(xe) > thr;
    }
    int tot = 0;
    const int pre = block_exclusive_scan<kBlock>(__popc(take) + (te ? 1 : 0), lds, &tot);
    uint32_t sent = 0;
    bool sente = false;
    if (tot > 0) {
      if (threadIdx.x == 0) bcast = atomicAdd(counter, tot);
      __syncthreads();
      int64_t p = (int64_t)bcast + pre;
#pragma unroll
      for (int j = 0; j < kV; ++j) {
        const uint32_t tj = (take >> (4 * j)) & 15u;
        if (tj) {
          const int64_t i = tb + 4 * ((int64_t)j * kBlock + threadIdx.x);
          const float e[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            if ((tj >> q) & 1u) {
              if (p < cap) {
                out_val[p] = e[q];
                out_idx[p] = (int32_t)(i + q);
                sent |= 1u << (4 * j + q);
              }
              ++p;
            }
          }
        }
      }
      if (te) {
        if (p < cap) {
          out_val[p] = xe;
          out_idx[p] = (int32_t)ie;
          sente = true;
        }
        ++p;
      }
    }
    if (resid != nullptr) {  // spilled (selected past the capacity) entries stay in the residual
#pragma unroll
      for (int j = 0; j < kV; ++j) {
        const int64_t i = tb + 4 * ((int64_t)j * kBlock + threadIdx.x);
        if (i < n4) {
          const uint32_t sj = (sent >> (4 * j)) & 15u;
          *reinterpret_cast<float4*>(resid + i) =
              make_float4((sj & 1u) ? 0.f : v[j].x, (sj & 2u) ? 0.f : v[j].y, (sj & 4u) ? 0.f : v[j].z,
                          (sj & 8u) ? 0.f : v[j].w);
        }
      }
      if (ie >= 0) resid[ie] = sente ? 0.f : xe;
    }
    first = false;
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
  auto a16 = [](const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (a16(g) && (mode != 1 || a16(r)) && a16(resid)) {
    int64_t tiles = (n + kTileV - 1) / kTileV;
    if (tiles > 2048) tiles = 2048;
    threshold_compact_v4_kernel<<<(int)tiles, kBlock, 0, stream>>>(g, r, mode, beta, gamma, n, thr, out_val,
                                                                   out_idx, cap, counter, resid);
    return;
  }
  int64_t tiles = (n + kTile - 1) / kTile;
  if (tiles > 2048) tiles = 2048;
  threshold_compact_kernel<<<(int)tiles, kBlock, 0, stream>>>(g, r, mode, beta, gamma, n, thr, out_val, out_idx,
                                                              cap, counter, resid);
}

}  // namespace grace
