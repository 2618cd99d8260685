// 16-bit casting and quantile-sketch codecs for CDNA4.
//
// FP16Compressor (reference /root/reference/grace_dl/dist/compressor/fp16.py:6-22): the cast
// itself, plus a W-rank decode-sum that reads every rank's 16-bit payload once and writes the
// fp32 average (Allgather/Broadcast) -- instead of W casts + W-1 adds + a divide.
//
// SketchCompressor (reference tensorflow/compressor/sketch.py:16-39): per segment, q+1 quantile
// edges (computed by one segmented sort on the host side), then ONE pass that bucketises every
// element (binary search over the segment's edges staged in LDS), writes its bin code and
// accumulates per-bin sums and counts in LDS (one global atomic per bin per workgroup); the
// decode-aggregate pass gathers means_r[seg][bin_r[i]] for all W ranks.
#include <hip/hip_fp16.h>

#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxQ = 1024;

inline int grid_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

template <bool BF16>
__global__ __launch_bounds__(kBlock) void cast16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                        int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    if constexpr (BF16) {
      // round-to-nearest-even fp32 -> bf16 (NaN kept quiet)
      const uint32_t u = __float_as_uint(x[i]);
      const uint32_t r = ((u & 0x7fffffffu) > 0x7f800000u) ? (u | 0x00400000u) : (u + 0x7fffu + ((u >> 16) & 1u));
      y[i] = (uint16_t)(r >> 16);
    } else {
      const __half h = __float2half_rn(x[i]);
      y[i] = *reinterpret_cast<const uint16_t*>(&h);
    }
  }
}

template <bool BF16>
__device__ __forceinline__ float from16(uint16_t v) {
  if constexpr (BF16) {
    return __uint_as_float((uint32_t)v << 16);
  } else {
    __half h;
    *reinterpret_cast<uint16_t*>(&h) = v;
    return __half2float(h);
  }
}

template <bool BF16>
__global__ __launch_bounds__(kBlock) void decode16_sum_kernel(const uint8_t* __restrict__ base, int64_t rank_stride,
                                                              int n_ranks, int64_t n, float scale,
                                                              float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r)
      acc += from16<BF16>(reinterpret_cast<const uint16_t*>(base + (int64_t)r * rank_stride)[i]);
    out[i] = acc * scale;
  }
}

// bins: uint8 (q <= 256) or uint16; edges: [n_seg][q+1]; sums/counts: [n_seg][q] (zeroed)
template <typename BinT>
__global__ __launch_bounds__(kBlock) void sketch_encode_kernel(ChunkTable ct, const float* __restrict__ x,
                                                               const float* __restrict__ edges, int q,
                                                               BinT* __restrict__ bins, float* __restrict__ sums,
                                                               float* __restrict__ counts) {
  __shared__ float le[kMaxQ + 1];
  __shared__ float ls[kMaxQ];
  __shared__ float lc[kMaxQ];
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const float* E = edges + (int64_t)sg * (q + 1);
  for (int i = threadIdx.x; i <= q; i += kBlock) le[i] = E[i];
  for (int i = threadIdx.x; i < q; i += kBlock) {
    ls[i] = 0.f;
    lc[i] = 0.f;
  }
  __syncthreads();
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    const float v = x[i];
    // bin = (#edges <= v) - 1 clamped to [0, q-1]
    int lo = 0, hi = q + 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (le[mid] <= v)
        lo = mid + 1;
      else
        hi = mid;
    }
    int bin = lo - 1;
    bin = bin < 0 ? 0 : (bin > q - 1 ? q - 1 : bin);
    bins[i] = (BinT)bin;
    atomicAdd(&ls[bin], v);
    atomicAdd(&lc[bin], 1.f);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < q; i += kBlock) {
    if (lc[i] != 0.f) {
      atomicAdd(&sums[(int64_t)sg * q + i], ls[i]);
      atomicAdd(&counts[(int64_t)sg * q + i], lc[i]);
    }
  }
}

template <typename BinT>
__global__ __launch_bounds__(kBlock) void sketch_decode_kernel(ChunkTable ct, const uint8_t* __restrict__ base,
                                                               int64_t rank_stride, int64_t bins_off,
                                                               int64_t means_off, int q, int n_ranks, float scale,
                                                               float* __restrict__ out) {
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) {
      const uint8_t* rb = base + (int64_t)r * rank_stride;
      const int bin = (int)reinterpret_cast<const BinT*>(rb + bins_off)[i];
      acc += reinterpret_cast<const float*>(rb + means_off)[(int64_t)sg * q + bin];
    }
    out[i] = acc * scale;
  }
}

}  // namespace

void cast16(const float* x, uint16_t* y, int64_t n, bool bf16, hipStream_t stream) {
  if (n <= 0) return;
  if (bf16)
    cast16_kernel<true><<<grid_for(n), kBlock, 0, stream>>>(x, y, n);
  else
    cast16_kernel<false><<<grid_for(n), kBlock, 0, stream>>>(x, y, n);
}

void decode16_sum(const uint8_t* base, int64_t rank_stride, int n_ranks, int64_t n, bool bf16, float scale, float* out,
                  hipStream_t stream) {
  if (n <= 0) return;
  if (bf16)
    decode16_sum_kernel<true><<<grid_for(n), kBlock, 0, stream>>>(base, rank_stride, n_ranks, n, scale, out);
  else
    decode16_sum_kernel<false><<<grid_for(n), kBlock, 0, stream>>>(base, rank_stride, n_ranks, n, scale, out);
}

void sketch_encode(const ChunkTable& ct, const float* x, const float* edges, int q, void* bins, int bin_bytes,
                   float* sums, float* counts, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  if (bin_bytes == 1)
    sketch_encode_kernel<uint8_t><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, edges, q, (uint8_t*)bins, sums, counts);
  else
    sketch_encode_kernel<uint16_t><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, edges, q, (uint16_t*)bins, sums, counts);
}

void sketch_decode(const ChunkTable& ct, const uint8_t* base, int64_t rank_stride, int64_t bins_off, int64_t means_off,
                   int q, int bin_bytes, int n_ranks, float scale, float* out, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  if (bin_bytes == 1)
    sketch_decode_kernel<uint8_t><<<ct.n_chunks, kBlock, 0, stream>>>(ct, base, rank_stride, bins_off, means_off, q,
                                                                      n_ranks, scale, out);
  else
    sketch_decode_kernel<uint16_t><<<ct.n_chunks, kBlock, 0, stream>>>(ct, base, rank_stride, bins_off, means_off, q,
                                                                       n_ranks, scale, out);
}

}  // namespace grace
