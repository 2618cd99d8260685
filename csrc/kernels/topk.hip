// Segmented exact Top-K of |x| with fused error-feedback, for CDNA4 (gfx950).
//
// Reference semantics (per parameter tensor of n elements):
//   k = max(1, int(n * ratio)); idx = topk(|x|, k); payload = (x[idx], idx)
//   -- /root/reference/grace_dl/dist/compressor/topk.py:6-30
// and ResidualMemory (residual.py:10-20): x = beta*r + gamma*g ; r' = x - decompress(payload).
//
// MI355X design: ONE set of launches for a whole bucket of many parameters ("segments")
// instead of ~7 launches per parameter:
//   pass 0  topk_hist<0>   : x = beta*r + gamma*g (stored), LDS histogram of key bits 30..20
//   select  topk_select    : one workgroup / segment walks its histogram from the top and
//                            fixes 11 bits of the k-th largest key; zeroes the histogram
//   pass 1  topk_hist<1>   : histogram bits 19..9 of keys that match the prefix
//   pass 2  topk_hist<2>   : histogram bits 8..0
//   compact topk_compact   : emits exactly k (value, flat index) pairs per segment with one
//                            atomic per 8K-element tile, resolves ties deterministically in
//                            count, and zeroes the emitted entries of the residual (which
//                            already holds x) in the same pass.
// The radix select is exact (no sampling), so the selected set equals torch.topk's up to
// the choice among equal |x| at the threshold.
#include "grace_common.h"
#include "grace_kernels.h"
#include "grace_scan.h"

namespace grace {

namespace {

constexpr int kBlock = 256;
constexpr int kBins0 = 2048;  // digit 0: bits 30..20
constexpr int kBins1 = 2048;  // digit 1: bits 19..9
constexpr int kBins2 = 512;   // digit 2: bits 8..0
constexpr int kHistStride = 2048;

template <int D>
struct Digit;
template <>
struct Digit<0> {
  static constexpr int shift = 20, bits = 11;
};
template <>
struct Digit<1> {
  static constexpr int shift = 9, bits = 11;
};
template <>
struct Digit<2> {
  static constexpr int shift = 0, bits = 9;
};

// mode: 0 -> x = g (no residual yet); 1 -> x = beta*r + gamma*g
template <int D>
__global__ __launch_bounds__(kBlock) void topk_hist_kernel(ChunkTable ct, const float* g,
                                                           const float* r, float* x, float beta,
                                                           float gamma, int mode,
                                                           const TopkState* __restrict__ st,
                                                           int32_t* __restrict__ hist) {
  constexpr int shift = Digit<D>::shift;
  constexpr int bits = Digit<D>::bits;
  constexpr int nbins = 1 << bits;
  __shared__ int32_t lh[nbins];
  for (int i = threadIdx.x; i < nbins; i += kBlock) lh[i] = 0;
  __syncthreads();
  const int c = blockIdx.x;
  const int seg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  uint32_t want = 0;
  if constexpr (D > 0) want = st[seg].prefix >> (shift + bits);
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    float v;
    if constexpr (D == 0) {
      v = g[i];
      if (mode == 1) v = fmaf(beta, r[i], gamma * v);
      if (x != g) x[i] = v;
    } else {
      v = x[i];
    }
    const uint32_t key = abs_key(v);
    if (D == 0 || (key >> (shift + bits)) == want) atomicAdd(&lh[(key >> shift) & (nbins - 1)], 1);
  }
  __syncthreads();
  int32_t* gh = hist + (int64_t)seg * kHistStride;
  for (int i = threadIdx.x; i < nbins; i += kBlock) {
    const int32_t cnt = lh[i];
    if (cnt) atomicAdd(&gh[i], cnt);
  }
}

// One workgroup per segment. Finds the digit value of the k-th largest key among the keys
// matching the current prefix.  Bins are scanned in DESCENDING order.
template <int D>
__global__ __launch_bounds__(kBlock) void topk_select_kernel(int n_seg, const int32_t* __restrict__ kseg,
                                                             TopkState* __restrict__ st,
                                                             int32_t* __restrict__ hist) {
  constexpr int shift = Digit<D>::shift;
  constexpr int bits = Digit<D>::bits;
  constexpr int nbins = 1 << bits;
  constexpr int per = nbins / kBlock;  // bins per thread (8 or 2)
  __shared__ int32_t part[kBlock];
  const int seg = blockIdx.x;
  if (seg >= n_seg) return;
  int32_t* gh = hist + (int64_t)seg * kHistStride;
  const int32_t krem = (D == 0) ? kseg[seg] : st[seg].krem;
  // thread t owns descending positions j in [t*per, t*per+per): bin = nbins-1-j
  int32_t loc[per];
  int32_t s = 0;
#pragma unroll
  for (int q = 0; q < per; ++q) {
    const int bin = nbins - 1 - (threadIdx.x * per + q);
    loc[q] = gh[bin];
    gh[bin] = 0;  // leave the histogram clean for the next digit / next call
    s += loc[q];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  // inclusive scan (Hillis-Steele) over 256 partial sums
  for (int off = 1; off < kBlock; off <<= 1) {
    const int32_t add = (threadIdx.x >= off) ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += add;
    __syncthreads();
  }
  const int32_t incl = part[threadIdx.x];
  const int32_t excl = incl - s;
  if (excl < krem && krem <= incl) {
    int32_t run = excl;
#pragma unroll
    for (int q = 0; q < per; ++q) {
      if (run + loc[q] >= krem) {
        const uint32_t bin = nbins - 1 - (threadIdx.x * per + q);
        const uint32_t pfx = (D == 0 ? 0u : st[seg].prefix) | (bin << shift);
        st[seg].prefix = pfx;
        st[seg].krem = krem - run;  // how many to take from this bin (and below digits)
        break;
      }
      run += loc[q];
    }
  }
}

// Compaction + residual.  One chunk per workgroup, processed in tiles of 256 x 32 elements.
//   take = key > T  or  (key == T and rank-among-ties < ties)
// Each thread keeps its 32 values in registers; output slots are reserved with ONE atomic per
// tile (workgroup prefix sums, grace_scan.h) instead of one per wave -- the per-segment counter
// is shared by every workgroup of the segment, so per-wave atomics serialised at the memory
// side (measured 0.5 ms per 25M-element bucket before this change).
constexpr int kPer = 32;
constexpr int kTile = kBlock * kPer;

// INPLACE (resid == x, the fused error-feedback path: x already holds the compensated values in
// the residual buffer): only the k emitted entries are zeroed -- no full rewrite of the bucket.
template <bool INPLACE>
__global__ __launch_bounds__(kBlock) void topk_compact_kernel(
    ChunkTable ct, const float* x, const TopkState* __restrict__ st,
    const int64_t* __restrict__ out_off, int32_t* __restrict__ counters /* [2*n_seg] */, int n_seg,
    float* __restrict__ out_val, int32_t* __restrict__ out_idx, float* resid,
    int64_t idx_base) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int bcast[2];
  const int c = blockIdx.x;
  const int seg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const uint32_t T = st[seg].prefix;
  const int32_t ties = st[seg].krem;
  const int64_t base_off = out_off[seg];
  int32_t* out_ctr = counters + seg;
  int32_t* tie_ctr = counters + n_seg + seg;
  for (int64_t tb = b; tb < e; tb += kTile) {
    float v[kPer];
    uint32_t take = 0, tie = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = tb + (int64_t)j * kBlock + threadIdx.x;
      v[j] = 0.f;
      if (i < e) {
        v[j] = x[i];
        const uint32_t key = abs_key(v[j]);
        take |= (key > T ? 1u : 0u) << j;
        tie |= (key == T ? 1u : 0u) << j;
      }
    }
    // ties: rank every tie of the tile, keep the first `ties` over the whole segment
    int tot_tie = 0;
    const int ntie = __popc(tie);
    const int tie_pre = block_exclusive_scan<kBlock>(ntie, lds, &tot_tie);
    if (tot_tie > 0) {
      if (threadIdx.x == 0) bcast[0] = atomicAdd(tie_ctr, tot_tie);
      __syncthreads();
      int r = bcast[0] + tie_pre;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {  // static indices keep v[] in registers
        if ((tie >> j) & 1u) {
          if (r < ties) take |= 1u << j;
          ++r;
        }
      }
    }
    int tot_take = 0;
    const int ntake = __popc(take);
    const int pre = block_exclusive_scan<kBlock>(ntake, lds, &tot_take);
    if (tot_take > 0) {
      if (threadIdx.x == 0) bcast[1] = atomicAdd(out_ctr, tot_take);
      __syncthreads();
      int64_t p = base_off + bcast[1] + pre;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if ((take >> j) & 1u) {
          out_val[p] = v[j];
          out_idx[p] = (int32_t)(tb + (int64_t)j * kBlock + threadIdx.x + idx_base);
          ++p;
        }
      }
    }
    if (INPLACE) {
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if ((take >> j) & 1u) resid[tb + (int64_t)j * kBlock + threadIdx.x] = 0.f;
    } else if (resid != nullptr) {
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int64_t i = tb + (int64_t)j * kBlock + threadIdx.x;
        if (i < e) resid[i] = ((take >> j) & 1u) ? 0.f : v[j];
      }
    }
    __syncthreads();  // lds / bcast reuse by the next tile
  }
}

// out[idx[j]] += val[j] * scale for j < K (indices unique within one payload -> no atomics)
__global__ __launch_bounds__(kBlock) void sparse_scatter_add_kernel(const float* __restrict__ val,
                                                                    const int32_t* __restrict__ idx,
                                                                    int64_t K, float* __restrict__ out,
                                                                    float scale, int accumulate) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < K; j += stride) {
    const int32_t t = idx[j];
    const float add = val[j] * scale;
    out[t] = accumulate ? out[t] + add : add;
  }
}

}  // namespace

void topk_select_bucket(const ChunkTable& ct, int n_seg, const float* g, const float* r, float* x,
                        float beta, float gamma, int mode, const int32_t* kseg, TopkState* st,
                        int32_t* hist, hipStream_t stream) {
  const dim3 grid(ct.n_chunks), block(kBlock);
  topk_hist_kernel<0><<<grid, block, 0, stream>>>(ct, g, r, x, beta, gamma, mode, st, hist);
  topk_select_kernel<0><<<n_seg, kBlock, 0, stream>>>(n_seg, kseg, st, hist);
  topk_hist_kernel<1><<<grid, block, 0, stream>>>(ct, x, nullptr, x, 1.f, 1.f, 0, st, hist);
  topk_select_kernel<1><<<n_seg, kBlock, 0, stream>>>(n_seg, kseg, st, hist);
  topk_hist_kernel<2><<<grid, block, 0, stream>>>(ct, x, nullptr, x, 1.f, 1.f, 0, st, hist);
  topk_select_kernel<2><<<n_seg, kBlock, 0, stream>>>(n_seg, kseg, st, hist);
}

void topk_compact_bucket(const ChunkTable& ct, int n_seg, const float* x, const TopkState* st,
                         const int64_t* out_off, int32_t* counters, float* out_val,
                         int32_t* out_idx, float* resid, int64_t idx_base, hipStream_t stream) {
  GRACE_HIP_CHECK(hipMemsetAsync(counters, 0, sizeof(int32_t) * 2 * n_seg, stream));
  if (resid != nullptr && resid == x)
    topk_compact_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, st, out_off, counters, n_seg, out_val,
                                                                  out_idx, resid, idx_base);
  else
    topk_compact_kernel<false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, st, out_off, counters, n_seg, out_val,
                                                                   out_idx, resid, idx_base);
}

void sparse_scatter_add(const float* val, const int32_t* idx, int64_t K, float* out, float scale,
                        bool accumulate, hipStream_t stream) {
  if (K <= 0) return;
  int64_t blocks = (K + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  sparse_scatter_add_kernel<<<(int)blocks, kBlock, 0, stream>>>(val, idx, K, out, scale, accumulate ? 1 : 0);
}

}  // namespace grace
