// Adaq (AdaComp-style two-sided sparsification, Dryden et al. MLHPC 2016) on CDNA4.
//
// Reference (TF only): /root/reference/grace_dl/tensorflow/compressor/adaq.py:15-93.  For the
// positive and the negative entries of a tensor separately: threshold from a 1% sample so that
// about `ratio` of that side passes, refined (x1.25 while the count > 1.25*target, x0.9 while
// < 0.8*target, <= 20 times; x0.8 if nothing passes), then only the MEAN of the selected values
// and their indices are sent.
//
// All segments of a bucket and both sides ("groups" g = 2*seg + side, key_side(x) = max(+-x, 0))
// are processed together, on the device, with one host read (the payload size):
//   adaq_sample   Philox positions (a 1% sample of the segment), both sides' keys written
//   adaq_prep     per group: side size n_g (counted by adaq_count with threshold 0), target
//                 ceil(ratio*n_g), and k' = ceil(ratio * expected side entries of the sample)
//   (segmented radix select of topk.hip on the sample keys -> initial thresholds)
//   adaq_init / adaq_count / adaq_adjust / adaq_post   the refinement loop, both sides per pass
//   adaq_scan     exclusive offsets of the final group counts (one workgroup)
//   adaq_compact  indices of every group written in (segment, side) order -- one atomic per
//                 tile and group -- plus fp64 per-chunk partial sums of the selected values
//   adaq_means    group means folded from the partials in chunk order (deterministic)
#include "grace_common.h"
#include "grace_kernels.h"
#include "grace_scan.h"

namespace grace {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float side_key(float v, int side) { return side == 0 ? fmaxf(v, 0.f) : fmaxf(-v, 0.f); }

__device__ __forceinline__ int find_seg(const int64_t* __restrict__ off, int n, int64_t j) {
  int lo = 0, hi = n;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// samples laid out by group: group 2s holds the + keys, 2s+1 the - keys of the same positions.
// samp_off: [n_seg+1] offsets of segment s's sample within ONE side.
__global__ __launch_bounds__(kBlock) void adaq_sample_kernel(const float* __restrict__ x, int n_seg,
                                                             const int64_t* __restrict__ seg_off,
                                                             const int64_t* __restrict__ samp_off, SeedArg sa,
                                                             float* __restrict__ samples) {
  const uint64_t seed = sa.get();
  const int64_t S = samp_off[n_seg];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < S; j += stride) {
    const int s = find_seg(samp_off, n_seg, j);
    const int64_t n = seg_off[s + 1] - seg_off[s];
    const uint4 r = Philox::gen(seed, (uint64_t)j, 0x61646171u);
    const uint64_t u = ((uint64_t)r.x << 16) ^ (uint64_t)(r.y >> 16);
    int64_t pos = (int64_t)__umul64hi(u << 16, (uint64_t)n);
    if (pos >= n) pos = n - 1;
    const float v = x[seg_off[s] + pos];
    const int64_t ns = samp_off[s + 1] - samp_off[s];
    const int64_t local = j - samp_off[s];
    // group-major layout: [seg0 +][seg0 -][seg1 +][seg1 -]...
    samples[2 * samp_off[s] + local] = side_key(v, 0);
    samples[2 * samp_off[s] + ns + local] = side_key(v, 1);
  }
}

// count[g] += #{ key_side(x) (>|>=) thr[g] } over the chunks of not-yet-converged groups
template <bool STRICT>
__global__ __launch_bounds__(kBlock) void adaq_count_kernel(ChunkTable ct, const float* __restrict__ x,
                                                            const float* __restrict__ thr,
                                                            const int32_t* __restrict__ done,
                                                            int32_t* __restrict__ count) {
  const int c = blockIdx.x;
  const int s = ct.seg[c];
  const bool d0 = done[2 * s] != 0, d1 = done[2 * s + 1] != 0;
  if (d0 && d1) return;
  const int64_t b = ct.begin[c], e = ct.end[c];
  const float t0 = thr[2 * s], t1 = thr[2 * s + 1];
  unsigned c0 = 0, c1 = 0;
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    const float v = x[i];
    const float k0 = side_key(v, 0), k1 = side_key(v, 1);
    c0 += (STRICT ? k0 > t0 : k0 >= t0) ? 1u : 0u;
    c1 += (STRICT ? k1 > t1 : k1 >= t1) ? 1u : 0u;
  }
  c0 = wave_sum_u32(c0);
  c1 = wave_sum_u32(c1);
  __shared__ unsigned red[2][kBlock / kWave];
  if (lane_id() == 0) {
    red[0][wave_id()] = c0;
    red[1][wave_id()] = c1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    unsigned tot = 0;
    for (int w = 0; w < kBlock / kWave; ++w) tot += red[threadIdx.x][w];
    const int g = 2 * s + (int)threadIdx.x;
    if (tot && !done[g]) atomicAdd(&count[g], (int32_t)tot);
  }
}

// side sizes are in count[]; derive target, k' (the sample has ns_s entries per side) and the
// fallback threshold (the side's mean |x| from the segment statistics)
__global__ void adaq_prep_kernel(int n_groups, const int64_t* __restrict__ seg_off,
                                 const int64_t* __restrict__ samp_off, const float* __restrict__ stats, float ratio,
                                 int32_t* __restrict__ count, float* __restrict__ target, int32_t* __restrict__ kseg,
                                 float* __restrict__ fallback, int32_t* __restrict__ done) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const int s = g >> 1;
  const int64_t n = seg_off[s + 1] - seg_off[s];
  const int64_t ns = samp_off[s + 1] - samp_off[s];
  const int32_t ng = count[g];
  target[g] = ceilf(ratio * (float)ng);
  // expected side entries among the ns samples, times ratio (reference: k = ceil(n_side*0.01*ratio)
  // out of ceil(n_side*0.01) side samples)
  const float expect = n > 0 ? (float)ns * (float)ng / (float)n : 0.f;
  int k = (int)ceilf(ratio * expect);
  if (k < 1) k = 1;
  if (k > ns) k = (int)ns;
  kseg[g] = ns > 0 ? k : 0;
  const float sum = stats[s * kSegStats + 0], abssum = stats[s * kSegStats + 3];
  const float side_abs = (g & 1) ? 0.5f * (abssum - sum) : 0.5f * (abssum + sum);
  fallback[g] = ng > 0 ? side_abs / (float)ng : 0.f;
  count[g] = 0;
  done[g] = ng == 0 ? 1 : 0;  // an empty side sends mean 0 and no index
}

// thr <- k'-th largest sample key (fallback: the side's mean |x| when the sample missed the side)
__global__ void adaq_init_kernel(int n_groups, const TopkState* __restrict__ st, const float* __restrict__ fallback,
                                 float* __restrict__ thr) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  float t = __uint_as_float(st[g].prefix);
  if (!(t > 0.f)) t = fallback[g];
  thr[g] = t;
}

// reference loop body (adaq.py:36-43): while the count is outside [0.8, 1.25]*target adjust
// and recount; count[] holds the latest count of every group (kept once converged)
__global__ void adaq_adjust_kernel(int n_groups, const float* __restrict__ target, float* __restrict__ thr,
                                   int32_t* __restrict__ count, int32_t* __restrict__ done) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups || done[g]) return;
  const float sel = (float)count[g];
  if (sel > 1.25f * target[g]) {
    thr[g] *= 1.25f;
  } else if (sel < 0.8f * target[g]) {
    thr[g] *= 0.9f;
  } else {
    done[g] = 1;
    return;
  }
  count[g] = 0;  // recounted by the next pass
}

// after the loop (adaq.py:44-48): nothing selected -> lower once more; then every group is
// recounted with the strict comparison of the final selection
__global__ void adaq_post_kernel(int n_groups, float* __restrict__ thr, int32_t* __restrict__ count,
                                 int32_t* __restrict__ done) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  if (count[g] < 1) thr[g] *= 0.8f;
  count[g] = 0;
  done[g] = 0;
}

// exclusive scan of count[] -> goff[0..n_groups], goff[n_groups] = total (one workgroup)
__global__ __launch_bounds__(kBlock) void adaq_scan_kernel(int n_groups, const int32_t* __restrict__ count,
                                                           int32_t* __restrict__ goff, int32_t* __restrict__ cursor) {
  __shared__ int lds[kBlock / kWave];
  int carry = 0;
  for (int g0 = 0; g0 < n_groups; g0 += kBlock) {
    const int g = g0 + threadIdx.x;
    const int v = g < n_groups ? count[g] : 0;
    int tot = 0;
    const int ex = block_exclusive_scan<kBlock>(v, lds, &tot);
    if (g < n_groups) {
      goff[g] = carry + ex;
      cursor[g] = carry + ex;
    }
    carry += tot;
  }
  if (threadIdx.x == 0) goff[n_groups] = carry;
}

constexpr int kPer = 32;
constexpr int kTile = kBlock * kPer;

// indices of key_side(x) > thr into idx[cursor[g]...]; per-chunk fp64 sums of the selected values
__global__ __launch_bounds__(kBlock) void adaq_compact_kernel(ChunkTable ct, const float* __restrict__ x,
                                                              const float* __restrict__ thr,
                                                              int32_t* __restrict__ cursor,
                                                              int32_t* __restrict__ idx, int64_t cap,
                                                              double* __restrict__ psum) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int bcast[2];
  __shared__ double red[2][kBlock / kWave];
  const int c = blockIdx.x;
  const int s = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const float t0 = thr[2 * s], t1 = thr[2 * s + 1];
  double sum0 = 0.0, sum1 = 0.0;
  for (int64_t tb = b; tb < e; tb += kTile) {
    uint32_t take0 = 0, take1 = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = tb + (int64_t)j * kBlock + threadIdx.x;
      if (i < e) {
        const float v = x[i];
        if (side_key(v, 0) > t0) {
          take0 |= 1u << j;
          sum0 += v;
        }
        if (side_key(v, 1) > t1) {
          take1 |= 1u << j;
          sum1 += v;
        }
      }
    }
    int tot0 = 0, tot1 = 0;
    const int pre0 = block_exclusive_scan<kBlock>(__popc(take0), lds, &tot0);
    const int pre1 = block_exclusive_scan<kBlock>(__popc(take1), lds, &tot1);
    if (threadIdx.x == 0) bcast[0] = tot0 ? atomicAdd(&cursor[2 * s], tot0) : 0;
    if (threadIdx.x == 1) bcast[1] = tot1 ? atomicAdd(&cursor[2 * s + 1], tot1) : 0;
    __syncthreads();
    int p0 = bcast[0] + pre0, p1 = bcast[1] + pre1;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int32_t i = (int32_t)(tb + (int64_t)j * kBlock + threadIdx.x);
      // slots past the payload capacity are not written (the group's sent count is clamped)
      if ((take0 >> j) & 1u) {
        if (p0 < cap) idx[p0] = i;
        ++p0;
      }
      if ((take1 >> j) & 1u) {
        if (p1 < cap) idx[p1] = i;
        ++p1;
      }
    }
    __syncthreads();
  }
  sum0 = wave_sum(sum0);
  sum1 = wave_sum(sum1);
  if (lane_id() == 0) {
    red[0][wave_id()] = sum0;
    red[1][wave_id()] = sum1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double t = 0.0;
    for (int w = 0; w < kBlock / kWave; ++w) t += red[threadIdx.x][w];
    psum[2 * (int64_t)c + threadIdx.x] = t;
  }
}

// one workgroup per segment: means of both sides from the chunk partials, in chunk order
__global__ __launch_bounds__(kBlock) void adaq_means_kernel(const int32_t* __restrict__ seg_chunk_begin,
                                                            const double* __restrict__ psum,
                                                            const int32_t* __restrict__ goff, int64_t cap,
                                                            float* __restrict__ means, int32_t* __restrict__ counts) {
  const int s = blockIdx.x;
  const int c0 = seg_chunk_begin[s], c1 = seg_chunk_begin[s + 1];
  double a0 = 0.0, a1 = 0.0;
  for (int c = c0 + (int)threadIdx.x; c < c1; c += kBlock) {
    a0 += psum[2 * (int64_t)c];
    a1 += psum[2 * (int64_t)c + 1];
  }
  __shared__ double red[2][kBlock / kWave];
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  if (lane_id() == 0) {
    red[0][wave_id()] = a0;
    red[1][wave_id()] = a1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double t = 0.0;
    for (int w = 0; w < kBlock / kWave; ++w) t += red[threadIdx.x][w];
    const int g = 2 * s + (int)threadIdx.x;
    const int cnt = goff[g + 1] - goff[g];
    // in-band header: the SENT count (slots inside the capacity); the mean is over the selection
    const int64_t hi = goff[g + 1] < cap ? goff[g + 1] : cap;
    counts[g] = hi > goff[g] ? (int)(hi - goff[g]) : 0;
    means[g] = cnt > 0 ? (float)(t / cnt) : 0.f;
  }
}

// decode one rank's payload: out[idx[j]] += means[group(j)] * scale for j < sum(counts), groups
// laid out back to back (exclusive scan of the in-band counts; no host read of the size)
__global__ __launch_bounds__(kBlock) void adaq_decode_scan_kernel(int n_groups, const int32_t* __restrict__ counts,
                                                                  int32_t* __restrict__ goff) {
  __shared__ int lds[kBlock / kWave];
  int carry = 0;
  for (int g0 = 0; g0 < n_groups; g0 += kBlock) {
    const int g = g0 + threadIdx.x;
    const int v = g < n_groups ? counts[g] : 0;
    int tot = 0;
    const int ex = block_exclusive_scan<kBlock>(v, lds, &tot);
    if (g < n_groups) goff[g] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) goff[n_groups] = carry;
}

__global__ __launch_bounds__(kBlock) void adaq_decode_kernel(int n_groups, const float* __restrict__ means,
                                                             const int32_t* __restrict__ goff,
                                                             const int32_t* __restrict__ idx, int64_t cap,
                                                             float* __restrict__ out, float scale) {
  const int64_t tot = goff[n_groups];
  const int64_t K = tot < cap ? tot : cap;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < K; j += stride) {
    int lo = 0, hi = n_groups;  // last group with goff[g] <= j
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (goff[mid] <= j)
        lo = mid;
      else
        hi = mid;
    }
    out[idx[j]] += means[lo] * scale;
  }
}

inline int grid_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

void adaq_sample(const float* x, int n_seg, const int64_t* seg_off, const int64_t* samp_off, int64_t n_samples,
                 SeedArg seed, float* samples, hipStream_t stream) {
  if (n_samples <= 0) return;
  adaq_sample_kernel<<<grid_for(n_samples), kBlock, 0, stream>>>(x, n_seg, seg_off, samp_off, seed, samples);
}

void adaq_prepare(const ChunkTable& ct, int n_seg, const float* x, const int64_t* seg_off, const int64_t* samp_off,
                  const float* stats, float ratio, int32_t* count, float* target, int32_t* kseg, float* fallback,
                  float* thr, int32_t* done, hipStream_t stream) {
  const int ng = 2 * n_seg;
  GRACE_HIP_CHECK(hipMemsetAsync(count, 0, sizeof(int32_t) * ng, stream));
  GRACE_HIP_CHECK(hipMemsetAsync(thr, 0, sizeof(float) * ng, stream));
  GRACE_HIP_CHECK(hipMemsetAsync(done, 0, sizeof(int32_t) * ng, stream));
  if (ct.n_chunks > 0) adaq_count_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, done, count);
  adaq_prep_kernel<<<(ng + 255) / 256, 256, 0, stream>>>(ng, seg_off, samp_off, stats, ratio, count, target, kseg,
                                                          fallback, done);
}

void adaq_refine(const ChunkTable& ct, int n_seg, const float* x, const TopkState* st, const float* fallback,
                 const float* target, int max_iters, float* thr, int32_t* count, int32_t* done, hipStream_t stream) {
  const int ng = 2 * n_seg;
  const int g = (ng + 255) / 256;
  adaq_init_kernel<<<g, 256, 0, stream>>>(ng, st, fallback, thr);
  if (ct.n_chunks > 0) adaq_count_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, done, count);
  for (int it = 0; it < max_iters; ++it) {
    adaq_adjust_kernel<<<g, 256, 0, stream>>>(ng, target, thr, count, done);
    if (ct.n_chunks > 0) adaq_count_kernel<false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, done, count);
  }
  adaq_post_kernel<<<g, 256, 0, stream>>>(ng, thr, count, done);
  if (ct.n_chunks > 0) adaq_count_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, done, count);
}

void adaq_offsets(int n_seg, const int32_t* count, int32_t* goff, int32_t* cursor, hipStream_t stream) {
  adaq_scan_kernel<<<1, kBlock, 0, stream>>>(2 * n_seg, count, goff, cursor);
}

void adaq_compact(const ChunkTable& ct, int n_seg, const int32_t* seg_chunk_begin, const float* x, const float* thr,
                  const int32_t* goff, int32_t* cursor, int32_t* idx, int64_t cap, double* psum, float* means,
                  int32_t* counts, hipStream_t stream) {
  if (ct.n_chunks > 0)
    adaq_compact_kernel<<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, cursor, idx, cap, psum);
  if (n_seg > 0) adaq_means_kernel<<<n_seg, kBlock, 0, stream>>>(seg_chunk_begin, psum, goff, cap, means, counts);
}

void adaq_decode(int n_groups, const float* means, const int32_t* counts, const int32_t* idx, int64_t cap,
                 int32_t* goff_ws, float* out, float scale, hipStream_t stream) {
  adaq_decode_scan_kernel<<<1, kBlock, 0, stream>>>(n_groups, counts, goff_ws);
  adaq_decode_kernel<<<grid_for(cap), kBlock, 0, stream>>>(n_groups, means, goff_ws, idx, cap, out, scale);
}

}  // namespace grace
