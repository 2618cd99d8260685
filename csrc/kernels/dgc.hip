// Deep Gradient Compression threshold selection on the device (CDNA4).
//
// Reference per tensor (/root/reference/grace_dl/dist/compressor/dgc.py:12-43): uniform 1%
// sample -> k'-th largest |sample| -> up to 10 host-side refinements (x1.3 / x0.7) each with a
// full mask + sum -> torch.where.  That is ~30 launches and up to 10 host syncs per tensor.
//
// Here, for all segments of a bucket at once:
//   dgc_sample   : Philox-uniform sample positions per segment, |x| gathered (1 thread/sample)
//   (top-k of the samples reuses the segmented radix select of topk.hip -> exact k'-th key)
//   dgc_count_tree: per-chunk counts of |x| >= each of the 7 thresholds the next 3 refinement
//                  steps can reach (segments already converged exit early), one atomic per
//                  workgroup and threshold
//   dgc_adjust_tree: per segment, the reference's rule walked 3 steps down the counted tree;
//                  marks converged segments done
//   dgc_compact  : ballot compaction of |x| >= thr[seg] into (value, flat index)
//   dgc_compact  : capacity-bounded (the payload has a fixed capacity and an in-band count, so
//                  the exchange needs no host sync and is graph-capturable), DgcMemory's u / v
//                  masking fused in
//   dgc_compensate: DgcMemory's momentum correction + accumulation in one pass
#include "grace_common.h"
#include "grace_kernels.h"
#include "grace_scan.h"

namespace grace {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ int find_seg64(const int64_t* __restrict__ off, int n_seg, int64_t j) {
  int lo = 0, hi = n_seg;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// Comp (optional): DgcMemory's compensate evaluated AT THE SAMPLE POSITIONS ONLY -- x is g and
// the sampled value is v' = v + fmaf(m, u, g) (first call: g), the exact float ops of
// dgc_compensate_kernel -- so the full compensate pass can run fused into the first count pass.
struct Comp {
  const float* u;
  const float* v;
  float m;
  int first;  // -1: off (x is the compensated v itself)
};

__device__ __forceinline__ float comp_at(const float* x, const Comp& c, int64_t i) {
  const float g = x[i];
  if (c.first < 0 || c.first == 1) return g;
  return c.v[i] + fmaf(c.m, c.u[i], g);
}

__global__ __launch_bounds__(kBlock) void dgc_sample_kernel(const float* __restrict__ x, int n_seg,
                                                            const int64_t* __restrict__ seg_off,
                                                            const int64_t* __restrict__ samp_off, SeedArg sa,
                                                            float* __restrict__ samples, Comp cp) {
  const int64_t S = samp_off[n_seg];
  const uint64_t seed = sa.get();  // device step mixed in: fresh samples on every graph replay
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < S; j += stride) {
    const int s = find_seg64(samp_off, n_seg, j);
    const int64_t n = seg_off[s + 1] - seg_off[s];
    const uint4 r = Philox::gen(seed, (uint64_t)j);
    // 48 random bits -> uniform position in [0, n)
    const uint64_t u = ((uint64_t)r.x << 16) ^ (uint64_t)(r.y >> 16);
    const int64_t pos = (int64_t)__umul64hi(u << 16, (uint64_t)n);  // floor(u * n / 2^48)
    samples[j] = fabsf(comp_at(x, cp, seg_off[s] + (pos < n ? pos : n - 1)));
  }
}

// thr[s] <- float(prefix of the k'-th largest sample key); count[s] = 0; done[s] = 0
__global__ void dgc_init_kernel(int n_seg, const TopkState* __restrict__ st, float* __restrict__ thr,
                                int32_t* __restrict__ count, int32_t* __restrict__ done) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_seg) return;
  thr[s] = __uint_as_float(st[s].prefix);
  count[s] = 0;
  done[s] = 0;
}

// Speculative refinement: the reference's loop (count at thr; x1.3 when too many, x0.7 when too
// few; stop inside [0.7, 1.3] x target or after max_iters adjustments) needs one count pass per
// step.  Its next kDepth thresholds form a binary tree from the current root (node k's children:
// 2k+1 = node x 1.3f, 2k+2 = node x 0.7f, the same float products the sequential loop forms),
// so ONE pass counts all kTree tree thresholds and the adjust kernel then walks kDepth steps
// down the tree: ceil(max_iters / kDepth) passes (2 for the reference's 10) instead of
// max_iters, with bit-identical thresholds and counts.  Per segment, count[32s + k] (k < kTree)
// holds the tree counts and count[32s + 31] the adjustments made so far.  (Depth 5: 31 register
// counters and 31 compares per element -- VALU work well under the pass's HBM time; depth 3
// needed 4 passes over the bucket.)
constexpr int kDepth = 5;
constexpr int kTree = (1 << kDepth) - 1;  // 31
constexpr int kCntStride = 32;

__device__ __forceinline__ void tree_thresholds(float root, float* t) {
  t[0] = root;
#pragma unroll
  for (int k = 0; k < kTree / 2; ++k) {
    t[2 * k + 1] = t[k] * 1.3f;
    t[2 * k + 2] = t[k] * 0.7f;
  }
}

// FUSE: the first count pass also performs DgcMemory's compensate for its chunk: x is g, and
// u / v are updated in place (u = m u + g; v = v + u; first: u = v = g) -- the counted value is
// the new v, exactly as a separate compensate pass followed by a count pass would see it.
template <bool FUSE>
__global__ __launch_bounds__(kBlock) void dgc_count_tree_kernel(ChunkTable ct, const float* __restrict__ x,
                                                                const float* __restrict__ thr,
                                                                const int32_t* __restrict__ done,
                                                                int32_t* __restrict__ count, float* __restrict__ uu,
                                                                float* __restrict__ vv, float m, int first) {
  const int c = blockIdx.x;
  const int s = ct.seg[c];
  if (!FUSE && done[s]) return;  // (the fused pass runs before any segment converged)
  const int64_t b = ct.begin[c], e = ct.end[c];
  float t[kTree];
  tree_thresholds(thr[s], t);
  unsigned cnt[kTree];
#pragma unroll
  for (int k = 0; k < kTree; ++k) cnt[k] = 0;
  auto one = [&](float val) {
    const float a = fabsf(val);
#pragma unroll
    for (int k = 0; k < kTree; ++k) cnt[k] += a >= t[k] ? 1u : 0u;
  };
  auto comp1 = [&](int64_t i) -> float {
    const float g = x[i];
    if (!FUSE) return g;
    float un, vn;
    if (first) {
      un = vn = g;
    } else {
      un = fmaf(m, uu[i], g);
      vn = vv[i] + un;
    }
    uu[i] = un;
    vv[i] = vn;
    return vn;
  };
  // 16-B body (x, u, v share their alignment: same offsets into equally aligned buffers)
  const int64_t mis = (int64_t)((reinterpret_cast<uintptr_t>(x) >> 2) & 3);
  int64_t a0 = b + ((4 - ((b + mis) & 3)) & 3);
  if (a0 > e) a0 = e;
  const int64_t a1 = a0 + ((e - a0) & ~(int64_t)3);
  for (int64_t i = b + threadIdx.x; i < a0; i += kBlock) one(comp1(i));
  for (int64_t i = a1 + threadIdx.x; i < e; i += kBlock) one(comp1(i));
  for (int64_t i = a0 + 4 * (int64_t)threadIdx.x; i < a1; i += 4 * kBlock) {
    float4 g4 = *reinterpret_cast<const float4*>(x + i);
    if constexpr (FUSE) {
      float4 u4, v4;
      if (first) {
        u4 = v4 = g4;
      } else {
        u4 = *reinterpret_cast<const float4*>(uu + i);
        v4 = *reinterpret_cast<const float4*>(vv + i);
        u4 = make_float4(fmaf(m, u4.x, g4.x), fmaf(m, u4.y, g4.y), fmaf(m, u4.z, g4.z), fmaf(m, u4.w, g4.w));
        v4 = make_float4(v4.x + u4.x, v4.y + u4.y, v4.z + u4.z, v4.w + u4.w);
      }
      *reinterpret_cast<float4*>(uu + i) = u4;
      *reinterpret_cast<float4*>(vv + i) = v4;
      g4 = v4;
    }
    one(g4.x);
    one(g4.y);
    one(g4.z);
    one(g4.w);
  }
  __shared__ unsigned red[kBlock / kWave][kTree];
#pragma unroll
  for (int k = 0; k < kTree; ++k) {
    const unsigned w = wave_sum_u32(cnt[k]);
    if (lane_id() == 0) red[wave_id()][k] = w;
  }
  __syncthreads();
  if (threadIdx.x < kTree) {
    unsigned tot = 0;
    for (int w = 0; w < kBlock / kWave; ++w) tot += red[w][threadIdx.x];
    if (tot) atomicAdd(&count[s * kCntStride + threadIdx.x], (int32_t)tot);
  }
}

// walk up to kDepth adjustments down the counted tree; the node reached becomes the next root
__global__ void dgc_adjust_tree_kernel(int n_seg, const float* __restrict__ target, float* __restrict__ thr,
                                       int32_t* __restrict__ count, int32_t* __restrict__ done, int max_iters) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_seg || done[s]) return;
  int32_t* cs = count + s * kCntStride;
  int it = cs[kTree];
  float t = thr[s];
  int node = 0;
  bool fin = false;
  for (int d = 0; d < kDepth; ++d) {
    if (it >= max_iters) {
      fin = true;
      break;
    }
    const float sel = (float)cs[node];
    ++it;
    if (sel > 1.3f * target[s]) {
      t *= 1.3f;
      node = 2 * node + 1;
    } else if (sel < 0.7f * target[s]) {
      t *= 0.7f;
      node = 2 * node + 2;
    } else {
      fin = true;
      break;
    }
  }
  thr[s] = t;
  if (fin || it >= max_iters) done[s] = 1;
  for (int k = 0; k < kTree; ++k) cs[k] = 0;  // recounted by the next pass
  cs[kTree] = it;
}

constexpr int kPer = 32;
constexpr int kTile = kBlock * kPer;

// |x| >= thr[seg] -> (value, flat index); one atomic per 256x32 tile (grace_scan.h)
// cap: payload capacity -- entries selected past it are not sent (and, with the fused DgcMemory
// masking, keep their u / v, so they are sent by a later step: spill instead of loss).
// vmask / umask (optional): DgcMemory.update fused in -- v and u are zeroed where sent.
__global__ __launch_bounds__(kBlock) void dgc_compact_kernel(ChunkTable ct, const float* __restrict__ x,
                                                             const float* __restrict__ thr,
                                                             float* __restrict__ out_val,
                                                             int32_t* __restrict__ out_idx, int64_t cap,
                                                             int32_t* __restrict__ counter, float* vmask,
                                                             float* __restrict__ umask) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int bcast;
  const int c = blockIdx.x;
  const int s = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const float t = thr[s];
  for (int64_t tb = b; tb < e; tb += kTile) {
    float v[kPer];
    uint32_t take = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = tb + (int64_t)j * kBlock + threadIdx.x;
      v[j] = 0.f;
      if (i < e) {
        v[j] = x[i];
        take |= (fabsf(v[j]) >= t ? 1u : 0u) << j;
      }
    }
    int tot = 0;
    const int pre = block_exclusive_scan<kBlock>(__popc(take), lds, &tot);
    if (tot > 0) {
      if (threadIdx.x == 0) bcast = atomicAdd(counter, tot);
      __syncthreads();
      int64_t p = (int64_t)bcast + pre;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if ((take >> j) & 1u) {
          if (p < cap) {
            const int64_t i = tb + (int64_t)j * kBlock + threadIdx.x;
            out_val[p] = v[j];
            out_idx[p] = (int32_t)i;
            if (vmask != nullptr) vmask[i] = 0.f;
            if (umask != nullptr) umask[i] = 0.f;
          }
          ++p;
        }
      }
    }
    __syncthreads();
  }
}

// DgcMemory.compensate fused: u = m*u + g; v = v + u (first call: u = v = g).  One pass reading
// g, u, v and writing u, v instead of three eager elementwise launches.
__global__ __launch_bounds__(kBlock) void dgc_compensate_kernel(const float* __restrict__ g, float* __restrict__ u,
                                                                float* __restrict__ v, float m, int64_t n,
                                                                int first) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* u4 = reinterpret_cast<float4*>(u);
  float4* v4 = reinterpret_cast<float4*>(v);
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += stride) {
    const float4 gg = g4[i];
    if (first) {
      u4[i] = gg;
      v4[i] = gg;
    } else {
      float4 uu = u4[i], vv = v4[i];
      uu = make_float4(fmaf(m, uu.x, gg.x), fmaf(m, uu.y, gg.y), fmaf(m, uu.z, gg.z), fmaf(m, uu.w, gg.w));
      vv = make_float4(vv.x + uu.x, vv.y + uu.y, vv.z + uu.z, vv.w + uu.w);
      u4[i] = uu;
      v4[i] = vv;
    }
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const float gg = g[i];
    const float uu = first ? gg : fmaf(m, u[i], gg);
    u[i] = uu;
    v[i] = first ? gg : v[i] + uu;
  }
}

inline int grid_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

void dgc_sample(const float* x, int n_seg, const int64_t* seg_off, const int64_t* samp_off, int64_t n_samples,
                SeedArg seed, float* samples, const float* u, const float* v, float momentum, int first,
                hipStream_t stream) {
  if (n_samples <= 0) return;
  const Comp cp{u, v, momentum, u != nullptr ? first : -1};
  dgc_sample_kernel<<<grid_for(n_samples), kBlock, 0, stream>>>(x, n_seg, seg_off, samp_off, seed, samples, cp);
}

void dgc_refine(const ChunkTable& ct, int n_seg, const float* x, const TopkState* st, const float* target,
                int max_iters, float* thr, int32_t* count, int32_t* done, float* u, float* v, float momentum,
                int first, int64_t n, hipStream_t stream) {
  const int g = (n_seg + 255) / 256;
  dgc_init_kernel<<<g, 256, 0, stream>>>(n_seg, st, thr, count, done);
  GRACE_HIP_CHECK(hipMemsetAsync(count, 0, sizeof(int32_t) * (size_t)n_seg * kCntStride, stream));
  const bool fuse = u != nullptr;
  if (fuse && max_iters <= 0) {  // no count pass to carry the compensate: run it alone
    dgc_compensate(x, u, v, momentum, n, first != 0, stream);
    return;
  }
  // ceil(max_iters / kDepth) count passes; the count after the last adjustment is never formed.
  // With u / v given, x is the raw gradient and the FIRST pass applies DgcMemory's compensate
  // (writing u, v); later passes (and the compaction) read v.
  for (int it = 0; it < max_iters; it += kDepth) {
    if (fuse && it == 0)
      dgc_count_tree_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, done, count, u, v, momentum, first);
    else
      dgc_count_tree_kernel<false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, fuse ? v : x, thr, done, count, nullptr,
                                                                       nullptr, 0.f, 0);
    dgc_adjust_tree_kernel<<<g, 256, 0, stream>>>(n_seg, target, thr, count, done, max_iters);
  }
}

void dgc_compact(const ChunkTable& ct, const float* x, const float* thr, float* out_val, int32_t* out_idx,
                 int64_t cap, int32_t* counter, float* vmask, float* umask, hipStream_t stream, int header_bytes) {
  GRACE_HIP_CHECK(hipMemsetAsync(counter, 0, header_bytes, stream));
  if (ct.n_chunks == 0) return;
  dgc_compact_kernel<<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, out_val, out_idx, cap, counter, vmask, umask);
}

void dgc_compensate(const float* g, float* u, float* v, float momentum, int64_t n, bool first, hipStream_t stream) {
  if (n <= 0) return;
  dgc_compensate_kernel<<<grid_for((n + 3) / 4), kBlock, 0, stream>>>(g, u, v, momentum, n, first ? 1 : 0);
}

}  // namespace grace
