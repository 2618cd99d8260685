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
//   dgc_scan     : output offset of every chunk = prefix sum of the chunk counts the last count
//                  pass already formed at the final threshold (one workgroup)
//   dgc_compact  : compaction of |x| >= thr[seg] into (value, flat index) at those offsets --
//                  no atomics, deterministic slots; capacity-bounded (the payload has a fixed
//                  capacity and an in-band count, so the exchange needs no host sync and is
//                  graph-capturable), DgcMemory's u / v masking fused in
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

constexpr int kCntStride = 32;

// The k'-th largest |sample| of every segment, exactly (3-digit radix select: bits 30..20,
// 19..9, 8..0 of the |x| key, as topk.hip's segmented select), ONE workgroup per segment with the
// samples cached in LDS -- and the refinement state initialised in the same launch: thr[s] = that
// value, the 32 count words = 0, done = 0, fnode = -1.  Replaces 3 histogram + 3 select launches
// over the (tiny) sample set plus the init launch: ~40 us of launch latency per DGC step.
constexpr int kSelBlock = 1024;
constexpr int kSelLds = 24576;  // samples cached in LDS (96 KB); a larger segment re-reads them

__global__ __launch_bounds__(kSelBlock) void dgc_select_init_kernel(
    const float* __restrict__ samples, const int64_t* __restrict__ samp_off, const int32_t* __restrict__ kseg,
    TopkState* __restrict__ st, float* __restrict__ thr, int32_t* __restrict__ count, int32_t* __restrict__ done,
    int32_t* __restrict__ fnode) {
  __shared__ uint32_t keys[kSelLds];
  __shared__ int32_t hist[2048];
  __shared__ int part[kSelBlock / kWave];
  __shared__ uint32_t s_prefix;
  __shared__ int32_t s_krem;
  const int s = blockIdx.x;
  const int64_t so = samp_off[s], ns = samp_off[s + 1] - so;
  const bool in_lds = ns <= kSelLds;
  if (in_lds)
    for (int64_t i = threadIdx.x; i < ns; i += kSelBlock) keys[i] = abs_key(samples[so + i]);
  if (threadIdx.x == 0) {
    s_prefix = 0u;
    s_krem = kseg[s];
  }
  __syncthreads();
  constexpr int kShift[3] = {20, 9, 0};
  constexpr int kBits[3] = {11, 11, 9};
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    const int shift = kShift[d], nbins = 1 << kBits[d];
    for (int i = threadIdx.x; i < nbins; i += kSelBlock) hist[i] = 0;
    __syncthreads();
    const uint32_t want = d == 0 ? 0u : s_prefix >> (shift + kBits[d]);
    const int32_t krem = s_krem;
    for (int64_t i = threadIdx.x; i < ns; i += kSelBlock) {
      const uint32_t key = in_lds ? keys[i] : abs_key(samples[so + i]);
      if (d == 0 || (key >> (shift + kBits[d])) == want) atomicAdd(&hist[(key >> shift) & (nbins - 1)], 1);
    }
    __syncthreads();
    // descending bins: thread t owns positions [2t, 2t + 2) (bin = nbins - 1 - position)
    int32_t loc[2] = {0, 0};
    int32_t sum = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int j = 2 * (int)threadIdx.x + q;
      if (j < nbins) loc[q] = hist[nbins - 1 - j];
      sum += loc[q];
    }
    int tot = 0;
    const int32_t excl = block_exclusive_scan<kSelBlock>(sum, part, &tot);
    if (excl < krem && krem <= excl + sum) {
      int32_t run = excl;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (run + loc[q] >= krem) {
          const uint32_t bin = (uint32_t)(nbins - 1 - (2 * (int)threadIdx.x + q));
          s_prefix = (d == 0 ? 0u : s_prefix) | (bin << shift);
          s_krem = krem - run;
          break;
        }
        run += loc[q];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    st[s].prefix = s_prefix;
    st[s].krem = s_krem;
    thr[s] = __uint_as_float(s_prefix);
    done[s] = 0;
    fnode[s] = -1;
  }
  if (threadIdx.x < kCntStride) count[s * kCntStride + threadIdx.x] = 0;
}

// thr[s] <- float(prefix of the k'-th largest sample key); the segment's 32 count words = 0;
// done[s] = 0; fnode[s] = -1 (no counted final threshold yet)
__global__ void dgc_init_kernel(int n_seg, const TopkState* __restrict__ st, float* __restrict__ thr,
                                int32_t* __restrict__ count, int32_t* __restrict__ done,
                                int32_t* __restrict__ fnode) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_seg) return;
  thr[s] = __uint_as_float(st[s].prefix);
#pragma unroll
  for (int k = 0; k < kCntStride; ++k) count[s * kCntStride + k] = 0;
  done[s] = 0;
  fnode[s] = -1;
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
                                                                float* __restrict__ vv, float m, int first,
                                                                int32_t* __restrict__ ccnt) {
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
    // this chunk's count at every tree threshold: the compaction's offset at the final one (a
    // segment that converged keeps the counts of the pass it converged in: later passes exit above)
    ccnt[(int64_t)c * kCntStride + threadIdx.x] = (int32_t)tot;
  }
}

// walk up to kDepth adjustments down the counted tree; the node reached becomes the next root
// fnode[s]: the tree node of the final threshold when the segment converges -- counted by this
// pass (node < kTree) -- or -1 when the walk ended one level below the counted tree (the
// compaction then reserves that segment's slots with atomics)
__global__ void dgc_adjust_tree_kernel(int n_seg, const float* __restrict__ target, float* __restrict__ thr,
                                       int32_t* __restrict__ count, int32_t* __restrict__ done, int max_iters,
                                       int32_t* __restrict__ fnode) {
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
  if (fin || it >= max_iters) {
    done[s] = 1;
    fnode[s] = node < kTree ? node : -1;
  }
  for (int k = 0; k < kTree; ++k) cs[k] = 0;  // recounted by the next pass
  cs[kTree] = it;
}

constexpr int kV = 8;                     // float4 per thread per tile
constexpr int kTileV = kBlock * kV * 4;   // 8192 elements
constexpr int kScanBlock = 1024;

// Chunk output offsets: an exclusive prefix sum over chunks of the count the last count pass
// formed at the segment's final threshold (ccnt[c][fnode[seg]]; chunks of a segment whose final
// threshold was not counted contribute 0 and reserve their slots with atomics after the total).
// Also writes the payload header: word 0 = that total (the atomics add to it), words 1.. = 0.
__global__ __launch_bounds__(kScanBlock) void dgc_scan_kernel(const int32_t* __restrict__ seg, int n_chunks,
                                                              const int32_t* __restrict__ ccnt,
                                                              const int32_t* __restrict__ fnode,
                                                              int32_t* __restrict__ coff, int32_t* counter,
                                                              int header_words) {
  __shared__ int lds[kScanBlock / kWave];
  int carry = 0;
  for (int c0 = 0; c0 < n_chunks; c0 += kScanBlock) {
    const int c = c0 + threadIdx.x;
    int v = 0;
    if (c < n_chunks) {
      const int f = fnode[seg[c]];
      v = f >= 0 ? ccnt[(int64_t)c * kCntStride + f] : 0;
    }
    int tot = 0;
    const int pre = block_exclusive_scan<kScanBlock>(v, lds, &tot);
    if (c < n_chunks) coff[c] = carry + pre;
    carry += tot;
  }
  if (threadIdx.x == 0) counter[0] = carry;
  if (threadIdx.x > 0 && threadIdx.x < header_words) counter[threadIdx.x] = 0;
}

// |x| >= thr[seg] -> (value, flat index) at the chunk's scanned offset (the selection repeats the
// count pass's comparison bit for bit, so the chunk fills exactly its range; chunk order, thread-
// major inside a 256 x 8 x float4 tile: the same payload bytes on every run); chunks of an
// uncounted final threshold reserve one atomic per tile.  No same-address atomics otherwise: the round-4 kernel
// took one per tile on the payload counter from every workgroup of the bucket (~2000 on ONE word,
// serialised at the memory side: 44 us for a 16.6 M-element bucket, 1.5 TB/s).
// cap: payload capacity -- entries selected past it are not sent (and, with the fused DgcMemory
// masking, keep their u / v, so they are sent by a later step: spill instead of loss).
// vmask / umask (optional): DgcMemory.update fused in -- v and u are zeroed where sent.
__global__ __launch_bounds__(kBlock) void dgc_compact_kernel(ChunkTable ct, const float* __restrict__ x,
                                                             const float* __restrict__ thr,
                                                             float* __restrict__ out_val,
                                                             int32_t* __restrict__ out_idx, int64_t cap,
                                                             int32_t* __restrict__ counter, float* vmask,
                                                             float* __restrict__ umask,
                                                             const int32_t* __restrict__ fnode,
                                                             const int32_t* __restrict__ coff) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int bcast;
  const int c = blockIdx.x;
  const int s = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const float t = thr[s];
  const bool scanned = fnode[s] >= 0;
  int64_t base = scanned ? coff[c] : 0;
  // 16-B body [a0, a1) in float4 loads (4-B loads ran the pass at ~1.5 TB/s); the <= 3 + 3 head /
  // tail elements of a misaligned chunk ride along with the first tile (threads 0..5)
  const int64_t mis = (int64_t)((reinterpret_cast<uintptr_t>(x) >> 2) & 3);
  int64_t a0 = b + ((4 - ((b + mis) & 3)) & 3);
  if (a0 > e) a0 = e;
  const int64_t a1 = a0 + ((e - a0) & ~(int64_t)3);
  const int nh = (int)(a0 - b), nt = (int)(e - a1);
  bool first = true;
  for (int64_t tb = a0; first || tb < a1; tb += kTileV) {
    float4 v[kV];
    uint32_t take = 0;
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      const int64_t i = tb + 4 * ((int64_t)j * kBlock + threadIdx.x);
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < a1) {
        v[j] = *reinterpret_cast<const float4*>(x + i);
        take |= ((fabsf(v[j].x) >= t ? 1u : 0u) | (fabsf(v[j].y) >= t ? 2u : 0u) | (fabsf(v[j].z) >= t ? 4u : 0u) |
                 (fabsf(v[j].w) >= t ? 8u : 0u)) << (4 * j);
      }
    }
    float xe = 0.f;
    int64_t ie = -1;
    if (first) {
      const int th = (int)threadIdx.x;
      ie = th < nh ? b + th : (th < nh + nt ? a1 + (th - nh) : -1);
      if (ie >= 0) {
        xe = x[ie];
        if (!(fabsf(xe) >= t)) ie = -1;
      }
    }
    int tot = 0;
    const int pre = block_exclusive_scan<kBlock>(__popc(take) + (ie >= 0 ? 1 : 0), lds, &tot);
    if (tot > 0) {
      if (!scanned) {
        if (threadIdx.x == 0) bcast = atomicAdd(counter, tot);
        __syncthreads();
        base = bcast;
      }
      int64_t p = base + pre;
      auto emit = [&](float val, int64_t i) {
        if (p < cap) {
          out_val[p] = val;
          out_idx[p] = (int32_t)i;
          if (vmask != nullptr) vmask[i] = 0.f;
          if (umask != nullptr) umask[i] = 0.f;
        }
        ++p;
      };
#pragma unroll
      for (int j = 0; j < kV; ++j) {
        const uint32_t tj = (take >> (4 * j)) & 15u;
        if (tj) {
          const int64_t i = tb + 4 * ((int64_t)j * kBlock + threadIdx.x);
          if (tj & 1u) emit(v[j].x, i);
          if (tj & 2u) emit(v[j].y, i + 1);
          if (tj & 4u) emit(v[j].z, i + 2);
          if (tj & 8u) emit(v[j].w, i + 3);
        }
      }
      if (ie >= 0) emit(xe, ie);
      if (scanned) base += tot;
    }
    first = false;
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
                int first, int64_t n, int32_t* ccnt, int32_t* fnode, bool init, hipStream_t stream) {
  const int g = (n_seg + 255) / 256;
  if (init) dgc_init_kernel<<<g, 256, 0, stream>>>(n_seg, st, thr, count, done, fnode);
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
      dgc_count_tree_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, done, count, u, v, momentum, first,
                                                                      ccnt);
    else
      dgc_count_tree_kernel<false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, fuse ? v : x, thr, done, count, nullptr,
                                                                       nullptr, 0.f, 0, ccnt);
    dgc_adjust_tree_kernel<<<g, 256, 0, stream>>>(n_seg, target, thr, count, done, max_iters, fnode);
  }
}

void dgc_select_init(int n_seg, const float* samples, const int64_t* samp_off, const int32_t* kseg, TopkState* st,
                     float* thr, int32_t* count, int32_t* done, int32_t* fnode, hipStream_t stream) {
  if (n_seg <= 0) return;
  dgc_select_init_kernel<<<n_seg, kSelBlock, 0, stream>>>(samples, samp_off, kseg, st, thr, count, done, fnode);
}

void dgc_compact(const ChunkTable& ct, const float* x, const float* thr, float* out_val, int32_t* out_idx,
                 int64_t cap, int32_t* counter, float* vmask, float* umask, const int32_t* ccnt,
                 const int32_t* fnode, int32_t* coff, hipStream_t stream, int header_bytes) {
  dgc_scan_kernel<<<1, kScanBlock, 0, stream>>>(ct.seg, ct.n_chunks, ccnt, fnode, coff, counter, header_bytes / 4);
  if (ct.n_chunks == 0) return;
  dgc_compact_kernel<<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, thr, out_val, out_idx, cap, counter, vmask, umask,
                                                         fnode, coff);
}

void dgc_compensate(const float* g, float* u, float* v, float momentum, int64_t n, bool first, hipStream_t stream) {
  if (n <= 0) return;
  dgc_compensate_kernel<<<grid_for((n + 3) / 4), kBlock, 0, stream>>>(g, u, v, momentum, n, first ? 1 : 0);
}

}  // namespace grace
