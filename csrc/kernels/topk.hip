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

// Finds the digit value of the k-th largest key among the keys matching the current prefix,
// one workgroup per segment (all threads enter).  Bins are scanned in DESCENDING order.
// `ctr` (optional): the segment's counters of the two-pass pipeline -- [n_seg] definite takes
// (written by digit 0), [n_seg] candidate emission counter (set to the above-digit-1 count by
// digit 1), [n_seg] tie counter (zeroed by digit 0): no memset node is needed.
template <int D>
__device__ __forceinline__ void select_digit(int n_seg, int seg, const int32_t* __restrict__ kseg,
                                             TopkState* __restrict__ st, int32_t* __restrict__ hist,
                                             int32_t* __restrict__ ctr) {
  constexpr int shift = Digit<D>::shift;
  constexpr int bits = Digit<D>::bits;
  constexpr int nbins = 1 << bits;
  constexpr int per = nbins / kBlock;  // bins per thread (8 or 2)
  __shared__ int32_t part[kBlock / kWave];
  if (D == 0 && ctr != nullptr && threadIdx.x == 2) ctr[2 * n_seg + seg] = 0;
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
  int tot_unused = 0;
  const int32_t excl = block_exclusive_scan<kBlock>(s, part, &tot_unused);  // wave shuffles + 1 LDS round
  const int32_t incl = excl + s;
  if (excl < krem && krem <= incl) {
    int32_t run = excl;
#pragma unroll
    for (int q = 0; q < per; ++q) {
      if (run + loc[q] >= krem) {
        const uint32_t bin = nbins - 1 - (threadIdx.x * per + q);
        const uint32_t pfx = (D == 0 ? 0u : st[seg].prefix) | (bin << shift);
        st[seg].prefix = pfx;
        st[seg].krem = krem - run;  // how many to take from this bin (and below digits)
        if (D == 0 && ctr != nullptr) ctr[seg] = run;  // keys above the bin: the definite takes
        // candidates above the digit-1 bin: their slots are assigned by prefix sums, the
        // emission counter of the remaining candidates starts after them
        if (D == 1 && ctr != nullptr) ctr[n_seg + seg] = run;
        break;
      }
      run += loc[q];
    }
  }
}

template <int D>
__global__ __launch_bounds__(kBlock) void topk_select_kernel(int n_seg, const int32_t* __restrict__ kseg,
                                                             TopkState* __restrict__ st,
                                                             int32_t* __restrict__ hist,
                                                             int32_t* __restrict__ ctr = nullptr) {
  if ((int)blockIdx.x >= n_seg) return;
  select_digit<D>(n_seg, blockIdx.x, kseg, st, hist, ctr);
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

// ================================================================ two-pass Top-K (the compressor path)
// The three-digit radix select above re-reads the whole bucket for digits 1 and 2 only to count
// the few keys that share the threshold's prefix.  The Top-K compressor instead runs:
//   pass A  topk2_hist     : x = beta*r + gamma*g (stored in place of r), 16-B loads, LDS
//                            histogram of key bits 30..20 (digit 0)              reads 2n, writes n
//   select 0               : the digit-0 bin b0 of the k-th largest key (one workgroup / segment)
//   pass B  topk2_split    : reads x once: key>>20 > b0 -> definite take; key>>20 == b0 ->
//                            CANDIDATE; both staged in LDS and written to the chunk's slice of the
//                            candidate buffers (no atomics), digit-1 LDS histogram of the
//                            candidates; select 1                                         reads n
//   topk2_cand_hist        : digit-2 histogram of the candidates sharing the 22-bit prefix;
//                            select 2 (the exact k-th key T and its tie count)
//   topk2_assemble         : payload = definites + candidates above the prefix at deterministic
//                            slots (prefix sums over chunks) + the few prefix-sharing ones > T and
//                            the first ties; the emitted entries of x are zeroed (residual update)
// Candidates are ~0.5-1 % of n for gradient data, and the candidate slices are sized like the
// chunks, so any distribution fits (no overflow path).  (Running each select in the last
// workgroup of the preceding kernel through an arrival counter was measured: the per-workgroup
// drain + arrival round trip cost as much as the three stand-alone launches it removed.)

struct Vec4Range {  // the 16-B vectors overlapping [b, e): first/last vector index
  int64_t v0, v1;
};
__device__ __forceinline__ Vec4Range vec_range(int64_t b, int64_t e) { return {b >> 2, (e + 3) >> 2}; }

// 4 elements of vector v, lanes outside [b, e) or past `total` masked (valid bits 0..3); the last
// vector of a buffer whose size is not a multiple of 4 is loaded element-wise (no over-read)
__device__ __forceinline__ float4 ld4m(const float* p, int64_t v, int64_t b, int64_t e, int64_t total,
                                       uint32_t* valid) {
  const int64_t i0 = v << 2;
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) m |= (i0 + j >= b && i0 + j < e ? 1u : 0u) << j;
  *valid = m;
  if (i0 + 4 <= total) return *reinterpret_cast<const float4*>(p + i0);
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i0 < total) r.x = p[i0];
  if (i0 + 1 < total) r.y = p[i0 + 1];
  if (i0 + 2 < total) r.z = p[i0 + 2];
  return r;
}

__device__ __forceinline__ float f4(const float4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }

constexpr int kVU = 4;      // vectors in flight per thread in pass A
constexpr int kHCopies = 4;  // interleaved LDS sub-histograms in pass A

// mode 0: x = g (x != g: copied, the residual starts as g); mode 1: x = beta*x + gamma*g
__global__ __launch_bounds__(kBlock) void topk2_hist_kernel(ChunkTable ct, const float* __restrict__ g, float* x,
                                                            int64_t total, float beta, float gamma, int mode,
                                                            int32_t* __restrict__ hist) {
  // kHCopies interleaved sub-histograms (word = bin * kHCopies + lane % kHCopies): lanes of a wave
  // that hit the same bin hit different words, so same-address LDS atomics serialise less
  // (gradient keys concentrate in a few dozen digit-0 bins)
  __shared__ __align__(16) int32_t lh[2048 * kHCopies];
  for (int i = threadIdx.x; i < 2048 * kHCopies / 4; i += kBlock)
    reinterpret_cast<int4*>(lh)[i] = make_int4(0, 0, 0, 0);
  __syncthreads();
  const int sub = threadIdx.x % kHCopies;
  const int seg = ct.seg[blockIdx.x];
  const int64_t b = ct.begin[blockIdx.x], e = ct.end[blockIdx.x];
  const Vec4Range vr = vec_range(b, e);
  const bool store = x != g;
  for (int64_t v = vr.v0 + threadIdx.x; v < vr.v1; v += kBlock * kVU) {
    float4 xv[kVU];
    uint32_t ok[kVU];
#pragma unroll
    for (int u = 0; u < kVU; ++u) {
      const int64_t vv = v + (int64_t)u * kBlock;
      ok[u] = 0;
      xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (vv < vr.v1) {
        xv[u] = ld4m(g, vv, b, e, total, &ok[u]);
        if (mode == 1) {
          uint32_t o2;
          const float4 rv = ld4m(x, vv, b, e, total, &o2);
          xv[u] = make_float4(fmaf(beta, rv.x, gamma * xv[u].x), fmaf(beta, rv.y, gamma * xv[u].y),
                              fmaf(beta, rv.z, gamma * xv[u].z), fmaf(beta, rv.w, gamma * xv[u].w));
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kVU; ++u) {
      if (!ok[u]) continue;
      const int64_t i0 = (v + (int64_t)u * kBlock) << 2;
      if (store) {
        if (ok[u] == 0xfu) {
          *reinterpret_cast<float4*>(x + i0) = xv[u];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if ((ok[u] >> j) & 1u) x[i0 + j] = f4(xv[u], j);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((ok[u] >> j) & 1u) atomicAdd(&lh[(abs_key(f4(xv[u], j)) >> 20) * kHCopies + sub], 1);
    }
  }
  __syncthreads();
  int32_t* gh = hist + (int64_t)seg * kHistStride;
  for (int i = threadIdx.x; i < 2048; i += kBlock) {
    const int4 q = reinterpret_cast<const int4*>(lh)[i];  // kHCopies == 4
    const int32_t cnt = q.x + q.y + q.z + q.w;
    if (cnt) atomicAdd(&gh[i], cnt);
  }
}

constexpr int kSV = 8;        // vectors per thread per tile in pass B (8192 elements per tile)
constexpr int kStage = 1024;  // LDS staging entries per tile (typical tile: ~1.75 % of 8192)

// Pass B: classify against the digit-0 bin b0 of the segment.  No global atomics: each chunk
// owns the slice [begin, end) of the candidate buffers and writes its definite takes from the
// front and its candidates from the back (a chunk's takes + candidates <= its size), then
// publishes the two counts; the assemble kernel places the takes into the payload and zeroes
// them in x.  Takes and candidates are staged in LDS and stored with full-wave coalesced writes,
// the candidates' digit-1 histogram is an LDS histogram flushed once per block (sparse per-lane
// global stores/atomics issue one wave-instruction per element slot: measured 3x slower).
__global__ __launch_bounds__(kBlock) void topk2_split_kernel(ChunkTable ct, const float* __restrict__ x, int64_t total,
                                                             const TopkState* __restrict__ st,
                                                             int32_t* __restrict__ ccnt, float* __restrict__ cand_val,
                                                             int32_t* __restrict__ cand_idx,
                                                             int32_t* __restrict__ hist) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int32_t lh[2048];
  __shared__ float sv[kStage];
  __shared__ int32_t si[kStage];
  for (int i = threadIdx.x; i < 2048; i += kBlock) lh[i] = 0;
  const int c = blockIdx.x;
  const int seg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const Vec4Range vr = vec_range(b, e);
  const uint32_t b0 = st[seg].prefix >> 20;
  int run_take = 0, run_cand = 0;  // block-uniform
  for (int64_t tv = vr.v0; tv < vr.v1; tv += kBlock * kSV) {
    float4 xv[kSV];
    uint32_t ok[kSV];
#pragma unroll
    for (int u = 0; u < kSV; ++u) {
      const int64_t vv = tv + (int64_t)u * kBlock + threadIdx.x;
      ok[u] = 0;
      xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (vv < vr.v1) xv[u] = ld4m(x, vv, b, e, total, &ok[u]);
    }
    uint32_t take = 0, cand = 0;  // bit 4u+j
#pragma unroll
    for (int u = 0; u < kSV; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t d = abs_key(f4(xv[u], j)) >> 20;
        const uint32_t okj = (ok[u] >> j) & 1u;
        take |= (okj & (d > b0 ? 1u : 0u)) << (4 * u + j);
        cand |= (okj & (d == b0 ? 1u : 0u)) << (4 * u + j);
      }
    int tot = 0;
    const int nt = __popc(take);
    const int packed = nt | (__popc(cand) << 16);
    const int pre = block_exclusive_scan<kBlock>(packed, lds, &tot);
    if (tot == 0) continue;  // block-uniform
    const int tt = tot & 0xffff, tc = tot >> 16;
    if (tt + tc <= kStage) {
      // LDS image: takes [0, tt), candidates [tt, tt + tc)
      int p = pre & 0xffff, q = tt + (pre >> 16);
#pragma unroll
      for (int u = 0; u < kSV; ++u) {
        const int32_t i0 = (int32_t)((tv + (int64_t)u * kBlock + threadIdx.x) << 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int bit = 4 * u + j;
          const float val = f4(xv[u], j);
          if ((take >> bit) & 1u) {
            sv[p] = val;
            si[p] = i0 + j;
            ++p;
          } else if ((cand >> bit) & 1u) {
            sv[q] = val;
            si[q] = i0 + j;
            ++q;
            atomicAdd(&lh[(abs_key(val) >> 9) & 2047], 1);
          }
        }
      }
      __syncthreads();
      for (int i = threadIdx.x; i < tt; i += kBlock) {
        cand_val[b + run_take + i] = sv[i];
        cand_idx[b + run_take + i] = si[i];
      }
      for (int i = threadIdx.x; i < tc; i += kBlock) {  // candidates grow down from the chunk end
        cand_val[e - 1 - (run_cand + i)] = sv[tt + i];
        cand_idx[e - 1 - (run_cand + i)] = si[tt + i];
      }
      __syncthreads();  // staging reuse by the next tile
    } else {  // dense tile: direct stores
      int64_t p = b + run_take + (pre & 0xffff);
      int64_t q = e - 1 - (run_cand + (pre >> 16));
#pragma unroll
      for (int u = 0; u < kSV; ++u) {
        const int32_t i0 = (int32_t)((tv + (int64_t)u * kBlock + threadIdx.x) << 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int bit = 4 * u + j;
          const float val = f4(xv[u], j);
          if ((take >> bit) & 1u) {
            cand_val[p] = val;
            cand_idx[p] = i0 + j;
            ++p;
          } else if ((cand >> bit) & 1u) {
            cand_val[q] = val;
            cand_idx[q] = i0 + j;
            --q;
            atomicAdd(&lh[(abs_key(val) >> 9) & 2047], 1);
          }
        }
      }
    }
    run_take += tt;
    run_cand += tc;
  }
  __syncthreads();
  if (run_cand > 0) {
    int32_t* gh = hist + (int64_t)seg * kHistStride;
    for (int i = threadIdx.x; i < 2048; i += kBlock) {
      const int32_t n = lh[i];
      if (n) atomicAdd(&gh[i], n);
    }
  }
  if (threadIdx.x == 0) {
    ccnt[c] = run_take;
    ccnt[ct.n_chunks + c] = run_cand;
  }
}

// Digit-2 histogram of the chunk's candidates that match the 22-bit prefix, and the count of the
// chunk's candidates ABOVE the prefix (all taken; ccnt[2 * n_chunks + c]).  One block per chunk.
__global__ __launch_bounds__(kBlock) void topk2_cand_hist_kernel(ChunkTable ct, const TopkState* __restrict__ st,
                                                                 int32_t* __restrict__ ccnt,
                                                                 const float* __restrict__ cand_val,
                                                                 int32_t* __restrict__ hist) {
  __shared__ int red[kBlock / kWave];
  const int c = blockIdx.x;
  const int32_t nc = ccnt[ct.n_chunks + c];
  const int seg = ct.seg[c];
  if (nc > 0) {  // block-uniform
    const int64_t e = ct.end[c];
    const uint32_t P = st[seg].prefix >> 9;
    int32_t* gh = hist + (int64_t)seg * kHistStride;
    int above = 0;
    for (int i = threadIdx.x; i < nc; i += kBlock) {
      const uint32_t key = abs_key(cand_val[e - 1 - i]);
      if ((key >> 9) == P) atomicAdd(&gh[key & 511], 1);
      above += (key >> 9) > P ? 1 : 0;
    }
    int tot = 0;
    (void)block_exclusive_scan<kBlock>(above, red, &tot);
    if (threadIdx.x == 0) ccnt[2 * ct.n_chunks + c] = tot;
  } else if (threadIdx.x == 0) {
    ccnt[2 * ct.n_chunks + c] = 0;
  }
}

// Final placement, one block per chunk.  Payload order per segment: definite takes, then the
// candidates above the 22-bit prefix ("above-1"), both at deterministic slots (prefix sums over
// the segment's earlier chunks); then the few candidates sharing the prefix that are > T, plus
// the first `ties` keys == T, through one atomic per 256 such candidates.  Emitted entries are
// zeroed in x (the residual).  Every payload store is bounds-checked against the segment's k.
__global__ __launch_bounds__(kBlock) void topk2_assemble_kernel(ChunkTable ct, const int32_t* __restrict__ seg_chunk_begin,
                                                                int n_seg, const int32_t* __restrict__ kseg,
                                                                const TopkState* __restrict__ st,
                                                                const int64_t* __restrict__ out_off,
                                                                int32_t* __restrict__ ctr,
                                                                const int32_t* __restrict__ ccnt,
                                                                const float* __restrict__ cand_val,
                                                                const int32_t* __restrict__ cand_idx,
                                                                float* __restrict__ out_val,
                                                                int32_t* __restrict__ out_idx, float* x, int zero) {
  __shared__ int lds[kBlock / kWave];
  __shared__ int bcast[2];
  const int c = blockIdx.x;
  const int N = ct.n_chunks;
  const int32_t ntake = ccnt[c], nc = ccnt[N + c];
  if (ntake == 0 && nc == 0) return;  // block-uniform
  const int seg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const int64_t obase = out_off[seg];
  const int64_t olim = obase + kseg[seg];
  const int64_t dbase = obase + ctr[seg];  // after the segment's definites
  // prefix over the segment's earlier chunks: takes (low 32 bits) and above-1 candidates
  int pt = 0, pa = 0;
  for (int cc = seg_chunk_begin[seg] + threadIdx.x; cc < c; cc += kBlock) {
    pt += ccnt[cc];
    pa += ccnt[2 * N + cc];
  }
  int pre_take = 0, pre_a1 = 0;
  (void)block_exclusive_scan<kBlock>(pt, lds, &pre_take);
  (void)block_exclusive_scan<kBlock>(pa, lds, &pre_a1);
  for (int i = threadIdx.x; i < ntake; i += kBlock) {
    const int64_t p = obase + pre_take + i;
    const int32_t ix = cand_idx[b + i];
    if (p < olim) {
      out_val[p] = cand_val[b + i];
      out_idx[p] = ix;
    }
    if (zero) x[ix] = 0.f;
  }
  if (nc == 0) return;
  const uint32_t T = st[seg].prefix;
  const int32_t ties = st[seg].krem;
  int run_a1 = 0;
  for (int i0 = 0; i0 < nc; i0 += kBlock) {
    const int i = i0 + threadIdx.x;
    float v = 0.f;
    int32_t ix = 0;
    uint32_t key = 0;
    const bool in = i < nc;
    if (in) {
      v = cand_val[e - 1 - i];
      ix = cand_idx[e - 1 - i];
      key = abs_key(v);
    }
    const int a1 = (in && (key >> 9) > (T >> 9)) ? 1 : 0;
    const int m_above = (in && (key >> 9) == (T >> 9) && key > T) ? 1 : 0;
    const int tie = (in && key == T) ? 1 : 0;
    int tot = 0;
    const int pre = block_exclusive_scan<kBlock>(a1 | (m_above << 10) | (tie << 20), lds, &tot);
    if (a1) {
      const int64_t p = dbase + pre_a1 + run_a1 + (pre & 0x3ff);
      if (p < olim) {
        out_val[p] = v;
        out_idx[p] = ix;
      }
      if (zero) x[ix] = 0.f;
    }
    run_a1 += tot & 0x3ff;
    if ((tot >> 10) == 0) continue;  // no prefix-sharing candidate in this slice (block-uniform)
    if (threadIdx.x == 0) bcast[1] = (tot >> 20) ? atomicAdd(ctr + 2 * n_seg + seg, tot >> 20) : 0;
    __syncthreads();
    const int take = m_above | ((tie && bcast[1] + (pre >> 20) < ties) ? 1 : 0);
    int ttot = 0;
    const int tpre = block_exclusive_scan<kBlock>(take, lds, &ttot);
    if (threadIdx.x == 0) bcast[0] = ttot ? atomicAdd(ctr + n_seg + seg, ttot) : 0;
    __syncthreads();
    if (take) {
      const int64_t p = dbase + bcast[0] + tpre;
      if (p < olim) {
        out_val[p] = v;
        out_idx[p] = ix;
      }
      if (zero) x[ix] = 0.f;
    }
    __syncthreads();
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

// out[idx[j]] += val[j] * scale for j < min(*count, cap): the count lives in the payload's
// in-band header (capacity payloads of the variable-size codecs: no host read of the size)
__global__ __launch_bounds__(kBlock) void sparse_scatter_add_dev_kernel(const float* __restrict__ val,
                                                                        const int32_t* __restrict__ idx,
                                                                        const int32_t* __restrict__ count,
                                                                        int64_t cap, float* __restrict__ out,
                                                                        float scale, int accumulate,
                                                                        uint32_t* health) {
  const int64_t c = *count;
  const int64_t K = c < cap ? c : cap;
  // health == null: not this process's own payload (a peer's, or a memory's zeroing scatter) --
  // an overflow is counted once, by the decode of the sender's own payload
  if (health != nullptr && c > cap && blockIdx.x == 0 && threadIdx.x == 0) health_count_overflow(health);
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

void topk_ef_bucket(const ChunkTable& ct, const int32_t* seg_chunk_begin, int n_seg, const float* g, float* x,
                    int64_t total, float beta, float gamma, int mode, int zero, const int32_t* kseg, TopkState* st,
                    int32_t* hist, int32_t* ctr, int32_t* ccnt, const int64_t* out_off, float* out_val,
                    int32_t* out_idx, float* cand_val, int32_t* cand_idx, hipStream_t stream) {
  const dim3 grid(ct.n_chunks), block(kBlock);
  topk2_hist_kernel<<<grid, block, 0, stream>>>(ct, g, x, total, beta, gamma, mode, hist);
  topk_select_kernel<0><<<n_seg, kBlock, 0, stream>>>(n_seg, kseg, st, hist, ctr);
  topk2_split_kernel<<<grid, block, 0, stream>>>(ct, x, total, st, ccnt, cand_val, cand_idx, hist);
  topk_select_kernel<1><<<n_seg, kBlock, 0, stream>>>(n_seg, kseg, st, hist, ctr);
  topk2_cand_hist_kernel<<<grid, block, 0, stream>>>(ct, st, ccnt, cand_val, hist);
  topk_select_kernel<2><<<n_seg, kBlock, 0, stream>>>(n_seg, kseg, st, hist, ctr);
  topk2_assemble_kernel<<<grid, block, 0, stream>>>(ct, seg_chunk_begin, n_seg, kseg, st, out_off, ctr, ccnt,
                                                    cand_val, cand_idx, out_val, out_idx, x, zero);
}

void sparse_scatter_add(const float* val, const int32_t* idx, int64_t K, float* out, float scale,
                        bool accumulate, hipStream_t stream) {
  if (K <= 0) return;
  int64_t blocks = (K + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  sparse_scatter_add_kernel<<<(int)blocks, kBlock, 0, stream>>>(val, idx, K, out, scale, accumulate ? 1 : 0);
}

void sparse_scatter_add_dev(const float* val, const int32_t* idx, const int32_t* count, int64_t cap, float* out,
                            float scale, bool accumulate, hipStream_t stream, bool count_overflow) {
  if (cap <= 0) return;
  int64_t blocks = (cap + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  sparse_scatter_add_dev_kernel<<<(int)blocks, kBlock, 0, stream>>>(val, idx, count, cap, out, scale,
                                                                    accumulate ? 1 : 0,
                                                                    count_overflow ? health_words().host_dev : nullptr);
}

}  // namespace grace
