// Segmented exact multi-rank selection (order statistics) for the Sketch codec on CDNA4 (gfx950).
//
// SketchCompressor needs, per parameter tensor ("segment"), the q+1 linear-interpolation quantile
// edges of its values (reference: /root/reference/grace_dl/tensorflow/compressor/sketch.py:22,
// tfp.stats.quantiles(x, q, interpolation='linear')): edge_j = a_j (1 - w_j) + b_j w_j with a_j, b_j
// the values of rank floor / ceil of j (n-1)/q in ascending order.  Sorting the bucket for that
// (torch.sort of 64-bit (segment, key) pairs) moved 25M elements at 27 GB/s.  This file selects
// the <= 2(q+1) order statistics of every segment directly, with a 4-digit MSD radix select over
// the order-preserving 32-bit key (digits 11 / 7 / 7 / 7 bits):
//
//   qsel_hist0         one pass, 16-B loads, interleaved LDS sub-histograms of digit 0
//   qsel_select<0>     one workgroup / segment: scan of the 2048 bins, every target rank's bin and
//                      residual rank; targets with the same prefix share a SLOT (ranks are sorted,
//                      so equal prefixes are adjacent); the histogram is left zeroed
//   qsel_hist<D>       D = 1..3: one pass, the element's known prefix is looked up among the
//                      segment's slots (open-addressing LDS hash table) and digit D is
//                      counted in that slot's 128-bin LDS histogram (only elements sharing a
//                      target's prefix count)
//   qsel_select<D>     per slot: wave scan of its 128 bins; targets refine prefix and rank; the
//                      last digit resolves the full key = the exact value, and the same kernel
//                      emits the interpolated edges (unfused mul/add: torch's rounding)
//
// Traffic: four reads of the bucket (no writes) instead of a sort's ~8 read+write passes of
// 12-byte records; every launch is graph-capturable (no host reads, fixed-size workspaces).
#include "grace_common.h"
#include "grace_kernels.h"
#include "grace_scan.h"

namespace grace {
namespace {

constexpr int kSelBlock = 256;  // select kernels: one thread per target rank
constexpr int kHBlock = 512;    // histogram passes
constexpr int kHCopies = 4;     // interleaved digit-0 sub-histograms (same-bin lanes -> distinct words)

template <int D>
struct QDigit;
template <>
struct QDigit<0> {
  static constexpr int shift = 21, bits = 11;
};
template <>
struct QDigit<1> {
  static constexpr int shift = 14, bits = 7;
};
template <>
struct QDigit<2> {
  static constexpr int shift = 7, bits = 7;
};
template <>
struct QDigit<3> {
  static constexpr int shift = 0, bits = 7;
};

// ascending order-preserving key of a float (negative values: all bits flipped)
__device__ __forceinline__ uint32_t ord_key(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_value(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// first index >= b whose address is 16-B aligned (clamped to e): scalar head, float4 body
__device__ __forceinline__ int64_t aligned_begin(const float* x, int64_t b, int64_t e) {
  const int64_t mis = (int64_t)((reinterpret_cast<uintptr_t>(x) >> 2) & 3);
  const int64_t a = b + ((4 - ((b + mis) & 3)) & 3);
  return a < e ? a : e;
}

__global__ __launch_bounds__(kHBlock) void qsel_hist0_kernel(ChunkTable ct, const float* __restrict__ x,
                                                             int32_t* __restrict__ h0) {
  __shared__ __align__(16) int32_t lh[2048 * kHCopies];
  for (int i = threadIdx.x; i < 2048 * kHCopies / 4; i += kHBlock)
    reinterpret_cast<int4*>(lh)[i] = make_int4(0, 0, 0, 0);
  __syncthreads();
  const int sub = threadIdx.x % kHCopies;
  const int seg = ct.seg[blockIdx.x];
  const int64_t b = ct.begin[blockIdx.x], e = ct.end[blockIdx.x];
  const int64_t a0 = aligned_begin(x, b, e);
  const int64_t a1 = a0 + ((e - a0) & ~(int64_t)3);
  for (int64_t i = b + threadIdx.x; i < a0; i += kHBlock) atomicAdd(&lh[(ord_key(x[i]) >> 21) * kHCopies + sub], 1);
  for (int64_t i = a1 + threadIdx.x; i < e; i += kHBlock) atomicAdd(&lh[(ord_key(x[i]) >> 21) * kHCopies + sub], 1);
  const float4* x4 = reinterpret_cast<const float4*>(x + a0);
  const int64_t nv = (a1 - a0) >> 2;
  for (int64_t v = threadIdx.x; v < nv; v += 2 * kHBlock) {
    const float4 p = x4[v];
    const bool two = v + kHBlock < nv;
    const float4 q = two ? x4[v + kHBlock] : make_float4(0.f, 0.f, 0.f, 0.f);
    atomicAdd(&lh[(ord_key(p.x) >> 21) * kHCopies + sub], 1);
    atomicAdd(&lh[(ord_key(p.y) >> 21) * kHCopies + sub], 1);
    atomicAdd(&lh[(ord_key(p.z) >> 21) * kHCopies + sub], 1);
    atomicAdd(&lh[(ord_key(p.w) >> 21) * kHCopies + sub], 1);
    if (two) {
      atomicAdd(&lh[(ord_key(q.x) >> 21) * kHCopies + sub], 1);
      atomicAdd(&lh[(ord_key(q.y) >> 21) * kHCopies + sub], 1);
      atomicAdd(&lh[(ord_key(q.z) >> 21) * kHCopies + sub], 1);
      atomicAdd(&lh[(ord_key(q.w) >> 21) * kHCopies + sub], 1);
    }
  }
  __syncthreads();
  int32_t* gh = h0 + (int64_t)seg * 2048;
  for (int i = threadIdx.x; i < 2048; i += kHBlock) {
    const int4 c = reinterpret_cast<const int4*>(lh)[i];
    const int32_t n = c.x + c.y + c.z + c.w;
    if (n) atomicAdd(&gh[i], n);
  }
}

// Count digit D of every element whose known (32 - shift - bits)-bit prefix is one of the
// segment's slot prefixes.  Slots are found through an open-addressing LDS hash table (1024
// entries for <= 256 slots: load <= 1/4, ~1 probe), so the common miss costs a hash, one LDS read
// and one compare.  Dynamic LDS: [max_slots] prefixes + [max_slots][64] words of two packed 16-bit
// bin counts (a chunk holds < 65536 elements -- sketch.py clamps GRACE_QSEL_CHUNK -- so a
// half-word never carries into its neighbour):
// ~38 KB for q = 64, four 512-thread workgroups per CU -- with 32-bit counts and a 4096-entry
// table it was 83 KB, one workgroup (8 waves) per CU, and the passes were latency bound.
constexpr int kHash = 1024;
__device__ __forceinline__ uint32_t qhash(uint32_t p) { return (p * 0x9E3779B1u) >> 22; }

template <int D>
__global__ __launch_bounds__(kHBlock) void qsel_hist_kernel(ChunkTable ct, const float* __restrict__ x, int max_slots,
                                                            const uint32_t* __restrict__ uniq,
                                                            const int32_t* __restrict__ nuniq,
                                                            int32_t* __restrict__ h) {
  constexpr int shift = QDigit<D>::shift;
  constexpr int hi = shift + QDigit<D>::bits;  // the known prefix is key >> hi
  extern __shared__ __align__(16) uint32_t dyn[];
  __shared__ int32_t tab[kHash];  // slot + 1, 0 = empty
  uint32_t* up = dyn;
  uint32_t* lh = dyn + max_slots;  // [slot][64] packed 16-bit pairs
  const int seg = ct.seg[blockIdx.x];
  const int nu = nuniq[seg];
  if (nu == 0) return;  // block-uniform
  const uint32_t* su = uniq + (int64_t)seg * max_slots;
  for (int i = threadIdx.x; i < kHash; i += kHBlock) tab[i] = 0;
  for (int i = threadIdx.x; i < nu * 64; i += kHBlock) lh[i] = 0u;
  __syncthreads();
  for (int sl = threadIdx.x; sl < nu; sl += kHBlock) {
    const uint32_t p = su[sl];
    up[sl] = p;
    uint32_t idx = qhash(p);
    while (atomicCAS(&tab[idx], 0, sl + 1) != 0) idx = (idx + 1) & (kHash - 1);
  }
  __syncthreads();
  const int64_t b = ct.begin[blockIdx.x], e = ct.end[blockIdx.x];
  auto count = [&](float v) {
    const uint32_t k = ord_key(v);
    const uint32_t p = k >> hi;
    uint32_t idx = qhash(p);
    int32_t ent = tab[idx];
    while (ent != 0) {
      if (up[ent - 1] == p) {
        const uint32_t d = (k >> shift) & 127;
        atomicAdd(&lh[(ent - 1) * 64 + (d >> 1)], 1u << ((d & 1) << 4));
        return;
      }
      idx = (idx + 1) & (kHash - 1);
      ent = tab[idx];
    }
  };
  const int64_t a0 = aligned_begin(x, b, e);
  const int64_t a1 = a0 + ((e - a0) & ~(int64_t)3);
  for (int64_t i = b + threadIdx.x; i < a0; i += kHBlock) count(x[i]);
  for (int64_t i = a1 + threadIdx.x; i < e; i += kHBlock) count(x[i]);
  const float4* x4 = reinterpret_cast<const float4*>(x + a0);
  const int64_t nv = (a1 - a0) >> 2;
  constexpr int U = 8;  // 8 x 16 B in flight per thread before the (LDS-bound) counting
  for (int64_t v0 = threadIdx.x; v0 < nv; v0 += (int64_t)U * kHBlock) {
    float4 xs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + (int64_t)u * kHBlock;
      xs[u] = v < nv ? x4[v] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v0 + (int64_t)u * kHBlock >= nv) break;
      count(xs[u].x);
      count(xs[u].y);
      count(xs[u].z);
      count(xs[u].w);
    }
  }
  __syncthreads();
  int32_t* gh = h + (int64_t)seg * max_slots * 128;
  for (int i = threadIdx.x; i < nu * 64; i += kHBlock) {
    const uint32_t n = lh[i];
    if (n & 0xffffu) atomicAdd(&gh[2 * i], (int32_t)(n & 0xffffu));
    if (n >> 16) atomicAdd(&gh[2 * i + 1], (int32_t)(n >> 16));
  }
}

// One workgroup per segment, one thread per (sorted, unique) target rank.
//   st_pfx / st_rank : the target's known key prefix and its rank inside that prefix group
//   uniq / nuniq     : the distinct prefixes after this digit (the next pass's slots)
//   slot             : target -> slot
// D == 3 additionally writes the selected values and the interpolated edges.
template <int D>
__global__ __launch_bounds__(kSelBlock) void qsel_select_kernel(
    int max_slots, const int32_t* __restrict__ ranks, const int32_t* __restrict__ nrank, int32_t* __restrict__ h0,
    int32_t* __restrict__ h, uint32_t* __restrict__ st_pfx, int32_t* __restrict__ st_rank,
    int32_t* __restrict__ slot, uint32_t* __restrict__ uniq, int32_t* __restrict__ nuniq, int q,
    const int32_t* __restrict__ lo_idx, const int32_t* __restrict__ hi_idx, const float* __restrict__ w,
    float* __restrict__ edges) {
  constexpr int bits = QDigit<D>::bits;
  extern __shared__ __align__(16) int32_t cum[];  // D == 0: [2048]; else [nu][128]
  __shared__ int lds[kSelBlock / kWave];
  __shared__ uint32_t npfx[kSelBlock];
  __shared__ float vals[kSelBlock];
  const int seg = blockIdx.x;
  const int nr = nrank[seg];
  const int t = threadIdx.x;
  const int64_t tb = (int64_t)seg * max_slots;
  if constexpr (D == 0) {
    int32_t* gh = h0 + (int64_t)seg * 2048;
    constexpr int per = 2048 / kSelBlock;
    int32_t loc[per];
    int s = 0;
#pragma unroll
    for (int j = 0; j < per; ++j) {
      loc[j] = gh[t * per + j];
      gh[t * per + j] = 0;  // leave the histogram clean for the next call
      s += loc[j];
    }
    int tot = 0;
    int run = block_exclusive_scan<kSelBlock>(s, lds, &tot);
#pragma unroll
    for (int j = 0; j < per; ++j) {
      run += loc[j];
      cum[t * per + j] = run;  // inclusive
    }
    __syncthreads();
    if (t < nr) {
      const int32_t r = ranks[tb + t];
      int l = 0, u = 2047;  // first bin whose inclusive count exceeds r (a non-empty bin)
      while (l < u) {
        const int m = (l + u) >> 1;
        if (cum[m] > r)
          u = m;
        else
          l = m + 1;
      }
      npfx[t] = (uint32_t)l;
      st_rank[tb + t] = r - (l > 0 ? cum[l - 1] : 0);
    }
  } else {
    const int nu = nuniq[seg];
    int32_t* gh = h + tb * 128;
    // wave w scans slots w, w + 4, ...: two bins per lane (one 8-B load); the loads of B slots are
    // issued before any of them is used (one HBM round trip per B slots, not per slot: these
    // one-workgroup-per-segment kernels are latency bound)
    constexpr int NWv = kSelBlock / kWave, B = 4;
    const int l = lane_id();
    for (int s0 = wave_id(); s0 < nu; s0 += NWv * B) {
      int2 cc[B];
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int sl = s0 + k * NWv;
        cc[k] = sl < nu ? reinterpret_cast<const int2*>(gh + sl * 128)[l] : make_int2(0, 0);
      }
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const int sl = s0 + k * NWv;
        if (sl >= nu) break;  // wave-uniform
        reinterpret_cast<int2*>(gh + sl * 128)[l] = make_int2(0, 0);
        const int incl = wave_inclusive_scan(cc[k].x + cc[k].y);
        cum[sl * 128 + 2 * l] = incl - cc[k].y;  // inclusive counts
        cum[sl * 128 + 2 * l + 1] = incl;
      }
    }
    __syncthreads();
    if (t < nr) {
      const int s = slot[tb + t];
      const int32_t r = st_rank[tb + t];
      const int32_t* cs = cum + s * 128;
      int l = 0, u = 127;
      while (l < u) {
        const int m = (l + u) >> 1;
        if (cs[m] > r)
          u = m;
        else
          l = m + 1;
      }
      npfx[t] = (st_pfx[tb + t] << bits) | (uint32_t)l;
      st_rank[tb + t] = r - (l > 0 ? cs[l - 1] : 0);
    }
  }
  __syncthreads();
  if constexpr (D < 3) {
    // slots of the next digit: distinct prefixes (adjacent in rank order)
    const int first = (t < nr && (t == 0 || npfx[t] != npfx[t - 1])) ? 1 : 0;
    int nu = 0;
    const int pos = block_exclusive_scan<kSelBlock>(first, lds, &nu);
    if (t < nr) {
      st_pfx[tb + t] = npfx[t];
      if (first) uniq[tb + pos] = npfx[t];
      slot[tb + t] = pos + first - 1;  // inclusive count - 1
    }
    if (t == 0) nuniq[seg] = nu;
  } else {
    if (t < nr) vals[t] = key_value(npfx[t]);
    if (t == 0) nuniq[seg] = 0;
    __syncthreads();
    if (nr == 0) return;
    const int64_t eb = (int64_t)seg * (q + 1);
    for (int j = t; j <= q; j += kSelBlock) {
      const float a = vals[lo_idx[eb + j]], bv = vals[hi_idx[eb + j]], ww = w[eb + j];
      // torch: a * (1 - w) + b * w, three separately rounded ops
      edges[eb + j] = __fadd_rn(__fmul_rn(a, __fsub_rn(1.f, ww)), __fmul_rn(bv, ww));
    }
  }
}

}  // namespace

void quantile_select(const ChunkTable& ct, int n_seg, const float* x, int max_slots, const int32_t* ranks,
                     const int32_t* nrank, int32_t* h0, int32_t* h, uint32_t* st_pfx, int32_t* st_rank, int32_t* slot,
                     uint32_t* uniq, int32_t* nuniq, int q, const int32_t* lo_idx, const int32_t* hi_idx,
                     const float* w, float* edges, hipStream_t stream) {
  if (n_seg == 0) return;
  static bool lds_attr = false;  // > 64 KB of dynamic LDS has to be opted into per kernel
  if (!lds_attr) {
    const int mx = 150 * 1024;
    const int mxh = 140 * 1024;  // + 4 KB static hash table <= 160 KB; max_slots <= 256 needs 66 KB
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)qsel_hist_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, mxh));
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)qsel_hist_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, mxh));
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)qsel_hist_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, mxh));
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)qsel_select_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)qsel_select_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)qsel_select_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    lds_attr = true;
  }
  const size_t hist_lds = (size_t)max_slots * (sizeof(uint32_t) + 64 * sizeof(uint32_t));
  const size_t cum_lds = (size_t)max_slots * 128 * sizeof(int32_t);
  if (ct.n_chunks > 0) qsel_hist0_kernel<<<ct.n_chunks, kHBlock, 0, stream>>>(ct, x, h0);
  qsel_select_kernel<0><<<n_seg, kSelBlock, 2048 * sizeof(int32_t), stream>>>(
      max_slots, ranks, nrank, h0, h, st_pfx, st_rank, slot, uniq, nuniq, q, lo_idx, hi_idx, w, edges);
  if (ct.n_chunks > 0)
    qsel_hist_kernel<1><<<ct.n_chunks, kHBlock, hist_lds, stream>>>(ct, x, max_slots, uniq, nuniq, h);
  qsel_select_kernel<1><<<n_seg, kSelBlock, cum_lds, stream>>>(max_slots, ranks, nrank, h0, h, st_pfx, st_rank, slot,
                                                              uniq, nuniq, q, lo_idx, hi_idx, w, edges);
  if (ct.n_chunks > 0)
    qsel_hist_kernel<2><<<ct.n_chunks, kHBlock, hist_lds, stream>>>(ct, x, max_slots, uniq, nuniq, h);
  qsel_select_kernel<2><<<n_seg, kSelBlock, cum_lds, stream>>>(max_slots, ranks, nrank, h0, h, st_pfx, st_rank, slot,
                                                              uniq, nuniq, q, lo_idx, hi_idx, w, edges);
  if (ct.n_chunks > 0)
    qsel_hist_kernel<3><<<ct.n_chunks, kHBlock, hist_lds, stream>>>(ct, x, max_slots, uniq, nuniq, h);
  qsel_select_kernel<3><<<n_seg, kSelBlock, cum_lds, stream>>>(max_slots, ranks, nrank, h0, h, st_pfx, st_rank, slot,
                                                              uniq, nuniq, q, lo_idx, hi_idx, w, edges);
}

}  // namespace grace
