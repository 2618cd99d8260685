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

// first index >= b whose address is 16-B aligned for a float array (clamped to e)
__device__ __forceinline__ int64_t vec4_begin(const void* x, int64_t b, int64_t e) {
  const int64_t mis = (int64_t)((reinterpret_cast<uintptr_t>(x) >> 2) & 3);
  const int64_t a = b + ((4 - ((b + mis) & 3)) & 3);
  return a < e ? a : e;
}

__device__ __forceinline__ uint32_t sk_key(float v) {  // ascending order-preserving key
  const uint32_t u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// bins: uint8 (q <= 256) or uint16; edges: [n_seg][q+1].
// Bin = (#edges <= v) - 1 clamped to [0, q-1] (torch.searchsorted(right=True) - 1).  The edges
// are staged in LDS with a 2048-entry table over the top 11 bits of the order-preserving key:
// start[d] = #edges whose key is below bucket d, so an element only scans the few edges inside
// its own bucket (quantile edges spread over the value range: ~1-2 per populated bucket) -- a
// per-element binary search was 4x slower.  Bin codes are stored 4 per 4/8-B store.
//
// Bin sums in FIXED POINT with integer LDS atomics: an LDS fp32 atomic add (ds_add_f32) costs
// ~25x an integer one on gfx950 -- measured with tools/diag/sketch_encode_probe.py on ResNet-50's
// 25.5 M elements: 178 us with fp32 bin sums, 61 us without them, 171 us without the u32 counts.
// Every value of bin j lies between edges j and j+1, so |v| <= M_j = max(|e_j|, |e_j+1|) < 2^E_j;
// with 2^L >= the segment's size, v * 2^(62 - L - E_j) rounded to int64 sums over the whole
// segment without overflow, at a resolution of 2^-50 (or finer) of the bin's magnitude -- finer
// than an fp32 accumulation, and order-independent: the means are deterministic.  Per-wave LDS
// copies of the q sums (u64) and counts (u32), folded once per workgroup into one global integer
// atomic per bin.
//
// Means finisher: sums / counts / arrive are a persistent zeroed workspace; every workgroup adds
// its bin totals, then counts itself in arrive[seg]; the segment's last workgroup turns the totals
// into the bin means (0 for an empty bin) and re-zeroes the workspace for the next call -- no
// zero-fills and no elementwise mean kernels.  (Non-finite edges -- a gradient holding inf/NaN --
// give meaningless means, as any average of such a segment is.)
template <typename BinT>
__global__ __launch_bounds__(kBlock) void sketch_encode_kernel(ChunkTable ct, const float* __restrict__ x,
                                                               const float* __restrict__ edges, int q,
                                                               BinT* __restrict__ bins,
                                                               unsigned long long* __restrict__ sums,
                                                               uint32_t* __restrict__ counts, int32_t* __restrict__ arrive,
                                                               const int32_t* __restrict__ seg_chunk_begin,
                                                               float* __restrict__ means) {
  constexpr int NW = kBlock / kWave;
  __shared__ float le[kMaxQ + 2];
  __shared__ uint16_t start[2048];
  __shared__ int last;
  extern __shared__ __align__(16) unsigned long long sk_dyn[];
  unsigned long long* ls_all = sk_dyn;                                    // [NW][q] fixed-point sums
  double* scale = reinterpret_cast<double*>(sk_dyn + NW * q);            // [q] 2^(62 - L - E_j)
  uint32_t* lc_all = reinterpret_cast<uint32_t*>(sk_dyn + NW * q + q);   // [NW][q] counts
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const int c0 = seg_chunk_begin[sg], c1 = seg_chunk_begin[sg + 1];
  const int64_t nseg = ct.end[c1 - 1] - ct.begin[c0];
  const int L = nseg > 1 ? 64 - __clzll((unsigned long long)(nseg - 1)) : 0;  // 2^L >= nseg
  const float* E = edges + (int64_t)sg * (q + 1);
  for (int i = threadIdx.x; i <= q; i += kBlock) le[i] = E[i];
  if (threadIdx.x == 0) le[q + 1] = __int_as_float(0x7fc00000);  // NaN sentinel: `<= v` is false
  for (int i = threadIdx.x; i < NW * q; i += kBlock) {
    ls_all[i] = 0ull;
    lc_all[i] = 0u;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < q; j += kBlock) {
    const float m = fmaxf(fabsf(le[j]), fabsf(le[j + 1]));
    int ex = 0;
    if (m > 0.f && isfinite(m)) frexpf(m, &ex);  // m = f 2^ex, f in [0.5, 1): every |v| of bin j < 2^ex
    scale[j] = ldexp(1.0, 62 - L - ex);          // a power of two: exact in double
  }
  for (int d = threadIdx.x; d < 2048; d += kBlock) {  // lower bound of bucket d among the edge keys
    const uint32_t lo = (uint32_t)d << 21;
    int l = 0, r = q + 1;
    while (l < r) {
      const int m = (l + r) >> 1;
      if (sk_key(le[m]) < lo)
        l = m + 1;
      else
        r = m;
    }
    start[d] = (uint16_t)l;
  }
  __syncthreads();
  unsigned long long* wls = ls_all + wave_id() * q;
  uint32_t* wlc = lc_all + wave_id() * q;
  auto bin_of = [&](float v) {
    int cnt = start[sk_key(v) >> 21];
    while (le[cnt] <= v) ++cnt;  // stops at the NaN sentinel (index q + 1) at the latest
    const int bb = cnt - 1;
    return bb < 0 ? 0 : (bb > q - 1 ? q - 1 : bb);
  };
  auto add = [&](int bin, float v) {
    atomicAdd(&wls[bin], (unsigned long long)__double2ll_rn((double)v * scale[bin]));  // two's complement
    atomicAdd(&wlc[bin], 1u);
  };
  auto one = [&](int64_t i) {
    const float v = x[i];
    const int bin = bin_of(v);
    bins[i] = (BinT)bin;
    add(bin, v);
  };
  const int64_t a0 = vec4_begin(x, b, e);
  const int64_t a1 = a0 + ((e - a0) & ~(int64_t)3);
  for (int64_t i = b + threadIdx.x; i < a0; i += kBlock) one(i);
  for (int64_t i = a1 + threadIdx.x; i < e; i += kBlock) one(i);
  const bool vec_bins = ((reinterpret_cast<uintptr_t>(bins + a0)) % (4 * sizeof(BinT))) == 0;
  // 8 x 16 B in flight per thread before any use: one vector at a time left every wave waiting
  // on HBM latency with ~12 KB in flight per CU
  constexpr int U = 8;
  for (int64_t i0 = a0 + 4 * (int64_t)threadIdx.x; i0 < a1; i0 += 4 * kBlock * U) {
   float4 xs[U];
#pragma unroll
   for (int u = 0; u < U; ++u) {
     const int64_t i = i0 + (int64_t)u * 4 * kBlock;
     xs[u] = i < a1 ? *reinterpret_cast<const float4*>(x + i) : make_float4(0.f, 0.f, 0.f, 0.f);
   }
#pragma unroll
   for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + (int64_t)u * 4 * kBlock;
    if (i >= a1) break;
    const float4 v4 = xs[u];
    const float v[4] = {v4.x, v4.y, v4.z, v4.w};
    // the bucket-table reads and the first edge reads of the four elements are independent LDS
    // reads issued together; only the (short) scans past the first edge are per element
    int bn[4], cn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) cn[j] = start[sk_key(v[j]) >> 21];
    float fe[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fe[j] = le[cn[j]];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int cnt = cn[j];
      if (fe[j] <= v[j]) {
        ++cnt;
        while (le[cnt] <= v[j]) ++cnt;  // stops at the NaN sentinel (index q + 1) at the latest
      }
      const int bb = cnt - 1;
      bn[j] = bb < 0 ? 0 : (bb > q - 1 ? q - 1 : bb);
      add(bn[j], v[j]);
    }
    if (vec_bins) {
      if constexpr (sizeof(BinT) == 1) {
        *reinterpret_cast<uint32_t*>(bins + i) =
            (uint32_t)bn[0] | ((uint32_t)bn[1] << 8) | ((uint32_t)bn[2] << 16) | ((uint32_t)bn[3] << 24);
      } else {
        *reinterpret_cast<uint2*>(bins + i) = make_uint2((uint32_t)bn[0] | ((uint32_t)bn[1] << 16),
                                                         (uint32_t)bn[2] | ((uint32_t)bn[3] << 16));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) bins[i + j] = (BinT)bn[j];
    }
   }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < q; i += kBlock) {
    unsigned long long sv = 0ull;
    uint32_t cv = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      sv += ls_all[w * q + i];
      cv += lc_all[w * q + i];
    }
    if (cv != 0) {
      __hip_atomic_fetch_add(&sums[(int64_t)sg * q + i], sv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&counts[(int64_t)sg * q + i], cv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // hand-off without fences (cdna_hip_programming.md Guideline 16; as bnact.hip arrive()): every
  // wave drains its no-return atomics, barrier, ONE relaxed agent add; the last block reads the
  // totals with device-scope loads.  (A __threadfence() here is an L2 write-back per block -- it
  // flushed the bin codes and made this kernel 1.7x slower.)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&arrive[sg], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c1 - c0 - 1;
  __syncthreads();
  if (!last) return;
  for (int i = threadIdx.x; i < q; i += kBlock) {
    unsigned long long* sp = sums + (int64_t)sg * q + i;
    uint32_t* cp = counts + (int64_t)sg * q + i;
    const long long sv = (long long)__hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t cv = __hip_atomic_load(cp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    means[(int64_t)sg * q + i] = cv ? (float)((double)sv / scale[i] / (double)cv) : 0.f;
    __hip_atomic_store(sp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) __hip_atomic_store(&arrive[sg], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- q > 1024 (up to 65535 with uint16 bins, the reference's range: sketch.py:22-27) --------
// The per-wave LDS bin tables above do not fit (56 q bytes per workgroup), so the large-q encode
// keeps the bin accumulators in global memory: the same int64 fixed-point sums (order-independent,
// deterministic) and u32 counts, added per element with device-scope atomics, and the same
// last-workgroup means finisher.  The bin is found by torch.searchsorted's own upper-bound
// binary search over the whole edge row (start 0, end q + 1, mid = lo + (hi - lo) / 2, step right
// while !(edge > v)): interpolated quantile edges are NOT always monotone (a (1 - w) + b w with
// a == b can land one ulp off a), and only the identical probe sequence gives identical bins.
__device__ __forceinline__ double sk_scale(const float* E, int j, int L) {
  const float m = fmaxf(fabsf(E[j]), fabsf(E[j + 1]));
  int ex = 0;
  if (m > 0.f && isfinite(m)) frexpf(m, &ex);
  return ldexp(1.0, 62 - L - ex);
}

template <typename BinT>
__global__ __launch_bounds__(kBlock) void sketch_encode_big_kernel(ChunkTable ct, const float* __restrict__ x,
                                                                   const float* __restrict__ edges, int q,
                                                                   BinT* __restrict__ bins,
                                                                   unsigned long long* __restrict__ sums,
                                                                   uint32_t* __restrict__ counts,
                                                                   int32_t* __restrict__ arrive,
                                                                   const int32_t* __restrict__ seg_chunk_begin,
                                                                   float* __restrict__ means) {
  __shared__ int last;
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const int c0 = seg_chunk_begin[sg], c1 = seg_chunk_begin[sg + 1];
  const int64_t nseg = ct.end[c1 - 1] - ct.begin[c0];
  const int L = nseg > 1 ? 64 - __clzll((unsigned long long)(nseg - 1)) : 0;
  const float* E = edges + (int64_t)sg * (q + 1);
  unsigned long long* SU = sums + (int64_t)sg * q;
  uint32_t* CN = counts + (int64_t)sg * q;
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    const float v = x[i];
    int l = 0, r = q + 1;  // torch's cus_upper_bound, probe for probe
    while (l < r) {
      const int m = l + ((r - l) >> 1);
      if (!(E[m] > v))
        l = m + 1;
      else
        r = m;
    }
    const int bb = l - 1;
    const int bin = bb < 0 ? 0 : (bb > q - 1 ? q - 1 : bb);
    bins[i] = (BinT)bin;
    __hip_atomic_fetch_add(&SU[bin], (unsigned long long)__double2ll_rn((double)v * sk_scale(E, bin, L)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&CN[bin], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave drained its atomics (as above)
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&arrive[sg], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c1 - c0 - 1;
  __syncthreads();
  if (!last) return;
  for (int i = threadIdx.x; i < q; i += kBlock) {
    const long long sv = (long long)__hip_atomic_load(&SU[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t cv = __hip_atomic_load(&CN[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    means[(int64_t)sg * q + i] = cv ? (float)((double)sv / sk_scale(E, i, L) / (double)cv) : 0.f;
    __hip_atomic_store(&SU[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&CN[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) __hip_atomic_store(&arrive[sg], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename BinT>
__global__ __launch_bounds__(kBlock) void sketch_decode_kernel(ChunkTable ct, const uint8_t* __restrict__ base,
                                                               int64_t rank_stride, int64_t bins_off,
                                                               int64_t means_off, int q, int n_ranks, float scale,
                                                               float* __restrict__ out) {
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  auto one = [&](int64_t i) {
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) {
      const uint8_t* rb = base + (int64_t)r * rank_stride;
      const int bin = (int)reinterpret_cast<const BinT*>(rb + bins_off)[i];
      acc += reinterpret_cast<const float*>(rb + means_off)[(int64_t)sg * q + bin];
    }
    out[i] = acc * scale;
  };
  const bool vec = (reinterpret_cast<uintptr_t>(base + bins_off) % (4 * sizeof(BinT))) == 0 &&
                   (rank_stride % (4 * sizeof(BinT))) == 0;
  const int64_t a0 = vec ? vec4_begin(out, b, e) : e;
  const int64_t a1 = a0 + ((e - a0) & ~(int64_t)3);
  for (int64_t i = b + threadIdx.x; i < a0; i += kBlock) one(i);
  for (int64_t i = a1 + threadIdx.x; i < e; i += kBlock) one(i);
  for (int64_t i = a0 + 4 * (int64_t)threadIdx.x; i < a1; i += 4 * kBlock) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int r = 0; r < n_ranks; ++r) {
      const uint8_t* rb = base + (int64_t)r * rank_stride;
      const float* M = reinterpret_cast<const float*>(rb + means_off) + (int64_t)sg * q;
      uint32_t bn[4];
      if constexpr (sizeof(BinT) == 1) {
        const uint32_t u = *reinterpret_cast<const uint32_t*>(rb + bins_off + i);
        bn[0] = u & 0xff;
        bn[1] = (u >> 8) & 0xff;
        bn[2] = (u >> 16) & 0xff;
        bn[3] = u >> 24;
      } else {
        const uint2 u = *reinterpret_cast<const uint2*>(rb + bins_off + 2 * i);
        bn[0] = u.x & 0xffff;
        bn[1] = u.x >> 16;
        bn[2] = u.y & 0xffff;
        bn[3] = u.y >> 16;
      }
      acc.x += M[bn[0]];
      acc.y += M[bn[1]];
      acc.z += M[bn[2]];
      acc.w += M[bn[3]];
    }
    *reinterpret_cast<float4*>(out + i) = make_float4(acc.x * scale, acc.y * scale, acc.z * scale, acc.w * scale);
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
                   unsigned long long* sums, uint32_t* counts, int32_t* arrive, const int32_t* seg_chunk_begin,
                   float* means, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  static bool lds_attr = false;  // q up to 1024: 4 waves x 1024 x 12 B + 8 KB of scales = 56 KB of dynamic LDS
  if (!lds_attr) {
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)sketch_encode_kernel<uint8_t>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    GRACE_HIP_CHECK(hipFuncSetAttribute((const void*)sketch_encode_kernel<uint16_t>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    lds_attr = true;
  }
  constexpr int NW = kBlock / kWave;
  const size_t lds = (size_t)NW * q * 8 + (size_t)q * 8 + (size_t)NW * q * 4;
  if (bin_bytes == 1)
    sketch_encode_kernel<uint8_t><<<ct.n_chunks, kBlock, lds, stream>>>(ct, x, edges, q, (uint8_t*)bins, sums, counts,
                                                                        arrive, seg_chunk_begin, means);
  else
    sketch_encode_kernel<uint16_t><<<ct.n_chunks, kBlock, lds, stream>>>(ct, x, edges, q, (uint16_t*)bins, sums,
                                                                         counts, arrive, seg_chunk_begin, means);
}

void sketch_encode_big(const ChunkTable& ct, int n_seg, const float* x, const float* edges, int q, void* bins,
                       int bin_bytes, unsigned long long* sums, uint32_t* counts, int32_t* arrive,
                       const int32_t* seg_chunk_begin, float* means, hipStream_t stream) {
  if (ct.n_chunks == 0 || n_seg == 0) return;
  if (bin_bytes == 1)
    sketch_encode_big_kernel<uint8_t><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, edges, q, (uint8_t*)bins, sums,
                                                                          counts, arrive, seg_chunk_begin, means);
  else
    sketch_encode_big_kernel<uint16_t><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, edges, q, (uint16_t*)bins, sums,
                                                                           counts, arrive, seg_chunk_begin, means);
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
