// INCEPTIONN lossy floating-point codec (Li et al., MICRO 2018) on CDNA4.
//
// Reference: /root/reference/grace_dl/tensorflow/compressor/inceptionn.py:17-188 (TF graph of
// boolean masks, tf.boolean_mask compactions, tfp.stats.find_bins to recover exponents).
// Elements are classed by biased exponent e (e_b = 127 + int(log10(eb / 2)),
// mid = e_b + ceil((127 - e_b) / 2)):
//   class 3  e >= 127        value kept as fp32
//   class 2  mid <= e < 127  16-bit fixed point (sign | 1.mantissa >> (127 - e)) >> 8
//   class 1  e_b <= e < mid   8-bit fixed point (same) >> 16
//   class 0  e < e_b          dropped
// Payload (fixed capacity, graph-capturable): [int32 header = class totals (0, n8, n16, n32) |
// value stream of `cap` bytes: v32 fp32, v16 uint16, v8 uint8 back to back | class codes, 2
// bits/element, 4 per byte].  The decoder recounts the classes from the codes, so it needs no
// size exchange and no host read.
//
// The three value streams are ORDER-PRESERVING compactions (the decoder pairs the i-th class-c
// code with the i-th class-c value), so the workgroup mapping is "contiguous per thread":
// a 256-thread workgroup owns a tile of 256 x 32 consecutive elements, thread t its 32
// consecutive elements; ordered ranks come from one packed workgroup exclusive scan
// (grace_scan.h) plus a device scan of the per-tile counts:
//   inc_count    per-tile class counts          (encode pass 1, or from codes when decoding)
//   inc_scan     exclusive per-tile offsets      (one workgroup; class totals at the end)
//   inc_encode   codes + compacted streams       (encode pass 2)
//   inc_decode   all W ranks' payloads decoded and summed in rank order in one pass
#include "grace_common.h"
#include "grace_kernels.h"
#include "grace_scan.h"

namespace grace {
namespace {

constexpr int kBlock = 256;
constexpr int kPer = 32;
constexpr int kTile = kBlock * kPer;

__device__ __forceinline__ int inc_class(uint32_t u, int e_b, int mid) {
  const int e = (int)((u >> 23) & 0xFF);
  return e >= 127 ? 3 : (e >= mid ? 2 : (e >= e_b ? 1 : 0));
}

__device__ __forceinline__ uint32_t inc_fixed(uint32_t u) {
  const int e = (int)((u >> 23) & 0xFF);
  const int shift = 127 - e;  // >= 1 for the fixed-point classes
  const uint32_t m = ((u & 0x7FFFFFu) >> 1) | 0x400000u;
  const uint32_t sh = shift >= 32 ? 0u : (m >> shift);
  return ((u & 0x80000000u) >> 8) | sh;
}

// floor(log2(v)) for v >= 2, else 0  (reference find_bins over [0, 2, 4, 8, ...])
__device__ __forceinline__ int lead_bin(uint32_t v) { return v >= 2 ? 31 - __clz(v) : 0; }

__device__ __forceinline__ float dec16(uint32_t w) {
  const uint32_t s = (w & 0x8000u) << 16;
  const uint32_t vs = (w << 1) & 0xFFFFu;
  const int nsh = 16 - lead_bin(vs);
  const uint32_t e = (uint32_t)(127 - (nsh - 1)) << 23;
  const uint32_t m = ((vs << nsh) & 0xFFFFu) << 7;
  return __uint_as_float(s | e | m);
}

__device__ __forceinline__ float dec8(uint32_t w) {
  const uint32_t s = (w & 0x80u) << 24;
  const uint32_t vs = (w << 1) & 0xFFu;
  const int nsh = 8 - lead_bin(vs);
  const uint32_t e = (uint32_t)(127 - (nsh - 1)) << 23;
  const uint32_t m = ((vs << nsh) & 0xFFu) << 15;
  return __uint_as_float(s | e | m);
}

// 2-bit code of element i from the packed code bytes
__device__ __forceinline__ int code_at(const uint8_t* codes, int64_t i) { return (codes[i >> 2] >> (2 * (i & 3))) & 3; }

// Per-tile class counts.  FROM_CODES: classes come from a payload's code bytes (decode side),
// else from the fp32 input.  cnt: int32 [n_src][n_tiles][4] (class 0 unused).
template <bool FROM_CODES>
__global__ __launch_bounds__(kBlock) void inc_count_kernel(const float* __restrict__ x, const int64_t* code_ptrs,
                                                           int64_t n, int64_t n_tiles, int e_b, int mid,
                                                           int32_t* __restrict__ cnt) {
  const int src = blockIdx.y;
  const int64_t tile = blockIdx.x;
  const uint8_t* codes = FROM_CODES ? reinterpret_cast<const uint8_t*>(code_ptrs[src]) : nullptr;
  const int64_t base = tile * kTile + (int64_t)threadIdx.x * kPer;
  int c[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = base + j;
    if (i < n) {
      const int k = FROM_CODES ? code_at(codes, i) : inc_class(__float_as_uint(x[i]), e_b, mid);
      c[1] += k == 1;
      c[2] += k == 2;
      c[3] += k == 3;
    }
  }
  __shared__ int red[3][kBlock / kWave];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const int v = (int)wave_sum_u32((unsigned)c[k]);
    if (lane_id() == 0) red[k - 1][wave_id()] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int s = 0;
    for (int w = 0; w < kBlock / kWave; ++w) s += red[threadIdx.x][w];
    cnt[((int64_t)src * n_tiles + tile) * 4 + 1 + threadIdx.x] = s;
  }
  if (threadIdx.x == 3) cnt[((int64_t)src * n_tiles + tile) * 4] = 0;
}

// In-place exclusive scan of the per-tile counts of one source (one workgroup per source);
// totals[src][4] receives the class totals.
__global__ __launch_bounds__(kBlock) void inc_scan_kernel(int32_t* __restrict__ cnt, int64_t n_tiles,
                                                          int32_t* __restrict__ totals) {
  const int src = blockIdx.x;
  int32_t* c = cnt + (int64_t)src * n_tiles * 4;
  __shared__ int lds[kBlock / kWave];
  int carry[4] = {0, 0, 0, 0};
  for (int64_t t0 = 0; t0 < n_tiles; t0 += kBlock) {
    const int64_t t = t0 + threadIdx.x;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const int v = t < n_tiles ? c[t * 4 + k] : 0;
      int tot = 0;
      const int ex = block_exclusive_scan<kBlock>(v, lds, &tot);
      if (t < n_tiles) c[t * 4 + k] = carry[k] + ex;
      carry[k] += tot;
    }
  }
  if (threadIdx.x < 4) totals[src * 4 + threadIdx.x] = threadIdx.x == 0 ? 0 : carry[threadIdx.x];
}

// Unified value stream of a capacity payload: [v32 fp32 (n32) | v16 (n16) | v8 (n8)] starting at
// byte 0, 4 * n32 and 4 * n32 + 2 * n16 (n* = class totals, device-resident).  `cap` bytes of
// stream: when the classes do not fit, the lowest-precision classes are dropped first (class 1,
// then class 2 -> code 0), and class-3 values past cap / 4 in element order are dropped; the
// decoder recounts from the codes, so it stays consistent.  cap >= 4 n never drops anything.
struct IncPlan {
  bool keep1, keep2;
  int64_t cap3;
  int64_t off16, off8;
};

__device__ __forceinline__ IncPlan inc_plan(const int32_t* tot, int64_t cap) {
  const int64_t n8 = tot[1], n16 = tot[2], n32 = tot[3];
  IncPlan p;
  p.keep2 = 4 * n32 + 2 * n16 <= cap;
  p.keep1 = p.keep2 && 4 * n32 + 2 * n16 + n8 <= cap;
  p.cap3 = cap / 4;
  p.off16 = 4 * (n32 < p.cap3 ? n32 : p.cap3);
  p.off8 = p.off16 + (p.keep2 ? 2 * n16 : 0);
  return p;
}

// Encode pass 2.  off: scanned per-tile offsets of the single source; tot: its class totals.
__global__ __launch_bounds__(kBlock) void inc_encode_kernel(const float* __restrict__ x, int64_t n, int e_b, int mid,
                                                            const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ tot,
                                                            uint8_t* __restrict__ stream, int64_t cap,
                                                            uint8_t* __restrict__ codes, uint32_t* health) {
  __shared__ int lds[kBlock / kWave];
  const IncPlan pl = inc_plan(tot, cap);
  if (blockIdx.x == 0 && threadIdx.x == 0 && (!pl.keep1 && tot[1] > 0 || !pl.keep2 && tot[2] > 0 || tot[3] > pl.cap3))
    health_count_overflow(health);  // a class (or class-3 tail) is dropped this step
  float* v32 = reinterpret_cast<float*>(stream);
  uint16_t* v16 = reinterpret_cast<uint16_t*>(stream + pl.off16);
  uint8_t* v8 = stream + pl.off8;
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * kTile + (int64_t)threadIdx.x * kPer;
  uint32_t u[kPer];
  int c1 = 0, c23 = 0;  // c23 packs class-2 count (low 16 bits) and class-3 count (high 16 bits)
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = base + j;
    u[j] = i < n ? __float_as_uint(x[i]) : 0u;
    const int k = i < n ? inc_class(u[j], e_b, mid) : 0;
    c1 += k == 1;
    c23 += k == 2 ? 1 : (k == 3 ? 0x10000 : 0);
  }
  int t1 = 0, t23 = 0;
  const int p1 = block_exclusive_scan<kBlock>(c1, lds, &t1);
  const int p23 = block_exclusive_scan<kBlock>(c23, lds, &t23);
  int o1 = off[tile * 4 + 1] + p1;
  int o2 = off[tile * 4 + 2] + (p23 & 0xFFFF);
  int o3 = off[tile * 4 + 3] + (p23 >> 16);
  uint32_t packed[kPer / 16] = {};
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = base + j;
    int k = i < n ? inc_class(u[j], e_b, mid) : 0;
    if (k == 3) {
      if (o3 < pl.cap3)
        v32[o3] = __uint_as_float(u[j]);
      else
        k = 0;  // past the capacity (always the LAST class-3 elements in order)
      ++o3;
    } else if (k == 2) {
      if (pl.keep2) v16[o2++] = (uint16_t)((inc_fixed(u[j]) >> 8) & 0xFFFFu);
      else k = 0;
    } else if (k == 1) {
      if (pl.keep1) v8[o1++] = (uint8_t)((inc_fixed(u[j]) >> 16) & 0xFFu);
      else k = 0;
    }
    packed[j >> 4] |= (uint32_t)k << (2 * (j & 15));
  }
  // 32 elements -> 8 code bytes (element base+j at byte (base+j)/4, bits 2*(j%4))
#pragma unroll
  for (int h = 0; h < kPer / 16; ++h) {
    const int64_t b0 = (base >> 2) + 4 * h;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if ((base + 16 * h + 4 * q) < n) codes[b0 + q] = (uint8_t)(packed[h] >> (8 * q));
  }
}

// W rank-strided capacity payloads in ONE buffer: rank r's stream at base + r*stride + stream_off,
// its codes at base + r*stride + codes_off (no per-rank pointer table: graph-capturable).
// off: [W][n_tiles][4] scanned counts recounted from the codes; tot: [W][4] their totals.
__global__ __launch_bounds__(kBlock) void inc_decode_kernel(const uint8_t* __restrict__ base_u8, int64_t stride,
                                                            int64_t stream_off, int64_t codes_off, int n_ranks,
                                                            int64_t n, int64_t n_tiles, const int32_t* __restrict__ off,
                                                            const int32_t* __restrict__ tot, float scale,
                                                            float* __restrict__ out, int accumulate) {
  __shared__ int lds[kBlock / kWave];
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * kTile + (int64_t)threadIdx.x * kPer;
  float acc[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) acc[j] = 0.f;
  for (int r = 0; r < n_ranks; ++r) {
    const uint8_t* row = base_u8 + (int64_t)r * stride;
    const uint8_t* codes = row + codes_off;
    // after the encoder's drops the codes ARE the kept classes: plain back-to-back layout
    const int32_t* t = tot + 4 * r;
    const float* v32 = reinterpret_cast<const float*>(row + stream_off);
    const uint16_t* v16 = reinterpret_cast<const uint16_t*>(row + stream_off + 4 * (int64_t)t[3]);
    const uint8_t* v8 = row + stream_off + 4 * (int64_t)t[3] + 2 * (int64_t)t[2];
    int k[kPer];
    int c1 = 0, c23 = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int64_t i = base + j;
      k[j] = i < n ? code_at(codes, i) : 0;
      c1 += k[j] == 1;
      c23 += k[j] == 2 ? 1 : (k[j] == 3 ? 0x10000 : 0);
    }
    int t1 = 0, t23 = 0;
    const int p1 = block_exclusive_scan<kBlock>(c1, lds, &t1);
    const int p23 = block_exclusive_scan<kBlock>(c23, lds, &t23);
    const int32_t* o = off + ((int64_t)r * n_tiles + tile) * 4;
    int o1 = o[1] + p1, o2 = o[2] + (p23 & 0xFFFF), o3 = o[3] + (p23 >> 16);
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      float v = 0.f;
      if (k[j] == 3)
        v = v32[o3++];
      else if (k[j] == 2)
        v = dec16(v16[o2++]);
      else if (k[j] == 1)
        v = dec8(v8[o1++]);
      acc[j] += v;
    }
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = base + j;
    if (i < n) out[i] = accumulate ? out[i] + scale * acc[j] : scale * acc[j];
  }
}

// recount from codes: per-tile class counts of W rank-strided code arrays
__global__ __launch_bounds__(kBlock) void inc_count_codes_kernel(const uint8_t* __restrict__ base_u8, int64_t stride,
                                                                 int64_t codes_off, int64_t n, int64_t n_tiles,
                                                                 int32_t* __restrict__ cnt) {
  const int src = blockIdx.y;
  const int64_t tile = blockIdx.x;
  const uint8_t* codes = base_u8 + (int64_t)src * stride + codes_off;
  const int64_t base = tile * kTile + (int64_t)threadIdx.x * kPer;
  int c[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t i = base + j;
    if (i < n) {
      const int k = code_at(codes, i);
      c[1] += k == 1;
      c[2] += k == 2;
      c[3] += k == 3;
    }
  }
  __shared__ int red[3][kBlock / kWave];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const int v = (int)wave_sum_u32((unsigned)c[k]);
    if (lane_id() == 0) red[k - 1][wave_id()] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int s = 0;
    for (int w = 0; w < kBlock / kWave; ++w) s += red[threadIdx.x][w];
    cnt[((int64_t)src * n_tiles + tile) * 4 + 1 + threadIdx.x] = s;
  }
  if (threadIdx.x == 3) cnt[((int64_t)src * n_tiles + tile) * 4] = 0;
}

}  // namespace

int64_t inceptionn_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

void inceptionn_count(const float* x, int64_t n, int e_b, int mid, int32_t* cnt, int32_t* totals,
                      hipStream_t stream) {
  const int64_t nt = inceptionn_tiles(n);
  if (nt == 0) {
    GRACE_HIP_CHECK(hipMemsetAsync(totals, 0, 4 * sizeof(int32_t), stream));
    return;
  }
  inc_count_kernel<false><<<dim3((unsigned)nt, 1), kBlock, 0, stream>>>(x, nullptr, n, nt, e_b, mid, cnt);
  inc_scan_kernel<<<1, kBlock, 0, stream>>>(cnt, nt, totals);
}

void inceptionn_encode(const float* x, int64_t n, int e_b, int mid, const int32_t* off, const int32_t* totals,
                       uint8_t* stream, int64_t cap_bytes, uint8_t* codes, hipStream_t stream_) {
  const int64_t nt = inceptionn_tiles(n);
  if (nt == 0) return;
  inc_encode_kernel<<<(unsigned)nt, kBlock, 0, stream_>>>(x, n, e_b, mid, off, totals, stream, cap_bytes, codes,
                                                       health_words().host_dev);
}

void inceptionn_decode(const uint8_t* base, int64_t rank_stride, int64_t stream_off, int64_t codes_off, int n_ranks,
                       int64_t n, int32_t* cnt, int32_t* totals, float scale, float* out, bool accumulate,
                       hipStream_t stream) {
  const int64_t nt = inceptionn_tiles(n);
  if (nt == 0 || n_ranks <= 0) return;
  inc_count_codes_kernel<<<dim3((unsigned)nt, (unsigned)n_ranks), kBlock, 0, stream>>>(base, rank_stride, codes_off,
                                                                                       n, nt, cnt);
  inc_scan_kernel<<<n_ranks, kBlock, 0, stream>>>(cnt, nt, totals);
  inc_decode_kernel<<<(unsigned)nt, kBlock, 0, stream>>>(base, rank_stride, stream_off, codes_off, n_ranks, n, nt, cnt,
                                                         totals, scale, out, accumulate ? 1 : 0);
}

}  // namespace grace
