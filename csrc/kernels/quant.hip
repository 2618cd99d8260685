// Stochastic / fixed quantizers for CDNA4: QSGD, TernGrad, Natural compression, 8-bit (U8bit).
//
// All kernels run over the bucket's chunk table (a workgroup knows its segment and loads that
// segment's scale once).  Randomness is counter-based Philox4x32-10 keyed by (seed, element):
// element i uses word (i & 3) of Philox(seed, i >> 2), so results do not depend on the launch
// geometry; seeds differ per rank (independent rounding noise, as in the reference's
// per-process torch RNG) and per step.
//
//  QSGD     (qsgd.py:12-38)     q = sign(x) * (floor(l) + [u < frac(l)]),  l = s*|x|/||x||_2
//                               codes int8 (s < 128) or int16 (the reference's fp16 for s >= 128
//                               is lossy above 2048 levels: survey 2.14 #12)
//  TernGrad (terngrad.py:8-32)  t = sign(clamp(x,+-c)) * [u*scal < |clamp(x,+-c)|], c = 2.5*std,
//                               scal = max|clamp| ; sent as TWO bit planes per 64 elements
//                               (nonzero, negative) = 2 bits/element (reference: int8)
//  Natural  (natural.py:13-40)  stochastic rounding of the exponent, 8-bit sign+exponent code
//  U8bit    (tensorflow/compressor/u8bit.py:11-110)  |x|/max|x| bucketised into a fixed
//                               128-entry table (constant memory, binary search), int8 code
//
// Every *_aggregate kernel decodes all W ranks' payloads (rank-strided rows of the all-gather
// output, fixed rank order -> bit-identical on every rank) and writes scale * sum in ONE pass.
#include <type_traits>

#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

__device__ __forceinline__ uint32_t pick(const uint4& r, int k) {
  return k == 0 ? r.x : (k == 1 ? r.y : (k == 2 ? r.z : r.w));
}

// ------------------------------------------------------------------------------------ QSGD
template <typename CodeT, bool RESID>
__global__ __launch_bounds__(kBlock) void qsgd_quant_kernel(ChunkTable ct, const float* x,
                                                            const float* __restrict__ norms, float s,
                                                            SeedArg sa, CodeT* __restrict__ codes,
                                                            float* resid) {
  const uint64_t seed = sa.get();
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const float norm = norms[sg];
  const float inv = norm > 0.f ? s / norm : 0.f;
  const float deq = norm / s;
  for (int64_t base = (b & ~int64_t(3)) + 4 * (int64_t)threadIdx.x; base < e; base += 4 * kBlock) {
    const uint4 rnd = Philox::gen(seed, (uint64_t)base >> 2);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + k;
      if (i < b || i >= e) continue;
      const float v = x[i];
      const float l = inv * fabsf(v);
      const float fl = floorf(l);
      const float q = fl + ((u01(pick(rnd, k)) < (l - fl)) ? 1.f : 0.f);
      const float code = v < 0.f ? -q : (v > 0.f ? q : 0.f);
      codes[i] = (CodeT)code;
      if constexpr (RESID) resid[i] = v - deq * code;
    }
  }
}

// Bit-packed QSGD codes for small s (ceil(log2(2s+1)) bits): code + s stored
// unsigned in B = 2 (s = 1) or 4 (s <= 7) bits, element i at bit (i * B) of the row.
template <int B>
struct PackedCode {};

template <typename CodeT>
struct CodeIO {  // plain int8 / int16 / fp16 / int32 codes
  static __device__ __forceinline__ float at(const uint8_t* row, int64_t i, float) {
    return (float)reinterpret_cast<const CodeT*>(row)[i];
  }
};
template <int B>
struct CodeIO<PackedCode<B>> {
  static __device__ __forceinline__ float at(const uint8_t* row, int64_t i, float s) {
    const int64_t bit = i * B;
    const uint32_t v = (row[bit >> 3] >> (bit & 7)) & ((1u << B) - 1u);
    return (float)v - s;
  }
};

// 4 codes of one rank as floats (one 4/8/16-B load)
template <typename CodeT>
__device__ __forceinline__ float4 load_codes4(const CodeT* p) {
  if constexpr (sizeof(CodeT) == 1) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
    return make_float4((float)(int8_t)(u & 0xff), (float)(int8_t)((u >> 8) & 0xff), (float)(int8_t)((u >> 16) & 0xff),
                       (float)(int8_t)(u >> 24));
  } else if constexpr (sizeof(CodeT) == 2) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    CodeT c[4];
    *reinterpret_cast<uint2*>(c) = u;
    return make_float4((float)c[0], (float)c[1], (float)c[2], (float)c[3]);
  } else {
    const int4 u = *reinterpret_cast<const int4*>(p);
    return make_float4((float)u.x, (float)u.y, (float)u.z, (float)u.w);
  }
}

// 4 codes starting at element i (i % 4 == 0) of one rank's code row
template <typename CodeT>
__device__ __forceinline__ float4 load4(const uint8_t* row, int64_t i, float) {
  return load_codes4(reinterpret_cast<const CodeT*>(row) + i);
}
template <>
__device__ __forceinline__ float4 load4<PackedCode<2>>(const uint8_t* row, int64_t i, float s) {
  const uint32_t v = row[i >> 2];  // 4 x 2-bit codes in one byte
  return make_float4((float)(v & 3u) - s, (float)((v >> 2) & 3u) - s, (float)((v >> 4) & 3u) - s,
                     (float)(v >> 6) - s);
}
template <>
__device__ __forceinline__ float4 load4<PackedCode<4>>(const uint8_t* row, int64_t i, float s) {
  const uint32_t v = *reinterpret_cast<const uint16_t*>(row + (i >> 1));  // 4 x 4-bit codes
  return make_float4((float)(v & 15u) - s, (float)((v >> 4) & 15u) - s, (float)((v >> 8) & 15u) - s,
                     (float)(v >> 12) - s);
}

// Pack int8 codes in [-s, s] into B-bit fields (code + s); thread t handles codes 16t..16t+15.
template <int B>
__global__ __launch_bounds__(kBlock) void qsgd_pack_kernel(const int8_t* __restrict__ codes, int64_t n, int s,
                                                           uint8_t* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t * 16 < n; t += (int64_t)gridDim.x * kBlock) {
    const int64_t i0 = t * 16;
    uint64_t word = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t i = i0 + j;
      const uint64_t v = i < n ? (uint64_t)(codes[i] + s) : 0ull;
      word |= v << (j * B);
    }
    // 16 codes -> 16 * B / 8 bytes (4 or 8), byte-granular tail
    uint8_t* o = out + i0 * B / 8;
    const int64_t nbytes_all = (n * B + 7) / 8;
    const int64_t nb = min<int64_t>(16 * B / 8, nbytes_all - i0 * B / 8);
    if (nb == 16 * B / 8) {
      if constexpr (B == 2) *reinterpret_cast<uint32_t*>(o) = (uint32_t)word;
      else *reinterpret_cast<uint64_t*>(o) = word;
    } else {
      for (int64_t k = 0; k < nb; ++k) o[k] = (uint8_t)(word >> (8 * k));
    }
  }
}

// out[i] (+)= scale * sum_r norm_r[seg] / s * code_r[i].  `shared_norms` (shared-scale all-reduced
// codes: one norm for every rank) replaces the per-rank norms of the payload rows.  VEC: the
// codes and out are 16-B aligned at element 0 (host-checked), so the chunk body runs 4
// elements per thread with one vector load per rank.
template <typename CodeT, bool VEC>
__global__ __launch_bounds__(kBlock) void qsgd_aggregate_kernel(ChunkTable ct, const uint8_t* __restrict__ base,
                                                                int64_t rank_stride, int64_t codes_off,
                                                                int64_t norms_off, const float* __restrict__ shared_norms,
                                                                int n_ranks, float s, float inv_s, float scale,
                                                                float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  auto norm = [&](int r) {
    return shared_norms ? shared_norms[sg]
                        : reinterpret_cast<const float*>(base + (int64_t)r * rank_stride + norms_off)[sg];
  };
  auto scalar = [&](int64_t i) {
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) {
      const float q = CodeIO<CodeT>::at(base + (int64_t)r * rank_stride + codes_off, i, s);
      acc += norm(r) * inv_s * q;
    }
    acc *= scale;
    out[i] = accumulate ? out[i] + acc : acc;
  };
  if constexpr (!VEC) {
    for (int64_t i = b + threadIdx.x; i < e; i += kBlock) scalar(i);
  } else {
    const int64_t a0 = ((b + 3) & ~(int64_t)3) < e ? ((b + 3) & ~(int64_t)3) : e;
    const int64_t a1 = a0 + ((e - a0) & ~(int64_t)3);
    for (int64_t i = b + threadIdx.x; i < a0; i += kBlock) scalar(i);
    for (int64_t i = a1 + threadIdx.x; i < e; i += kBlock) scalar(i);
    for (int64_t i = a0 + 4 * (int64_t)threadIdx.x; i < a1; i += 4 * kBlock) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int r = 0; r < n_ranks; ++r) {
        const float f = norm(r) * inv_s;
        const float4 q = load4<CodeT>(base + (int64_t)r * rank_stride + codes_off, i, s);
        acc.x += f * q.x;
        acc.y += f * q.y;
        acc.z += f * q.z;
        acc.w += f * q.w;
      }
      float4 o = make_float4(acc.x * scale, acc.y * scale, acc.z * scale, acc.w * scale);
      if (accumulate) {
        const float4 p = *reinterpret_cast<const float4*>(out + i);
        o.x += p.x;
        o.y += p.y;
        o.z += p.z;
        o.w += p.w;
      }
      *reinterpret_cast<float4*>(out + i) = o;
    }
  }
}

// ------------------------------------------------------------------------------------ TernGrad
template <bool RESID>
__global__ __launch_bounds__(kBlock) void tern_quant_kernel(ChunkTable ct, const int64_t* __restrict__ seg_start,
                                                            const int64_t* __restrict__ word_off, const float* x,
                                                            const float* __restrict__ clips,
                                                            const float* __restrict__ scal, SeedArg sa,
                                                            uint64_t* __restrict__ words, float* resid) {
  const uint64_t seed = sa.get();
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const int64_t g0 = (b - seg_start[sg]) >> 6;
  const int64_t ngroups = (e - b + kWave - 1) / kWave;
  const float clip = clips[sg], sc = scal[sg];
  for (int64_t q = wave_id(); q < ngroups; q += kWavesPerBlock) {
    const int64_t i = b + q * kWave + lane_id();
    const bool valid = i < e;
    float t = 0.f, v = 0.f;
    if (valid) {
      v = x[i];
      const float gc = fminf(fmaxf(v, -clip), clip);
      const uint4 rnd = Philox::gen(seed, (uint64_t)i >> 2);
      const float u = u01(pick(rnd, (int)(i & 3))) * sc;
      if (u < fabsf(gc)) t = gc > 0.f ? 1.f : (gc < 0.f ? -1.f : 0.f);
    }
    const unsigned long long nz = __ballot(t != 0.f);
    const unsigned long long ng = __ballot(t < 0.f);
    if (lane_id() == 0) {
      const int64_t w = 2 * (word_off[sg] + g0 + q);
      words[w] = nz;
      words[w + 1] = ng;
    }
    if constexpr (RESID) {
      if (valid) resid[i] = v - t * sc;
    }
  }
}

__global__ __launch_bounds__(kBlock) void tern_aggregate_kernel(ChunkTable ct, const int64_t* __restrict__ seg_start,
                                                                const int64_t* __restrict__ word_off,
                                                                const uint8_t* __restrict__ base, int64_t rank_stride,
                                                                int64_t words_off, int64_t scal_off, int n_ranks,
                                                                float scale, float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const int64_t g0 = (b - seg_start[sg]) >> 6;
  const int64_t ngroups = (e - b + kWave - 1) / kWave;
  for (int64_t q = wave_id(); q < ngroups; q += kWavesPerBlock) {
    const int64_t i = b + q * kWave + lane_id();
    const int64_t w = 2 * (word_off[sg] + g0 + q);
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) {
      const uint8_t* rb = base + (int64_t)r * rank_stride;
      const uint64_t* wp = reinterpret_cast<const uint64_t*>(rb + words_off);
      const uint64_t nz = wp[w], ng = wp[w + 1];
      const float sc = reinterpret_cast<const float*>(rb + scal_off)[sg];
      const int l = lane_id();
      if ((nz >> l) & 1ull) acc += ((ng >> l) & 1ull) ? -sc : sc;
    }
    if (i < e) {
      acc *= scale;
      out[i] = accumulate ? out[i] + acc : acc;
    }
  }
}

// ------------------------------------------------------------------------------------ Natural
__device__ __forceinline__ uint8_t natural_encode(float v, uint32_t rnd23) {
  const uint32_t bits = __float_as_uint(v);
  const uint32_t sign = bits & 0x80000000u;
  uint32_t expo = bits & 0x7f800000u;
  const uint32_t mant = bits & 0x007fffffu;
  if (mant > rnd23) expo += 0x00800000u;  // round the exponent up w.p. mantissa / 2^23
  expo = expo < 0x09000000u ? 0x09000000u : (expo > 0x48800000u ? 0x48800000u : expo);
  return (uint8_t)((sign >> 24) | ((expo >> 23) - 18u));
}

__device__ __forceinline__ float natural_decode(uint8_t code) {
  const uint32_t e = code & 0x7fu;
  if (e < 1u) return 0.f;
  const float f = __uint_as_float((e + 18u) << 23);
  return (code & 0x80u) ? -f : f;
}

template <bool RESID>
__global__ __launch_bounds__(kBlock) void natural_encode_kernel(const float* x, int64_t n, SeedArg sa,
                                                                uint8_t* __restrict__ codes, float* resid) {
  const uint64_t seed = sa.get();
  const int64_t stride = (int64_t)gridDim.x * kBlock * 4;
  for (int64_t base = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4; base < n; base += stride) {
    const uint4 rnd = Philox::gen(seed, (uint64_t)base >> 2);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + k;
      if (i >= n) break;
      const float v = x[i];
      const uint8_t cd = natural_encode(v, pick(rnd, k) & 0x007fffffu);
      codes[i] = cd;
      if constexpr (RESID) resid[i] = v - natural_decode(cd);
    }
  }
}

__global__ __launch_bounds__(kBlock) void natural_aggregate_kernel(const uint8_t* __restrict__ base,
                                                                   int64_t rank_stride, int64_t n, int n_ranks,
                                                                   float scale, float* __restrict__ out,
                                                                   int accumulate) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) acc += natural_decode(base[(int64_t)r * rank_stride + i]);
    acc *= scale;
    out[i] = accumulate ? out[i] + acc : acc;
  }
}

// ------------------------------------------------------------------------------------ U8bit
__constant__ float kDict128[128] = {
    1.5000001e-06f, 2.7500000e-06f, 7.2499997e-06f, 1.8750001e-05f, 3.6250000e-05f, 5.8749996e-05f,
    8.6249995e-05f, 1.4375000e-04f, 2.3125000e-04f, 3.1875001e-04f, 4.0625001e-04f, 5.1874999e-04f,
    6.5624999e-04f, 7.9374999e-04f, 9.3124999e-04f, 1.2187500e-03f, 1.6562500e-03f, 2.0937501e-03f,
    2.5312500e-03f, 2.9687500e-03f, 3.4062499e-03f, 3.8437501e-03f, 4.2812498e-03f, 4.8437500e-03f,
    5.5312500e-03f, 6.2187500e-03f, 6.9062500e-03f, 7.5937500e-03f, 8.2812496e-03f, 8.9687500e-03f,
    9.6562495e-03f, 1.1093750e-02f, 1.3281250e-02f, 1.5468750e-02f, 1.7656250e-02f, 1.9843750e-02f,
    2.2031249e-02f, 2.4218749e-02f, 2.6406251e-02f, 2.8593751e-02f, 3.0781250e-02f, 3.2968748e-02f,
    3.5156250e-02f, 3.7343752e-02f, 3.9531250e-02f, 4.1718751e-02f, 4.3906249e-02f, 4.6718750e-02f,
    5.0156251e-02f, 5.3593751e-02f, 5.7031251e-02f, 6.0468748e-02f, 6.3906237e-02f, 6.7343749e-02f,
    7.0781253e-02f, 7.4218743e-02f, 7.7656247e-02f, 8.1093743e-02f, 8.4531240e-02f, 8.7968737e-02f,
    9.1406241e-02f, 9.4843738e-02f, 9.8281242e-02f, 1.0546875e-01f, 1.1640625e-01f, 1.2734374e-01f,
    1.3828126e-01f, 1.4921875e-01f, 1.6015625e-01f, 1.7109375e-01f, 1.8203124e-01f, 1.9296876e-01f,
    2.0390625e-01f, 2.1484375e-01f, 2.2578125e-01f, 2.3671874e-01f, 2.4765626e-01f, 2.5859374e-01f,
    2.6953125e-01f, 2.8046876e-01f, 2.9140624e-01f, 3.0234376e-01f, 3.1328124e-01f, 3.2421875e-01f,
    3.3515626e-01f, 3.4609374e-01f, 3.5703126e-01f, 3.6796874e-01f, 3.7890625e-01f, 3.8984376e-01f,
    4.0078124e-01f, 4.1171876e-01f, 4.2265624e-01f, 4.3359375e-01f, 4.4453126e-01f, 4.5859376e-01f,
    4.7578123e-01f, 4.9296874e-01f, 5.1015621e-01f, 5.2734375e-01f, 5.4453123e-01f, 5.6171870e-01f,
    5.7890624e-01f, 5.9609371e-01f, 6.1328125e-01f, 6.3046873e-01f, 6.4765620e-01f, 6.6484374e-01f,
    6.8203121e-01f, 6.9921869e-01f, 7.1640623e-01f, 7.3359370e-01f, 7.5078118e-01f, 7.6796871e-01f,
    7.8515619e-01f, 8.0234367e-01f, 8.1953120e-01f, 8.3671868e-01f, 8.5390615e-01f, 8.7109369e-01f,
    8.8828117e-01f, 9.0546864e-01f, 9.2265618e-01f, 9.3984365e-01f, 9.5703113e-01f, 9.7421867e-01f,
    9.9140614e-01f, 9.9570298e-01f};

// bin = (#edges <= v) - 1, clamped to [0, 126]
__device__ __forceinline__ int u8_bin(float v) {
  int lo = 0, hi = 128;  // first index with edge > v
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (kDict128[mid] <= v)
      lo = mid + 1;
    else
      hi = mid;
  }
  int b = lo - 1;
  return b < 0 ? 0 : (b > 126 ? 126 : b);
}

template <bool RESID>
__global__ __launch_bounds__(kBlock) void u8_encode_kernel(ChunkTable ct, const float* x,
                                                           const float* __restrict__ scales, int8_t* __restrict__ codes,
                                                           float* resid) {
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const float sc = scales[sg];
  const float inv = sc > 0.f ? 1.f / sc : 0.f;
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    const float v = x[i];
    const int bin = u8_bin(fabsf(v) * inv);
    const int code = v > 0.f ? bin : (v < 0.f ? -bin : 0);
    codes[i] = (int8_t)code;
    if constexpr (RESID) resid[i] = v - (code == 0 ? 0.f : (code > 0 ? 1.f : -1.f) * kDict128[bin] * sc);
  }
}

__global__ __launch_bounds__(kBlock) void u8_aggregate_kernel(ChunkTable ct, const uint8_t* __restrict__ base,
                                                              int64_t rank_stride, int64_t codes_off, int64_t scal_off,
                                                              int n_ranks, float scale, float* __restrict__ out,
                                                              int accumulate) {
  const int c = blockIdx.x;
  const int sg = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    float acc = 0.f;
    for (int r = 0; r < n_ranks; ++r) {
      const uint8_t* rb = base + (int64_t)r * rank_stride;
      const int q = reinterpret_cast<const int8_t*>(rb + codes_off)[i];
      const float sc = reinterpret_cast<const float*>(rb + scal_off)[sg];
      const int a = q < 0 ? -q : q;
      if (q != 0) acc += (q > 0 ? 1.f : -1.f) * kDict128[a] * sc;
    }
    acc *= scale;
    out[i] = accumulate ? out[i] + acc : acc;
  }
}

inline int grid_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

// code_bytes: 1 = int8, 2 = int16, 4 = int32, 3 = fp16 (integer levels; exact up to 2048, the
// all-reducible 16-bit code: RCCL has no int16 reduction)
void qsgd_quantize(const ChunkTable& ct, const float* x, const float* norms, float s, SeedArg seed, void* codes,
                   int code_bytes, float* resid, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  auto go = [&](auto* typed) {
    using T = std::remove_pointer_t<decltype(typed)>;
    if (resid)
      qsgd_quant_kernel<T, true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, norms, s, seed, (T*)codes, resid);
    else
      qsgd_quant_kernel<T, false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, norms, s, seed, (T*)codes, nullptr);
  };
  if (code_bytes == 1) go((int8_t*)nullptr);
  else if (code_bytes == 2) go((int16_t*)nullptr);
  else if (code_bytes == 3) go((_Float16*)nullptr);
  else go((int32_t*)nullptr);
}

void qsgd_aggregate(const ChunkTable& ct, const uint8_t* base, int64_t rank_stride, int64_t codes_off,
                    int64_t norms_off, const float* shared_norms, int code_bytes, int n_ranks, float s, float scale,
                    float* out, bool accumulate, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  const float inv_s = 1.f / s;
  const bool vec = ((reinterpret_cast<uintptr_t>(base) + codes_off) % 16 == 0) && (rank_stride % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  auto go = [&](auto* typed) {
    using T = std::remove_pointer_t<decltype(typed)>;
    if (vec)
      qsgd_aggregate_kernel<T, true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, base, rank_stride, codes_off, norms_off,
                                                                         shared_norms, n_ranks, s, inv_s, scale, out,
                                                                         accumulate);
    else
      qsgd_aggregate_kernel<T, false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, base, rank_stride, codes_off, norms_off,
                                                                          shared_norms, n_ranks, s, inv_s, scale, out,
                                                                          accumulate);
  };
  if (code_bytes == 1) go((int8_t*)nullptr);
  else if (code_bytes == 2) go((int16_t*)nullptr);
  else if (code_bytes == 3) go((_Float16*)nullptr);
  else if (code_bytes == kPacked2) go((PackedCode<2>*)nullptr);
  else if (code_bytes == kPacked4) go((PackedCode<4>*)nullptr);
  else go((int32_t*)nullptr);
}

void qsgd_pack(const int8_t* codes, int64_t n, int s, int bits, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  const int64_t th = (n + 15) / 16;
  const int grid = (int)std::min<int64_t>((th + kBlock - 1) / kBlock, 4096);
  if (bits == 2) qsgd_pack_kernel<2><<<grid, kBlock, 0, stream>>>(codes, n, s, out);
  else qsgd_pack_kernel<4><<<grid, kBlock, 0, stream>>>(codes, n, s, out);
}

void tern_quantize(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const float* x,
                   const float* clips, const float* scal, SeedArg seed, uint64_t* words, float* resid,
                   hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  if (resid)
    tern_quant_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, seg_start, word_off, x, clips, scal, seed, words,
                                                                resid);
  else
    tern_quant_kernel<false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, seg_start, word_off, x, clips, scal, seed, words,
                                                                 nullptr);
}

void tern_aggregate(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const uint8_t* base,
                    int64_t rank_stride, int64_t words_off, int64_t scal_off, int n_ranks, float scale, float* out,
                    bool accumulate, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  tern_aggregate_kernel<<<ct.n_chunks, kBlock, 0, stream>>>(ct, seg_start, word_off, base, rank_stride, words_off,
                                                            scal_off, n_ranks, scale, out, accumulate ? 1 : 0);
}

void natural_encode(const float* x, int64_t n, SeedArg seed, uint8_t* codes, float* resid, hipStream_t stream) {
  if (n <= 0) return;
  const int grid = grid_for((n + 3) / 4);
  if (resid)
    natural_encode_kernel<true><<<grid, kBlock, 0, stream>>>(x, n, seed, codes, resid);
  else
    natural_encode_kernel<false><<<grid, kBlock, 0, stream>>>(x, n, seed, codes, nullptr);
}

void natural_aggregate(const uint8_t* base, int64_t rank_stride, int64_t n, int n_ranks, float scale, float* out,
                       bool accumulate, hipStream_t stream) {
  if (n <= 0) return;
  natural_aggregate_kernel<<<grid_for(n), kBlock, 0, stream>>>(base, rank_stride, n, n_ranks, scale, out,
                                                               accumulate ? 1 : 0);
}

void u8_encode(const ChunkTable& ct, const float* x, const float* scales, int8_t* codes, float* resid,
               hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  if (resid)
    u8_encode_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, scales, codes, resid);
  else
    u8_encode_kernel<false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, x, scales, codes, nullptr);
}

void u8_aggregate(const ChunkTable& ct, const uint8_t* base, int64_t rank_stride, int64_t codes_off, int64_t scal_off,
                  int n_ranks, float scale, float* out, bool accumulate, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  u8_aggregate_kernel<<<ct.n_chunks, kBlock, 0, stream>>>(ct, base, rank_stride, codes_off, scal_off, n_ranks, scale,
                                                          out, accumulate ? 1 : 0);
}

}  // namespace grace
