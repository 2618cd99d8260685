// Shared device helpers for the grace_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64: lane = threadIdx.x & 63, ballots are 64-bit.
//   * A "bucket" is a flat fp32 buffer holding many parameter gradients back to back
//     ("segments").  Work is decomposed into CHUNKS that never straddle a segment, so a
//     workgroup always knows its segment id without searching (chunk table built once per
//     bucket layout on the host, grace_amd/ops/layout.py).
//   * Randomness is counter-based (Philox4x32-10) keyed by (seed, element index) so results
//     are independent of the launch geometry and reproducible across ranks when required.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace grace {

constexpr int kWave = 64;

struct ChunkTable {
  const int32_t* seg;    // segment id of chunk c
  const int64_t* begin;  // flat begin (inclusive) of chunk c
  const int64_t* end;    // flat end (exclusive) of chunk c
  int32_t n_chunks;
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ unsigned wave_sum_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Block-wide reduction through LDS; `scratch` must hold blockDim.x/64 elements.
// Every thread receives the result.
template <typename T, typename Op>
__device__ __forceinline__ T block_reduce(T v, T* scratch, Op op, T (*wave_fn)(T)) {
  v = wave_fn(v);
  const int w = wave_id();
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) scratch[w] = v;
  __syncthreads();
  T r = scratch[0];
  for (int i = 1; i < nw; ++i) r = op(r, scratch[i]);
  return r;
}

// Order-preserving 31-bit key of |x| (sign cleared): for finite non-negative floats the IEEE
// bit pattern is monotonic, so radix-selecting the largest keys selects the largest |x|.
// NaN maps above +inf, i.e. it is always selected (it would poison the step anyway).
__device__ __forceinline__ uint32_t abs_key(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// ---------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (Salmon et al., SC'11).  One call yields 4 uint32.
// ---------------------------------------------------------------------------------------
struct Philox {
  static constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  static constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  __device__ __forceinline__ static uint4 round(uint4 c, uint2 k) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
  }
  __device__ __forceinline__ static uint4 gen(uint64_t seed, uint64_t counter, uint32_t stream = 0) {
    uint4 c = make_uint4((uint32_t)counter, (uint32_t)(counter >> 32), stream, 0x5ca1ab1eu);
    uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c = round(c, k);
      k.x += W0;
      k.y += W1;
    }
    return c;
  }
};

// RNG seed = host base seed, optionally mixed with a DEVICE step counter.  Reading the step
// from device memory (bumped by a captured kernel every step) keeps stochastic codecs correct
// under HIP-graph replay: a host-side seed would be frozen into the graph.
struct SeedArg {
  uint64_t base;
  const int64_t* step;  // nullptr: use base as is
  __device__ __forceinline__ uint64_t get() const {
    return step ? (base ^ ((uint64_t)(*step) * 0x9E3779B97F4A7C15ull)) : base;
  }
};

// fp32 -> bf16 bits, round-to-nearest-even; NaN -> canonical 0x7FC0 (c10::BFloat16's rule, so
// kernels produce exactly what tensor.to(torch.bfloat16) produces)
__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7FC0u;
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// uniform float in [0, 1) from 24 random bits
__device__ __forceinline__ float u01(uint32_t r) { return (r >> 8) * (1.0f / 16777216.0f); }

// Flat element index -> position of the element inside its chunk-local loop.
template <int BLOCK>
struct ChunkIter {
  int64_t b, e;
};

}  // namespace grace

#define GRACE_HIP_CHECK(expr)                                                                  \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(_e), __FILE__, __LINE__, \
              #expr);                                                                          \
      abort();                                                                                 \
    }                                                                                          \
  } while (0)
