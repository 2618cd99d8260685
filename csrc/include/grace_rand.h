// Keyed pseudo-random permutation of [0, n) (Random-K index generation).
//
// Reference Random-K draws ``torch.randperm(n)[:k]`` after reseeding the GLOBAL torch RNG
// (/root/reference/grace_dl/dist/compressor/randomk.py:6-12, 26-28): O(n log n) work for k << n
// and a side effect on every other RNG consumer.  Here index j of the selection is
// pi_seed(j) where pi is a 4-round balanced Feistel network on ceil-even(log2 n) bits with
// cycle walking -- a bijection on [0, n), O(1) per index, no state, identical on every rank.
// grace_amd/ops/randomk.py implements bit-identical integer arithmetic in PyTorch.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace grace {

__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

struct FeistelKey {
  uint32_t k[4];
  uint32_t half;  // bits per half
  uint32_t mask;  // (1 << half) - 1
};

__host__ __device__ __forceinline__ FeistelKey feistel_key(uint64_t seed, uint64_t n) {
  FeistelKey fk;
  uint32_t bits = 2;
  while (bits < 64 && (1ull << bits) < n) ++bits;
  if (bits & 1) ++bits;
  fk.half = bits >> 1;
  fk.mask = (fk.half >= 32) ? 0xffffffffu : ((1u << fk.half) - 1u);
  const uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
  for (int i = 0; i < 4; ++i) fk.k[i] = fmix32(lo ^ (0x9E3779B9u * (uint32_t)(i + 1)) ^ fmix32(hi + (uint32_t)i));
  return fk;
}

__host__ __device__ __forceinline__ uint64_t feistel_round4(uint64_t x, const FeistelKey& fk) {
  uint32_t L = (uint32_t)(x >> fk.half) & fk.mask;
  uint32_t R = (uint32_t)x & fk.mask;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t f = fmix32(R ^ fk.k[i]) & fk.mask;
    const uint32_t nL = R;
    R = L ^ f;
    L = nL;
  }
  return ((uint64_t)L << fk.half) | R;
}

// pi(j) for j < n: apply the Feistel permutation until the value falls inside [0, n).
__host__ __device__ __forceinline__ uint64_t feistel_perm(uint64_t j, uint64_t n, const FeistelKey& fk) {
  uint64_t y = feistel_round4(j, fk);
  while (y >= n) y = feistel_round4(y, fk);
  return y;
}

}  // namespace grace
