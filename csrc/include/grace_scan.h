// Workgroup-wide prefix sums for stream compaction (wave64 shuffles + one LDS round).
//
// Compaction kernels (top-k, threshold, DGC) used to take one global atomic per wave to
// reserve output slots; with all workgroups of a large tensor hitting ONE per-segment counter
// that serialises at the memory side (hundreds of microseconds per bucket).  The pattern here:
// every thread counts its selected elements in registers, the workgroup computes exclusive
// prefixes with these helpers, and a single atomic per workgroup-tile reserves the output.
#pragma once

#include "grace_common.h"

namespace grace {

// inclusive scan of v across the 64 lanes of a wave
__device__ __forceinline__ int wave_inclusive_scan(int v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int t = __shfl_up(v, o, kWave);
    if (l >= o) v += t;
  }
  return v;
}

// Exclusive scan over the workgroup. `lds` must hold (blockDim.x / 64) ints.
// Returns the thread's exclusive prefix; *total receives the workgroup sum (all threads).
template <int BLOCK>
__device__ __forceinline__ int block_exclusive_scan(int v, int* lds, int* total) {
  constexpr int NW = BLOCK / kWave;
  const int incl = wave_inclusive_scan(v);
  const int w = wave_id();
  __syncthreads();
  if (lane_id() == kWave - 1) lds[w] = incl;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int s = lds[i];
    off += (i < w) ? s : 0;
    tot += s;
  }
  *total = tot;
  return off + incl - v;
}

}  // namespace grace
