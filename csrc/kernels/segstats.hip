// Segmented statistics over a flat bucket: one pass computes, per segment,
//   sum, sum of squares, max|x|, sum|x|, sum of negatives, count of negatives
// (everything the reference computes with separate reductions per tensor: QSGD's norm
//  qsgd.py:12, TernGrad's mean/std/max terngrad.py:12-17, EF-SignSGD's mean|x|
//  efsignsgd.py:14, OneBit's per-sign means onebit.py:10-18, U8bit's max|x| u8bit.py:52).
//
// Deterministic two-stage reduction (no float atomics): stage 1 writes one partial per chunk,
// stage 2 folds the chunks of each segment in chunk order.  Partials accumulate in fp64 so
// sum/sumsq of multi-million-element tensors do not lose precision.
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kBlock = 256;
constexpr int kNW = kBlock / kWave;

__device__ __forceinline__ double wsum(double v) { return wave_sum(v); }

// mode 0: x = g ; mode 1: x = beta*r + gamma*g.  When xout != nullptr the compensated x is
// stored (fusing the error-feedback compensate into the statistics pass).
__global__ __launch_bounds__(kBlock) void segstats_partial_kernel(ChunkTable ct, const float* g, const float* r,
                                                                  int mode, float beta, float gamma, float* xout,
                                                                  double* __restrict__ part) {
  const int c = blockIdx.x;
  const int64_t b = ct.begin[c], e = ct.end[c];
  double s = 0, s2 = 0, sa = 0, sn = 0;
  float amax = 0.f;
  uint32_t nneg = 0;
  for (int64_t i = b + threadIdx.x; i < e; i += kBlock) {
    float v = g[i];
    if (mode == 1) v = fmaf(beta, r[i], gamma * v);
    if (xout != nullptr) xout[i] = v;
    s += v;
    s2 += (double)v * v;
    sa += fabsf(v);
    amax = fmaxf(amax, fabsf(v));
    if (v < 0.f) {
      sn += v;
      ++nneg;
    }
  }
  __shared__ double red[5][kNW];
  __shared__ float redm[kNW];
  s = wsum(s);
  s2 = wsum(s2);
  sa = wsum(sa);
  sn = wsum(sn);
  const double cn = wsum((double)nneg);
  amax = wave_max(amax);
  const int w = wave_id();
  if (lane_id() == 0) {
    red[0][w] = s;
    red[1][w] = s2;
    red[2][w] = sa;
    red[3][w] = sn;
    red[4][w] = cn;
    redm[w] = amax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double o[5] = {0, 0, 0, 0, 0};
    float m = 0.f;
    for (int i = 0; i < kNW; ++i) {
#pragma unroll
      for (int k = 0; k < 5; ++k) o[k] += red[k][i];
      m = fmaxf(m, redm[i]);
    }
    double* p = part + (int64_t)c * kSegStats;
    p[0] = o[0];
    p[1] = o[1];
    p[2] = m;
    p[3] = o[2];
    p[4] = o[3];
    p[5] = o[4];
  }
}

// one thread per segment folds its chunk partials in order
__global__ void segstats_fold_kernel(int n_seg, const int32_t* __restrict__ seg_chunk_begin,
                                     const double* __restrict__ part, float* __restrict__ stats) {
  const int sgi = blockIdx.x * blockDim.x + threadIdx.x;
  if (sgi >= n_seg) return;
  double o[kSegStats] = {0, 0, 0, 0, 0, 0};
  for (int c = seg_chunk_begin[sgi]; c < seg_chunk_begin[sgi + 1]; ++c) {
    const double* p = part + (int64_t)c * kSegStats;
    o[0] += p[0];
    o[1] += p[1];
    o[2] = fmax(o[2], p[2]);
    o[3] += p[3];
    o[4] += p[4];
    o[5] += p[5];
  }
  float* out = stats + (int64_t)sgi * kSegStats;
#pragma unroll
  for (int k = 0; k < kSegStats; ++k) out[k] = (float)o[k];
}

}  // namespace

void segment_stats(const ChunkTable& ct, int n_seg, const int32_t* seg_chunk_begin, const float* g,
                   const float* r, int mode, float beta, float gamma, float* xout, double* partials, float* stats,
                   hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  segstats_partial_kernel<<<ct.n_chunks, kBlock, 0, stream>>>(ct, g, r, mode, beta, gamma, xout, partials);
  segstats_fold_kernel<<<(n_seg + 255) / 256, 256, 0, stream>>>(n_seg, seg_chunk_begin, partials, stats);
}

}  // namespace grace
