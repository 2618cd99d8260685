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

// Per-thread accumulators: at most chunk/kBlock = 32 elements per thread, so fp32 is exact
// enough; the cross-thread / cross-chunk reductions run in fp64.
struct Acc {
  float s = 0.f, s2 = 0.f, sa = 0.f, sn = 0.f, amax = 0.f;
  uint32_t nneg = 0;
  __device__ __forceinline__ void add(float v) {
    s += v;
    s2 = fmaf(v, v, s2);
    const float a = fabsf(v);
    sa += a;
    amax = fmaxf(amax, a);
    if (v < 0.f) {
      sn += v;
      ++nneg;
    }
  }
};

template <int MODE>
__device__ __forceinline__ float comp(float g, float r, float beta, float gamma) {
  return MODE == 1 ? fmaf(beta, r, gamma * g) : g;
}

// MODE 0: x = g ; MODE 1: x = beta*r + gamma*g.  STORE: the compensated x is written to xout
// (fusing the error-feedback compensate into the statistics pass).  VEC: 16-B aligned bases,
// the chunk body is read with float4 loads (head/tail scalar).
template <int MODE, bool STORE, bool VEC>
__global__ __launch_bounds__(kBlock) void segstats_partial_kernel(ChunkTable ct, const float* g, const float* r,
                                                                  float beta, float gamma, float* xout,
                                                                  double* __restrict__ part) {
  const int c = blockIdx.x;
  const int64_t b = ct.begin[c], e = ct.end[c];
  Acc a;
  int64_t body_b = b, body_e = b;
  if (VEC) {
    body_b = (b + 3) & ~int64_t(3);
    if (body_b > e) body_b = e;
    body_e = body_b + ((e - body_b) & ~int64_t(3));
    const int64_t n4 = (body_e - body_b) >> 2;
    const float4* g4 = reinterpret_cast<const float4*>(g + body_b);
    const float4* r4 = reinterpret_cast<const float4*>(r + body_b);
    float4* x4 = reinterpret_cast<float4*>(xout + body_b);
    for (int64_t j = threadIdx.x; j < n4; j += kBlock) {
      const float4 gv = g4[j];
      float4 v = gv;
      if (MODE == 1) {
        const float4 rv = r4[j];
        v.x = comp<MODE>(gv.x, rv.x, beta, gamma);
        v.y = comp<MODE>(gv.y, rv.y, beta, gamma);
        v.z = comp<MODE>(gv.z, rv.z, beta, gamma);
        v.w = comp<MODE>(gv.w, rv.w, beta, gamma);
      }
      if (STORE) x4[j] = v;
      a.add(v.x);
      a.add(v.y);
      a.add(v.z);
      a.add(v.w);
    }
  }
  // scalar head [b, body_b) and tail [body_e, e) (the whole chunk when !VEC)
  const int64_t nh = body_b - b, nt = e - body_e;
  for (int64_t t = threadIdx.x; t < nh + nt; t += kBlock) {
    const int64_t i = t < nh ? b + t : body_e + (t - nh);
    const float v = comp<MODE>(g[i], MODE == 1 ? r[i] : 0.f, beta, gamma);
    if (STORE) xout[i] = v;
    a.add(v);
  }
  __shared__ double red[5][kNW];
  __shared__ float redm[kNW];
  const double s = wave_sum((double)a.s), s2 = wave_sum((double)a.s2), sa = wave_sum((double)a.sa),
               sn = wave_sum((double)a.sn), cn = wave_sum((double)a.nneg);
  const float amax = wave_max(a.amax);
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

// One workgroup per segment: thread t folds chunks c0+t, c0+t+256, ... then a fixed-order
// tree over the workgroup (deterministic for a given chunk table, so every rank computes
// bit-identical statistics from identical inputs).  A 23 M-element embedding segment has
// ~2900 chunks: the old one-thread-per-segment fold spent 113 us in a dependent chain.
__global__ __launch_bounds__(kBlock) void segstats_fold_kernel(const int32_t* __restrict__ seg_chunk_begin,
                                                               const double* __restrict__ part,
                                                               float* __restrict__ stats) {
  const int sg = blockIdx.x;
  const int c0 = seg_chunk_begin[sg], c1 = seg_chunk_begin[sg + 1];
  double o[kSegStats] = {0, 0, 0, 0, 0, 0};
  for (int c = c0 + (int)threadIdx.x; c < c1; c += kBlock) {
    const double* p = part + (int64_t)c * kSegStats;
    o[0] += p[0];
    o[1] += p[1];
    o[2] = fmax(o[2], p[2]);
    o[3] += p[3];
    o[4] += p[4];
    o[5] += p[5];
  }
  __shared__ double red[kSegStats][kNW];
#pragma unroll
  for (int k = 0; k < kSegStats; ++k) {
    double v = o[k];
    if (k == 2) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
    } else {
      v = wave_sum(v);
    }
    if (lane_id() == 0) red[k][wave_id()] = v;
  }
  __syncthreads();
  if (threadIdx.x < kSegStats) {
    const int k = threadIdx.x;
    double v = red[k][0];
    for (int i = 1; i < kNW; ++i) v = k == 2 ? fmax(v, red[k][i]) : v + red[k][i];
    stats[(int64_t)sg * kSegStats + k] = (float)v;
  }
}

template <int MODE, bool STORE>
void launch_partial(const ChunkTable& ct, const float* g, const float* r, float beta, float gamma, float* xout,
                    double* partials, hipStream_t stream) {
  const bool vec = (((uintptr_t)g | (uintptr_t)r | (uintptr_t)xout) & 15) == 0;
  if (vec)
    segstats_partial_kernel<MODE, STORE, true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, g, r, beta, gamma, xout,
                                                                                   partials);
  else
    segstats_partial_kernel<MODE, STORE, false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, g, r, beta, gamma, xout,
                                                                                    partials);
}

}  // namespace

void segment_stats(const ChunkTable& ct, int n_seg, const int32_t* seg_chunk_begin, const float* g,
                   const float* r, int mode, float beta, float gamma, float* xout, double* partials, float* stats,
                   hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  if (mode == 1) {
    if (xout)
      launch_partial<1, true>(ct, g, r, beta, gamma, xout, partials, stream);
    else
      launch_partial<1, false>(ct, g, r, beta, gamma, xout, partials, stream);
  } else {
    if (xout)
      launch_partial<0, true>(ct, g, r, beta, gamma, xout, partials, stream);
    else
      launch_partial<0, false>(ct, g, r, beta, gamma, xout, partials, stream);
  }
  segstats_fold_kernel<<<n_seg, kBlock, 0, stream>>>(seg_chunk_begin, partials, stats);
}

}  // namespace grace
