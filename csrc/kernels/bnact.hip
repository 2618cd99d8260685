// Fused training-mode BatchNorm (+ residual add) (+ ReLU) for channels_last bf16 activations.
//
// Why: in a ResNet-50 training step on MI355X the BN chain is the largest non-GEMM cost.  The
// stock path runs, per BN layer, MIOpen mean/var + final + normalise forward, a ReLU kernel, a
// residual add, a `num_batches_tracked += 1` kernel, and in backward a ReLU-backward, MIOpen
// dscale/dbias + final + dx, plus memsets (≈11 launches per layer, ~4.7 ms of a 9.4 ms step in
// profiles/r1_resnet50_topk_graph_bf16w_kernels.txt).  Here a layer is 4 kernels:
//
//   fwd  bn_stats   : per-channel Σx, Σx² over the NHWC rows (16-B bf16 loads, fp32 sums),
//                     per-block partials, the LAST block (agent-scope arrival counter) folds
//                     them in fp64 and writes mean/invstd, the folded affine (scale, shift),
//                     the running statistics and num_batches_tracked
//        bn_apply   : y = relu(x*scale + shift [+ residual]) -> bf16
//   bwd  bn_reduce  : Σdz, Σdz·(x-mean) with dz = dy·[y>0]; last block writes dgamma, dbeta
//                     and the 3 per-channel coefficients of dx = a·dz + b·x + c
//        bn_dx      : dx (bf16) and, for the fused residual, d(residual) = dz (bf16)
//
// Activations are [M = N·H·W rows, C channels] row-major (channels_last).  A thread owns 8
// consecutive channels (one 16-B load per row); TPR = C/8 threads cover a row.  C % 8 == 0 and
// C <= 2048 (checked on the host; other shapes use the PyTorch path).
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kB = 256;           // threads per block
constexpr int kMaxC = 2048;       // TPR <= 256
constexpr int kPartFloats = 131072;  // cap on nblk * C (fold cost of the last block)

struct Bf8 {
  float v[8];
};

__device__ __forceinline__ Bf8 load_bf8(const uint16_t* p) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  Bf8 r;
  r.v[0] = __uint_as_float(u.x << 16);
  r.v[1] = __uint_as_float(u.x & 0xffff0000u);
  r.v[2] = __uint_as_float(u.y << 16);
  r.v[3] = __uint_as_float(u.y & 0xffff0000u);
  r.v[4] = __uint_as_float(u.z << 16);
  r.v[5] = __uint_as_float(u.z & 0xffff0000u);
  r.v[6] = __uint_as_float(u.w << 16);
  r.v[7] = __uint_as_float(u.w & 0xffff0000u);
  return r;
}

__device__ __forceinline__ void store_bf8(uint16_t* p, const float* v) {
  uint4 u;
  u.x = (uint32_t)f32_to_bf16_rne(v[0]) | ((uint32_t)f32_to_bf16_rne(v[1]) << 16);
  u.y = (uint32_t)f32_to_bf16_rne(v[2]) | ((uint32_t)f32_to_bf16_rne(v[3]) << 16);
  u.z = (uint32_t)f32_to_bf16_rne(v[4]) | ((uint32_t)f32_to_bf16_rne(v[5]) << 16);
  u.w = (uint32_t)f32_to_bf16_rne(v[6]) | ((uint32_t)f32_to_bf16_rne(v[7]) << 16);
  *reinterpret_cast<uint4*>(p) = u;
}

struct Geo {
  int C, tpr, tprp, rpi;  // channels, threads per row, pow2 >= tpr, rows per block iteration
};

__device__ __forceinline__ Geo geo(int C) {
  Geo g;
  g.C = C;
  g.tpr = C >> 3;
  g.tprp = 1;
  while (g.tprp < g.tpr) g.tprp <<= 1;
  g.rpi = kB / g.tprp;
  return g;
}

// Block-level column reduction of two 8-wide per-thread accumulators into part[blk][2C]
// (first C: quantity A, next C: quantity B), then the arrival counter.  Returns true in every
// thread of the last-arriving block.
__device__ bool block_partials_and_arrive(const Geo& g, const float* a, const float* b, float* part,
                                          unsigned* counter) {
  __shared__ float sa[kB * 8];
  __shared__ float sb[kB * 8];
  __shared__ int last;
  const int cg = threadIdx.x % g.tprp, rs = threadIdx.x / g.tprp;
  if (cg < g.tpr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa[rs * g.C + cg * 8 + j] = a[j];
      sb[rs * g.C + cg * 8 + j] = b[j];
    }
  }
  __syncthreads();
  float* pb = part + (size_t)blockIdx.x * 2 * g.C;
  for (int c = threadIdx.x; c < g.C; c += kB) {
    float x = 0.f, y = 0.f;
    for (int i = 0; i < g.rpi; ++i) {
      x += sa[i * g.C + c];
      y += sb[i * g.C + c];
    }
    pb[c] = x;
    pb[g.C + c] = y;
  }
  __threadfence();  // partials visible at agent scope before this block's arrival
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (prev == gridDim.x - 1);
  }
  __syncthreads();
  if (last) __threadfence();  // acquire side for the other threads of the last block
  return last != 0;
}

// Last block: fold part[nblk][2C] into fp64 totals.  Calls fn(c, A, B) once per channel.
template <typename Fn>
__device__ void fold_partials(int C, int nblk, const float* part, Fn fn) {
  __shared__ double fa[kB];
  __shared__ double fb[kB];
  if (C >= kB) {
    for (int c = threadIdx.x; c < C; c += kB) {
      double x = 0.0, y = 0.0;
      for (int b = 0; b < nblk; ++b) {
        x += part[(size_t)b * 2 * C + c];
        y += part[(size_t)b * 2 * C + C + c];
      }
      fn(c, x, y);
    }
  } else {
    const int R = kB / C;  // threads per channel
    const int c = threadIdx.x % C, r = threadIdx.x / C;
    double x = 0.0, y = 0.0;
    if (r < R)
      for (int b = r; b < nblk; b += R) {
        x += part[(size_t)b * 2 * C + c];
        y += part[(size_t)b * 2 * C + C + c];
      }
    fa[threadIdx.x] = x;
    fb[threadIdx.x] = y;
    __syncthreads();
    if (threadIdx.x < C) {
      for (int i = 1; i < R; ++i) {
        x += fa[i * C + c];
        y += fb[i * C + c];
      }
      fn(c, x, y);
    }
  }
}

struct StatsOut {
  const float* gamma;   // may be null (affine=False -> 1)
  const float* beta;    // may be null (-> 0)
  float* running_mean;  // may be null
  float* running_var;   // may be null
  int64_t* nbt;         // num_batches_tracked, may be null
  float momentum, eps;
  float* save;          // [4C]: mean, invstd, scale, shift
};

__global__ __launch_bounds__(kB) void bn_stats_kernel(const uint16_t* __restrict__ x, int64_t M, int C,
                                                      int64_t rows_per_blk, float* __restrict__ part,
                                                      unsigned* counter, StatsOut o) {
  const Geo g = geo(C);
  const int cg = threadIdx.x % g.tprp, rs = threadIdx.x / g.tprp;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = min(M, r0 + rows_per_blk);
  if (cg < g.tpr) {
    const uint16_t* base = x + cg * 8;
    int64_t r = r0 + rs;
    for (; r + 3 * g.rpi < r1; r += 4 * g.rpi) {  // 4 independent 16-B loads in flight
      Bf8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = load_bf8(base + (r + u * g.rpi) * C);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += v[u].v[j];
          q[j] = fmaf(v[u].v[j], v[u].v[j], q[j]);
        }
    }
    for (; r < r1; r += g.rpi) {
      const Bf8 v = load_bf8(base + r * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v.v[j];
        q[j] = fmaf(v.v[j], v.v[j], q[j]);
      }
    }
  }
  if (!block_partials_and_arrive(g, s, q, part, counter)) return;
  const double inv_m = 1.0 / (double)M;
  const double unbias = M > 1 ? (double)M / (double)(M - 1) : 1.0;
  fold_partials(C, gridDim.x, part, [&](int c, double S, double Q) {
    const double mean = S * inv_m;
    const double var = fmax(Q * inv_m - mean * mean, 0.0);
    const float invstd = (float)(1.0 / sqrt(var + (double)o.eps));
    const float ga = o.gamma ? o.gamma[c] : 1.f;
    const float be = o.beta ? o.beta[c] : 0.f;
    const float scale = ga * invstd;
    o.save[c] = (float)mean;
    o.save[C + c] = invstd;
    o.save[2 * C + c] = scale;
    o.save[3 * C + c] = be - (float)mean * scale;
    if (o.running_mean) {
      o.running_mean[c] = (1.f - o.momentum) * o.running_mean[c] + o.momentum * (float)mean;
      o.running_var[c] = (1.f - o.momentum) * o.running_var[c] + o.momentum * (float)(var * unbias);
    }
  });
  if (threadIdx.x == 0) {
    if (o.nbt) *o.nbt += 1;
    *counter = 0;  // re-arm for the next launch (graph replays reuse the slot)
  }
}

// y = act(x*scale + shift [+ res]); scale/shift = save[2C..4C)
template <bool RELU, bool RES>
__global__ __launch_bounds__(kB) void bn_apply_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                      const float* __restrict__ save, uint16_t* __restrict__ y,
                                                      int64_t n_vec, int C) {
  const int tpr = C >> 3;
  const int64_t stride = (int64_t)gridDim.x * kB;
  int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  // stride % tpr == 0 (host picks the grid): the thread's channel group never changes
  const int cg = (int)(i % tpr);
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = save[2 * C + cg * 8 + j];
    sh[j] = save[3 * C + cg * 8 + j];
  }
  for (; i < n_vec; i += stride) {
    const Bf8 v = load_bf8(x + i * 8);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(v.v[j], sc[j], sh[j]);
    if constexpr (RES) {
      const Bf8 r = load_bf8(res + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += r.v[j];
    }
    if constexpr (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    store_bf8(y + i * 8, o);
  }
}

struct GradOut {
  const float* gamma;  // may be null
  const float* save;   // [4C] from the forward
  float* dgamma;       // may be null
  float* dbeta;        // may be null
  float* coef;         // [3C]: a, b, c with dx = a*dz + b*x + c
};

template <bool RELU>
__global__ __launch_bounds__(kB) void bn_reduce_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ y, int64_t M, int C,
                                                       int64_t rows_per_blk, float* __restrict__ part,
                                                       unsigned* counter, GradOut o) {
  const Geo g = geo(C);
  const int cg = threadIdx.x % g.tprp, rs = threadIdx.x / g.tprp;
  float s1[8], s2[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_blk;
  const int64_t r1 = min(M, r0 + rows_per_blk);
  if (cg < g.tpr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) mu[j] = o.save[cg * 8 + j];
    const int64_t off = cg * 8;
    int64_t r = r0 + rs;
    for (; r + g.rpi < r1; r += 2 * g.rpi) {
      Bf8 d[2], v[2], w[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t e = (r + u * g.rpi) * C + off;
        d[u] = load_bf8(dy + e);
        v[u] = load_bf8(x + e);
        if constexpr (RELU) w[u] = load_bf8(y + e);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float dz = d[u].v[j];
          if constexpr (RELU) dz = w[u].v[j] > 0.f ? dz : 0.f;
          s1[j] += dz;
          s2[j] = fmaf(dz, v[u].v[j] - mu[j], s2[j]);
        }
    }
    for (; r < r1; r += g.rpi) {
      const int64_t e = r * C + off;
      const Bf8 d = load_bf8(dy + e);
      const Bf8 v = load_bf8(x + e);
      Bf8 w;
      if constexpr (RELU) w = load_bf8(y + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float dz = d.v[j];
        if constexpr (RELU) dz = w.v[j] > 0.f ? dz : 0.f;
        s1[j] += dz;
        s2[j] = fmaf(dz, v.v[j] - mu[j], s2[j]);
      }
    }
  }
  if (!block_partials_and_arrive(g, s1, s2, part, counter)) return;
  const double inv_m = 1.0 / (double)M;
  fold_partials(C, gridDim.x, part, [&](int c, double S1, double S2) {
    const float mean = o.save[c], invstd = o.save[C + c];
    const float ga = o.gamma ? o.gamma[c] : 1.f;
    const double dg = S2 * (double)invstd;  // dgamma = Σ dz·x̂
    if (o.dgamma) o.dgamma[c] = (float)dg;
    if (o.dbeta) o.dbeta[c] = (float)S1;
    const double a = (double)ga * invstd;
    const double b = -a * invstd * dg * inv_m;
    o.coef[c] = (float)a;
    o.coef[C + c] = (float)b;
    o.coef[2 * C + c] = (float)(-a * S1 * inv_m - b * mean);
  });
  if (threadIdx.x == 0) *counter = 0;
}

template <bool RELU, bool RES>
__global__ __launch_bounds__(kB) void bn_dx_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                   const uint16_t* __restrict__ y, const float* __restrict__ coef,
                                                   uint16_t* __restrict__ dx, uint16_t* __restrict__ dres,
                                                   int64_t n_vec, int C) {
  const int tpr = C >> 3;
  const int64_t stride = (int64_t)gridDim.x * kB;
  int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int cg = (int)(i % tpr);
  float ca[8], cb[8], cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ca[j] = coef[cg * 8 + j];
    cb[j] = coef[C + cg * 8 + j];
    cc[j] = coef[2 * C + cg * 8 + j];
  }
  for (; i < n_vec; i += stride) {
    const Bf8 d = load_bf8(dy + i * 8);
    const Bf8 v = load_bf8(x + i * 8);
    float dz[8], o[8];
    if constexpr (RELU) {
      const Bf8 w = load_bf8(y + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = w.v[j] > 0.f ? d.v[j] : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = d.v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(ca[j], dz[j], fmaf(cb[j], v.v[j], cc[j]));
    store_bf8(dx + i * 8, o);
    if constexpr (RES) store_bf8(dres + i * 8, dz);
  }
}

// ---------------------------------------------------------------- launch geometry
// Arrival counters: a small device pool, each launch takes the next slot round-robin (the
// last block re-arms it), so concurrently running BN kernels never share a counter.
constexpr int kSlots = 1024;
unsigned* g_counters[64] = {};
int g_next[64] = {};

unsigned* next_counter(hipStream_t stream) {
  int dev = 0;
  GRACE_HIP_CHECK(hipGetDevice(&dev));
  if (!g_counters[dev]) {
    GRACE_HIP_CHECK(hipMalloc(&g_counters[dev], kSlots * sizeof(unsigned)));
    GRACE_HIP_CHECK(hipMemsetAsync(g_counters[dev], 0, kSlots * sizeof(unsigned), stream));
    GRACE_HIP_CHECK(hipStreamSynchronize(stream));
  }
  const int s = g_next[dev];
  g_next[dev] = (s + 1) % kSlots;
  return g_counters[dev] + s;
}

int64_t tprp_of(int C) {
  int64_t t = 1;
  while (t < C / 8) t <<= 1;
  return t;
}

// (#blocks, rows per block) for the two reduction kernels
void reduce_grid(int64_t M, int C, int* nblk, int64_t* rows_per_blk) {
  const int64_t rpi = kB / tprp_of(C);
  int64_t cap = kPartFloats / C;                  // bounded fold work for the last block
  if (cap > 2048) cap = 2048;
  int64_t want = (M + 4 * rpi - 1) / (4 * rpi);  // >= 4 row iterations per block when possible
  int64_t nb = want < cap ? want : cap;
  if (nb < 1) nb = 1;
  int64_t rpb = (M + nb - 1) / nb;
  rpb = (rpb + rpi - 1) / rpi * rpi;
  nb = (M + rpb - 1) / rpb;
  if (nb < 1) nb = 1;
  *nblk = (int)nb;
  *rows_per_blk = rpb;
}

int apply_grid(int64_t n_vec, int C) {
  const int64_t tpr = C / 8;
  int64_t b = (n_vec + kB - 1) / kB;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  // stride must be a multiple of tpr: kB*b % tpr == 0 always holds for tpr | kB; otherwise
  // round the grid up to a multiple of tpr / gcd(tpr, kB)
  int64_t g = tpr, h = kB;
  while (h) { const int64_t t = g % h; g = h; h = t; }
  const int64_t m = tpr / g;
  b = (b + m - 1) / m * m;
  return (int)b;
}

}  // namespace

int64_t bn_workspace_floats(int64_t M, int C) {
  int nblk;
  int64_t rpb;
  reduce_grid(M, C, &nblk, &rpb);
  return (int64_t)nblk * 2 * C;
}

void bn_act_forward(const uint16_t* x, const uint16_t* res, int64_t M, int C, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps, bool relu,
                    float* save, float* part, uint16_t* y, hipStream_t stream) {
  int nblk;
  int64_t rpb;
  reduce_grid(M, C, &nblk, &rpb);
  StatsOut o{gamma, beta, running_mean, running_var, nbt, momentum, eps, save};
  hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk), dim3(kB), 0, stream, x, M, C, rpb, part, next_counter(stream), o);
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  if (relu && res)
    hipLaunchKernelGGL((bn_apply_kernel<true, true>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, n_vec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<true, false>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, n_vec, C);
  else if (res)
    hipLaunchKernelGGL((bn_apply_kernel<false, true>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, n_vec, C);
  else
    hipLaunchKernelGGL((bn_apply_kernel<false, false>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, n_vec, C);
}

void bn_act_backward(const uint16_t* dy, const uint16_t* x, const uint16_t* y, int64_t M, int C, const float* gamma,
                     const float* save, bool relu, float* dgamma, float* dbeta, float* coef, float* part,
                     uint16_t* dx, uint16_t* dres, hipStream_t stream) {
  int nblk;
  int64_t rpb;
  reduce_grid(M, C, &nblk, &rpb);
  GradOut o{gamma, save, dgamma, dbeta, coef};
  unsigned* cnt = next_counter(stream);
  if (relu)
    hipLaunchKernelGGL(bn_reduce_kernel<true>, dim3(nblk), dim3(kB), 0, stream, dy, x, y, M, C, rpb, part, cnt, o);
  else
    hipLaunchKernelGGL(bn_reduce_kernel<false>, dim3(nblk), dim3(kB), 0, stream, dy, x, y, M, C, rpb, part, cnt, o);
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  if (relu && dres)
    hipLaunchKernelGGL((bn_dx_kernel<true, true>), dim3(gb), dim3(kB), 0, stream, dy, x, y, coef, dx, dres, n_vec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_dx_kernel<true, false>), dim3(gb), dim3(kB), 0, stream, dy, x, y, coef, dx, dres, n_vec, C);
  else if (dres)
    hipLaunchKernelGGL((bn_dx_kernel<false, true>), dim3(gb), dim3(kB), 0, stream, dy, x, y, coef, dx, dres, n_vec, C);
  else
    hipLaunchKernelGGL((bn_dx_kernel<false, false>), dim3(gb), dim3(kB), 0, stream, dy, x, y, coef, dx, dres, n_vec, C);
}

}  // namespace grace
