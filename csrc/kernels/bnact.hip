// Fused training-mode BatchNorm (+ residual add) (+ ReLU) for channels_last bf16 activations.
//
// Why: in a ResNet-50 training step on MI355X the BN chain is the largest non-GEMM cost.  The
// stock path runs, per BN layer, MIOpen mean/var + final + normalise forward, a ReLU kernel, a
// residual add, a `num_batches_tracked += 1` kernel, and in backward a ReLU-backward, MIOpen
// dscale/dbias + final + dx, plus memsets (≈11 launches per layer, ~4.7 ms of a 9.4 ms step in
// profiles/r1_resnet50_topk_graph_bf16w_kernels.txt).  Here a layer is 4 kernels:
//
//   fwd  bn_stats   : per-channel Σx, Σx² (fp32 per thread, 16-B bf16 loads), one partial row
//                     per block, folded by an in-kernel ARRIVAL TREE; the final block writes
//                     mean/invstd, the folded affine (scale, shift), the running statistics
//                     and num_batches_tracked
//        bn_apply   : y = relu(x*scale + shift [+ residual]) -> bf16
//   bwd  bn_reduce  : Σdz, Σdz·(x-mean) with dz = dy·[y>0]; the final block writes dgamma,
//                     dbeta and the 3 per-channel coefficients of dx = a·dz + b·x + c
//        bn_dx      : dx (bf16) and, for the fused residual, d(residual) = dz (bf16)
//
// Layout: activations are [M = N·H·W rows, C channels] row-major (channels_last).  The two
// reduction kernels use a 2-D grid: blockIdx.x = chunk of rows, blockIdx.y = TILE of CT =
// min(C, 256) channels (a thread owns 8 consecutive channels = one 16-B load per row).  Each
// tile has its own two-level arrival tree (group finishers fold ~sqrt(#chunks) partial rows in
// fp64, the last group finisher folds the group totals), so the serial tails stay short and
// the large-C layers still get hundreds of blocks.  Fold order is fixed: deterministic.
//
// In-launch hand-offs follow the gfx950 publish/consume recipe (cdna_hip_programming.md
// Guideline 16): partial rows are stored WRITE-THROUGH (`sc1`, relaxed agent-scope atomic
// stores: no L2-writeback release fence), every storing wave drains (`s_waitcnt vmcnt(0)`),
// workgroup barrier, ONE lane adds to the arrival counter; only the finishing block pays ONE
// agent-scope acquire before its plain loads.  (Measured on MI355X: a `__threadfence()` in
// every thread of every block made these kernels 5-10x slower than their streaming bound; a
// flat one-block fold of 1024 partial rows, or fp64 atomics from 1024 blocks onto the same
// 2C addresses, cost 25-130 us per launch.)
//
// Constraints (host-checked, other shapes use the PyTorch path): C % 8 == 0, C <= 2048, and
// C % 256 == 0 when C > 256.
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kB = 256;           // threads per block
constexpr int kMaxC = 2048;
constexpr int kTileC = 256;       // channels per reduction tile (32 threads x 8 channels per row)
constexpr int kMaxTiles = kMaxC / kTileC;
constexpr int kMaxGroups = 64;
constexpr int kSlotWords = kMaxTiles * (kMaxGroups + 1);

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

template <typename T>
__device__ __forceinline__ void store_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Reduction-kernel geometry, computed on the host.
struct Red {
  int64_t M;           // rows
  int C;               // channels (row stride)
  int CT;              // channels per tile (= min(C, 256))
  int tprp;            // pow2 >= CT/8: thread slots per row
  int rpi;             // rows per block iteration = kB / tprp
  int64_t rows_per_blk;
  int nchunks;         // gridDim.x
  int gsize, ngroups;  // arrival tree: chunks per group, groups
  float* part;         // [tiles][nchunks][2*CT]
  double* gpart;       // [tiles][ngroups][2*CT]
  double* total;       // [tiles][2*CT]
  unsigned* cnt;       // [tiles][kMaxGroups + 1]: group counters, top counter last
};

// Column fold of `rows` rows (stride C2 elements) for the columns this thread owns, fp64,
// fixed order.  Thread t owns column t % C2 and rows r ≡ t / C2 (mod P) when C2 <= kB
// (P = kB / C2 row phases, combined through LDS by the caller), else columns t and t + kB.
template <typename T>
__device__ __forceinline__ void fold_cols(const T* src, int rows, int C2, double (&acc)[2]) {
  acc[0] = acc[1] = 0.0;
  if (C2 <= kB) {
    const int P = kB / C2, p = threadIdx.x / C2, c = threadIdx.x % C2;
    if (p >= P) return;
    int r = p;
    for (; r + 7 * P < rows; r += 8 * P) {  // 8 independent loads in flight
      T v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(r + u * P) * C2 + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[0] += (double)v[u];
    }
    for (; r < rows; r += P) acc[0] += (double)src[(size_t)r * C2 + c];
  } else {  // C2 == 2 * kB (CT = 256)
    const int c = threadIdx.x;
    int r = 0;
    for (; r + 3 < rows; r += 4) {
      T v[4][2];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u][0] = src[(size_t)(r + u) * C2 + c];
        v[u][1] = src[(size_t)(r + u) * C2 + c + kB];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc[0] += (double)v[u][0];
        acc[1] += (double)v[u][1];
      }
    }
    for (; r < rows; ++r) {
      acc[0] += (double)src[(size_t)r * C2 + c];
      acc[1] += (double)src[(size_t)r * C2 + c + kB];
    }
  }
}

// Fold + combine the row phases; calls put(col, value) once per column (all threads enter).
template <typename T, typename Put>
__device__ __forceinline__ void fold_block(const T* src, int rows, int C2, double* lds, Put put) {
  double acc[2];
  fold_cols(src, rows, C2, acc);
  if (C2 <= kB) {
    const int P = kB / C2;
    lds[threadIdx.x] = acc[0];
    __syncthreads();
    if (threadIdx.x < C2) {
      double v = lds[threadIdx.x];
      for (int i = 1; i < P; ++i) v += lds[i * C2 + threadIdx.x];
      put(threadIdx.x, v);
    }
    __syncthreads();
  } else {
    put(threadIdx.x, acc[0]);
    put(threadIdx.x + kB, acc[1]);
  }
}

// Every wave has drained its sc1 stores -> barrier -> one relaxed agent add.  True in every
// thread of the block whose add completed the count; that block is acquired (one lane's agent
// acquire + drain, then the barrier) before its plain loads.
__device__ __forceinline__ bool arrive(unsigned* counter, unsigned expected_last) {
  __shared__ int flag;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = (prev == expected_last);
    if (flag) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return flag != 0;
}

// Per-thread 8-channel accumulators -> this block's partial row -> the tile's arrival tree.
// True in every thread of the tile's final block; totals then in total[tile][0..2CT).
__device__ bool block_reduce_tree(const Red& R, const float* a, const float* b) {
  __shared__ float sa[kB * 8];
  __shared__ float sb[kB * 8];
  __shared__ double lds[kB];
  const int CT = R.CT, C2 = 2 * CT, tile = blockIdx.y;
  const int cg = threadIdx.x % R.tprp, rs = threadIdx.x / R.tprp;
  if (cg < CT / 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sa[rs * CT + cg * 8 + j] = a[j];
      sb[rs * CT + cg * 8 + j] = b[j];
    }
  }
  __syncthreads();
  float* part = R.part + (size_t)tile * R.nchunks * C2;
  float* pb = part + (size_t)blockIdx.x * C2;
  for (int c = threadIdx.x; c < CT; c += kB) {
    float x = 0.f, y = 0.f;
    for (int i = 0; i < R.rpi; ++i) {
      x += sa[i * CT + c];
      y += sb[i * CT + c];
    }
    store_sc1(pb + c, x);
    store_sc1(pb + CT + c, y);
  }
  unsigned* cnt = R.cnt + tile * (kMaxGroups + 1);
  const int grp = blockIdx.x / R.gsize, g0 = grp * R.gsize;
  const int grows = min(R.nchunks - g0, R.gsize);
  if (!arrive(cnt + grp, (unsigned)grows - 1)) return false;
  double* gpart = R.gpart + (size_t)tile * R.ngroups * C2;
  fold_block(part + (size_t)g0 * C2, grows, C2, lds,
             [&](int c, double v) { store_sc1(gpart + (size_t)grp * C2 + c, v); });
  if (!arrive(cnt + kMaxGroups, (unsigned)R.ngroups - 1)) return false;
  double* total = R.total + (size_t)tile * C2;
  fold_block(gpart, R.ngroups, C2, lds, [&](int c, double v) { total[c] = v; });
  __syncthreads();
  for (int i = threadIdx.x; i <= kMaxGroups; i += kB) cnt[i] = 0;  // re-arm (visible at kernel end)
  return true;
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

// Row loop shared by the two reduction kernels: body(element_offset, row_step, n) for this
// thread's rows of the block's chunk, 4 rows per call (independent loads in flight), then 1.
template <typename Body>
__device__ __forceinline__ void for_rows(const Red& R, Body body) {
  const int cg = threadIdx.x % R.tprp, rs = threadIdx.x / R.tprp;
  if (cg >= R.CT / 8) return;
  const int64_t r0 = (int64_t)blockIdx.x * R.rows_per_blk;
  const int64_t r1 = min(R.M, r0 + R.rows_per_blk);
  const int64_t col = (int64_t)blockIdx.y * R.CT + cg * 8;
  int64_t r = r0 + rs;
  for (; r + 3 * R.rpi < r1; r += 4 * R.rpi) body(r * R.C + col, R.rpi * (int64_t)R.C, 4);
  for (; r < r1; r += R.rpi) body(r * R.C + col, (int64_t)0, 1);
}

__global__ __launch_bounds__(kB) void bn_stats_kernel(const uint16_t* __restrict__ x, Red R, StatsOut o) {
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  for_rows(R, [&](int64_t e, int64_t step, int n) {
    if (n == 4) {
      Bf8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = load_bf8(x + e + u * step);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += v[u].v[j];
          q[j] = fmaf(v[u].v[j], v[u].v[j], q[j]);
        }
    } else {
      const Bf8 v = load_bf8(x + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v.v[j];
        q[j] = fmaf(v.v[j], v.v[j], q[j]);
      }
    }
  });
  if (!block_reduce_tree(R, s, q)) return;
  const int CT = R.CT, C = R.C;
  const double* total = R.total + (size_t)blockIdx.y * 2 * CT;
  const double inv_m = 1.0 / (double)R.M;
  const double unbias = R.M > 1 ? (double)R.M / (double)(R.M - 1) : 1.0;
  for (int cl = threadIdx.x; cl < CT; cl += kB) {
    const int c = blockIdx.y * CT + cl;
    const double mean = total[cl] * inv_m;
    const double var = fmax(total[CT + cl] * inv_m - mean * mean, 0.0);
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
  }
  if (threadIdx.x == 0 && blockIdx.y == 0 && o.nbt) *o.nbt += 1;
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
                                                       const uint16_t* __restrict__ y, Red R, GradOut o) {
  float s1[8], s2[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = mu[j] = 0.f;
  {
    const int cg = threadIdx.x % R.tprp;
    if (cg < R.CT / 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) mu[j] = o.save[blockIdx.y * R.CT + cg * 8 + j];
    }
  }
  auto acc = [&](const Bf8& d, const Bf8& v, const Bf8& w) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dz = d.v[j];
      if constexpr (RELU) dz = w.v[j] > 0.f ? dz : 0.f;
      s1[j] += dz;
      s2[j] = fmaf(dz, v.v[j] - mu[j], s2[j]);
    }
  };
  for_rows(R, [&](int64_t e, int64_t step, int n) {
    if (n == 4) {
      Bf8 d[4], v[4], w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        d[u] = load_bf8(dy + e + u * step);
        v[u] = load_bf8(x + e + u * step);
        if constexpr (RELU) w[u] = load_bf8(y + e + u * step);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc(d[u], v[u], w[u]);
    } else {
      const Bf8 d = load_bf8(dy + e), v = load_bf8(x + e);
      Bf8 w;
      if constexpr (RELU) w = load_bf8(y + e);
      acc(d, v, w);
    }
  });
  if (!block_reduce_tree(R, s1, s2)) return;
  const int CT = R.CT, C = R.C;
  const double* total = R.total + (size_t)blockIdx.y * 2 * CT;
  const double inv_m = 1.0 / (double)R.M;
  for (int cl = threadIdx.x; cl < CT; cl += kB) {
    const int c = blockIdx.y * CT + cl;
    const double S1 = total[cl], S2 = total[CT + cl];
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
  }
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

// ---------------------------------------------------------------- host-side geometry
// Arrival counters: a device pool of per-launch slots (kSlotWords counters each) taken
// round-robin; the final blocks re-arm their tile's counters, so graph replays reuse a slot and
// BN kernels running concurrently never share one.  Zeroed once at allocation.
constexpr int kSlots = 256;
struct Slots {
  unsigned* counters = nullptr;
  int next = 0;
};
Slots g_slots[64];

unsigned* next_slot(hipStream_t stream) {
  int dev = 0;
  GRACE_HIP_CHECK(hipGetDevice(&dev));
  Slots& p = g_slots[dev];
  if (!p.counters) {  // first use happens eagerly (warm-up), never inside a graph capture
    GRACE_HIP_CHECK(hipMalloc(&p.counters, (size_t)kSlots * kSlotWords * sizeof(unsigned)));
    GRACE_HIP_CHECK(hipMemsetAsync(p.counters, 0, (size_t)kSlots * kSlotWords * sizeof(unsigned), stream));
    GRACE_HIP_CHECK(hipStreamSynchronize(stream));
  }
  const int s = p.next;
  p.next = (s + 1) % kSlots;
  return p.counters + (size_t)s * kSlotWords;
}

// Grid and tree shape.  Target >= ~512 blocks (2 per CU) with 4..16 16-B vectors per thread.
Red plan(int64_t M, int C) {
  Red R{};
  R.M = M;
  R.C = C;
  R.CT = C < kTileC ? C : kTileC;
  const int tiles = C / R.CT;
  R.tprp = 1;
  while (R.tprp < R.CT / 8) R.tprp <<= 1;
  R.rpi = kB / R.tprp;
  const int64_t n_vec = M * C / 8;
  int64_t vpt = n_vec / ((int64_t)kB * 512);
  if (vpt < 4) vpt = 4;
  if (vpt > 16) vpt = 16;
  const int64_t per_blk = R.rpi * vpt;
  int64_t nc = (M + per_blk - 1) / per_blk;
  if (nc * tiles > 2048) nc = (2048 + tiles - 1) / tiles;
  if (nc < 1) nc = 1;
  int64_t rpb = (M + nc - 1) / nc;
  rpb = (rpb + R.rpi - 1) / R.rpi * R.rpi;
  nc = (M + rpb - 1) / rpb;
  R.rows_per_blk = rpb;
  R.nchunks = (int)(nc < 1 ? 1 : nc);
  int gs = 1;
  while (gs * gs < R.nchunks) ++gs;
  int ng = (R.nchunks + gs - 1) / gs;
  while (ng > kMaxGroups) {
    ++gs;
    ng = (R.nchunks + gs - 1) / gs;
  }
  R.gsize = gs;
  R.ngroups = ng;
  return R;
}

int64_t even(int64_t n) { return (n + 1) & ~(int64_t)1; }

int64_t ws_floats(const Red& R) {
  const int tiles = R.C / R.CT, C2 = 2 * R.CT;
  return even((int64_t)tiles * R.nchunks * C2) + 2 * (int64_t)tiles * (R.ngroups + 1) * C2;
}

void bind_ws(Red& R, float* ws, hipStream_t stream) {
  const int tiles = R.C / R.CT, C2 = 2 * R.CT;
  R.part = ws;
  R.gpart = reinterpret_cast<double*>(ws + even((int64_t)tiles * R.nchunks * C2));  // 8-B aligned
  R.total = R.gpart + (size_t)tiles * R.ngroups * C2;
  R.cnt = next_slot(stream);
}

int apply_grid(int64_t n_vec, int C) {
  const int64_t tpr = C / 8;
  int64_t b = (n_vec + kB - 1) / kB;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  // the grid stride must be a multiple of tpr: round the grid to a multiple of tpr / gcd(tpr, kB)
  int64_t g = tpr, h = kB;
  while (h) {
    const int64_t t = g % h;
    g = h;
    h = t;
  }
  const int64_t m = tpr / g;
  return (int)((b + m - 1) / m * m);
}

}  // namespace

bool bn_supported(int C) { return C > 0 && C % 8 == 0 && C <= kMaxC && (C <= kTileC || C % kTileC == 0); }

int64_t bn_workspace_floats(int64_t M, int C) { return ws_floats(plan(M, C)); }

void bn_act_forward(const uint16_t* x, const uint16_t* res, int64_t M, int C, const float* gamma, const float* beta,
                    float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps, bool relu,
                    float* save, float* ws, uint16_t* y, hipStream_t stream) {
  Red R = plan(M, C);
  bind_ws(R, ws, stream);
  StatsOut o{gamma, beta, running_mean, running_var, nbt, momentum, eps, save};
  hipLaunchKernelGGL(bn_stats_kernel, dim3(R.nchunks, C / R.CT), dim3(kB), 0, stream, x, R, o);
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
                     const float* save, bool relu, float* dgamma, float* dbeta, float* coef, float* ws,
                     uint16_t* dx, uint16_t* dres, hipStream_t stream) {
  Red R = plan(M, C);
  bind_ws(R, ws, stream);
  GradOut o{gamma, save, dgamma, dbeta, coef};
  const dim3 grid(R.nchunks, C / R.CT);
  if (relu)
    hipLaunchKernelGGL(bn_reduce_kernel<true>, grid, dim3(kB), 0, stream, dy, x, y, R, o);
  else
    hipLaunchKernelGGL(bn_reduce_kernel<false>, grid, dim3(kB), 0, stream, dy, x, y, R, o);
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
