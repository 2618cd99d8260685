// Fused training-mode BatchNorm (+ residual add) (+ ReLU) for channels_last bf16 or fp32 activations.
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
// workgroup barrier, ONE lane adds to the arrival counter; the finishing block reads the rows
// with `sc1` loads only, so it pays no acquire fence either (round 2: the acquire was ~1.7 us
// per tree level, two levels per reduction kernel, 106 reduction kernels per ResNet-50 step).  (Measured on MI355X: a `__threadfence()` in
// every thread of every block made these kernels 5-10x slower than their streaming bound; a
// flat one-block fold of 1024 partial rows, or fp64 atomics from 1024 blocks onto the same
// 2C addresses, cost 25-130 us per launch.)
//
// Constraints (host-checked, other shapes use the PyTorch path): C % 8 == 0, C <= 2048, and
// C % 256 == 0 when C > 256.
#include <cstdlib>
#include <type_traits>

#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kB = 256;           // threads per block
constexpr int kMaxC = 2048;
constexpr int kTileC = 256;       // channels per reduction tile (32 threads x 8 channels per row)
constexpr int kMaxTiles = kMaxC / kTileC;
constexpr int kMaxGroups = 64;
constexpr int kTreeWords = kMaxTiles * (kMaxGroups + 1);
constexpr int kSlotWords = kTreeWords + 2 * kMaxTiles;  // + per-tile generation word (+ pad)

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

__device__ __forceinline__ uint4 pack_bf8(const float* v) {
  uint4 u;
  u.x = (uint32_t)f32_to_bf16_rne(v[0]) | ((uint32_t)f32_to_bf16_rne(v[1]) << 16);
  u.y = (uint32_t)f32_to_bf16_rne(v[2]) | ((uint32_t)f32_to_bf16_rne(v[3]) << 16);
  u.z = (uint32_t)f32_to_bf16_rne(v[4]) | ((uint32_t)f32_to_bf16_rne(v[5]) << 16);
  u.w = (uint32_t)f32_to_bf16_rne(v[6]) | ((uint32_t)f32_to_bf16_rne(v[7]) << 16);
  return u;
}

// ReLU mask of 8 packed bf16 outputs: bit j = (y_j > 0), i.e. 0 < bits <= +inf (the fp32
// compare `y > 0.f` on the rounded output, NaNs excluded).  The backward reads these 1-bit
// masks (M*C/8 bytes) instead of the bf16 output (2*M*C bytes) in both of its passes.
__device__ __forceinline__ uint32_t pos_bits(uint32_t w) {
  return ((w & 0xffffu) - 1u < 0x7f80u ? 1u : 0u) | ((w >> 16) - 1u < 0x7f80u ? 2u : 0u);
}
__device__ __forceinline__ uint8_t relu_byte(const uint4 u) {
  return (uint8_t)(pos_bits(u.x) | (pos_bits(u.y) << 2) | (pos_bits(u.z) << 4) | (pos_bits(u.w) << 6));
}
// mask byte -> per-dword AND masks for the packed bf16 pairs (channels 2k, 2k+1)
__device__ __forceinline__ uint32_t pair_mask(uint32_t mb, int k) {
  return ((mb >> (2 * k)) & 1u ? 0x0000ffffu : 0u) | ((mb >> (2 * k + 1)) & 1u ? 0xffff0000u : 0u);
}

// Element-type generic 8-channel row vectors for the two-kernel path: bf16 (one 16-B load) or
// fp32 (two 16-B loads; the reference harness trains in fp32).
__device__ __forceinline__ Bf8 ld8(const uint16_t* p) { return load_bf8(p); }
__device__ __forceinline__ Bf8 ld8(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  Bf8 r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}
__device__ __forceinline__ void st8(uint16_t* p, const float* v) { store_bf8(p, v); }
__device__ __forceinline__ void st8(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
// store y and return its ReLU mask byte (taken from the value as stored, like threshold_backward)
__device__ __forceinline__ uint8_t st8_mask(uint16_t* p, const float* v) {
  const uint4 u = pack_bf8(v);
  *reinterpret_cast<uint4*>(p) = u;
  return relu_byte(u);
}
__device__ __forceinline__ uint8_t st8_mask(float* p, const float* v) {
  st8(p, v);
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) b |= (v[j] > 0.f ? 1u : 0u) << j;
  return (uint8_t)b;
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
  float* ftot;         // forward statistics in ATOMIC mode: [2C] self-cleaning totals of the slot, or null
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-B `sc1` load (buffer instruction, aux 16 = sc1: L1 bypassed, L2-served) of a row that
// another workgroup stored `sc1` and drained before its arrival add.  Every load of the
// published partial rows is one of these, which is what lets the finisher skip the agent-scope
// acquire (cdna_hip_programming.md §6 Guideline 16; MI355X_MICROARCH.md "Valid forms", first
// row of the sc1 hand-off table: ≈1.7 us per acquire, two per reduction kernel).
template <typename V>
__device__ __forceinline__ V ld16_sc1(const void* base, int64_t bytes, int off) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
  const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
  return __builtin_bit_cast(V, w);
}

// Column fold of `rows` rows (row stride C2 elements, 16-B aligned) into fp64, fixed order.
// The rows were published by other blocks (possibly on other XCDs) with write-through stores
// and are read with sc1 loads, so every load misses the local L2: the fold is latency bound and
// issues ALL of a thread's loads before the first use.  16-B loads: thread t owns vector column g = t % G (G = C2 / VW) and the rows
// r = t / G (mod P), P = kB / G row phases (unrolled by U, independent); the phases are combined
// through LDS (lds: kB * VW doubles) in phase order, so the result is run-to-run deterministic.
// Calls put(col, value) once per column (all threads enter).
template <typename T, typename Put>
__device__ __forceinline__ void fold_block(const T* src, int rows, int C2, double* lds, Put put) {
  constexpr int VW = 16 / sizeof(T);
  constexpr int U = 16 / (sizeof(T) / 4);  // 16 float4 or 8 double2 loads in flight
  using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
  const int G = C2 / VW, P = kB / G;  // C2 <= 512: G <= 128 (float), 256 (double)
  const int g = threadIdx.x % G, p = threadIdx.x / G;
  double acc[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) acc[j] = 0.0;
  if (p < P) {
    const int64_t bytes = (int64_t)rows * C2 * (int64_t)sizeof(T);
    for (int r = p; r < rows; r += U * P) {  // predicated: a short fold is still ONE round trip
      V v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + u * P;
        if (rr < rows) v[u] = ld16_sc1<V>(src, bytes, (int)(((int64_t)rr * C2 + (int64_t)g * VW) * (int64_t)sizeof(T)));
        else v[u] = V{};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const T* e = reinterpret_cast<const T*>(&v[u]);
#pragma unroll
        for (int j = 0; j < VW; ++j) acc[j] += (double)e[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VW; ++j) lds[threadIdx.x * VW + j] = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C2; c += kB) {
    const int gc = c / VW, j = c % VW;
    double v = 0.0;
    for (int i = 0; i < P; ++i) v += lds[(i * G + gc) * VW + j];
    put(c, v);
  }
  __syncthreads();
}

// Every wave has drained its sc1 stores -> barrier -> one relaxed agent add.  True in every
// thread of the block whose add completed the count; its waves load the published rows only
// after the barrier that follows the add's return, and only with sc1 loads (fold_block), so no
// acquire fence is needed.
__device__ __forceinline__ bool arrive(unsigned* counter, unsigned expected_last) {
  __shared__ int flag;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = (prev == expected_last);
  }
  __syncthreads();
  return flag != 0;
}

// Per-thread 8-channel accumulators -> this block's partial row -> the tile's arrival tree.
// True in every thread of the tile's final block; totals then in total[tile][0..2CT).
// atot != nullptr (the backward's ATOMIC mode): the block's partial row is added into atot[0..2C)
// with fp32 no-return atomics instead of being stored and folded; one arrival per block, the
// tile's last block reads the totals (no partial-row fold) and finishes as the tree does.
__device__ bool block_reduce_tree(const Red& R, const float* a, const float* b, float* atot = nullptr) {
  __shared__ __align__(16) float sa[kB * 8];
  __shared__ float sb[kB * 8];
  double* lds = reinterpret_cast<double*>(sa);  // fold scratch (kB * 4 doubles), after sa is consumed
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
  if (atot != nullptr) {
    for (int c = threadIdx.x; c < CT; c += kB) {
      float x = 0.f, y = 0.f;
      for (int i = 0; i < R.rpi; ++i) {
        x += sa[i * CT + c];
        y += sb[i * CT + c];
      }
      const int cc = tile * CT + c;
      __hip_atomic_fetch_add(atot + cc, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(atot + R.C + cc, y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // one arrival per block (the drain inside arrive() covers the no-return atomics); the tile's
    // last block reads the totals (device-scope loads: never a stale L1 line), re-zeroes them and
    // finishes exactly like the tree's finisher (coefficients, dgamma / dbeta)
    unsigned* top = R.cnt + tile * (kMaxGroups + 1) + kMaxGroups;
    if (!arrive(top, (unsigned)R.nchunks - 1)) return false;
    double* total = R.total + (size_t)tile * C2;
    for (int c = threadIdx.x; c < CT; c += kB) {
      const int cc = tile * CT + c;
      total[c] = (double)__hip_atomic_load(atot + cc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      total[CT + c] = (double)__hip_atomic_load(atot + R.C + cc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atot[cc] = 0.f;
      atot[R.C + cc] = 0.f;
    }
    __syncthreads();
    if (threadIdx.x == 0) *top = 0;  // re-arm (visible at kernel end)
    return true;
  }
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
  if (R.ngroups == 1) {  // one-level tree: the only group's finisher is the tile's finisher
    double* total = R.total + (size_t)tile * C2;
    fold_block(part, grows, C2, lds, [&](int c, double v) { total[c] = v; });
    __syncthreads();
    if (threadIdx.x == 0) cnt[0] = 0;  // re-arm (visible at kernel end)
    return true;
  }
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

template <typename T>
__global__ __launch_bounds__(kB) void bn_stats_kernel(const T* __restrict__ x, Red R, StatsOut o) {
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  for_rows(R, [&](int64_t e, int64_t step, int n) {
    if (n == 4) {
      Bf8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ld8(x + e + u * step);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += v[u].v[j];
          q[j] = fmaf(v[u].v[j], v[u].v[j], q[j]);
        }
    } else {
      const Bf8 v = ld8(x + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v.v[j];
        q[j] = fmaf(v.v[j], v.v[j], q[j]);
      }
    }
  });
  if (!block_reduce_tree(R, s, q, R.ftot)) return;
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
    o.save[4 * C + c] = 0.f;  // the backward's atomic totals (bn_reduce_kernel ATOMIC mode)
    o.save[5 * C + c] = 0.f;
    if (o.running_mean) {
      o.running_mean[c] = (1.f - o.momentum) * o.running_mean[c] + o.momentum * (float)mean;
      o.running_var[c] = (1.f - o.momentum) * o.running_var[c] + o.momentum * (float)(var * unbias);
    }
  }
  if (threadIdx.x == 0 && blockIdx.y == 0 && o.nbt) *o.nbt += 1;
}

// y = act(x*scale + shift [+ res]); scale/shift = save[2C..4C)
template <typename T, bool RELU, bool RES>
__global__ __launch_bounds__(kB) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                      const float* __restrict__ save, T* __restrict__ y,
                                                      uint8_t* __restrict__ mask, int64_t n_vec, int C) {
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
    const Bf8 v = ld8(x + i * 8);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(v.v[j], sc[j], sh[j]);
    if constexpr (RES) {
      const Bf8 r = ld8(res + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += r.v[j];
    }
    if constexpr (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
    }
    if constexpr (RELU) mask[i] = st8_mask(y + i * 8, o);
    else st8(y + i * 8, o);
  }
}

struct GradOut {
  const float* gamma;  // may be null
  const float* save;   // [4C] from the forward
  float* dgamma;       // may be null
  float* dbeta;        // may be null
  float* coef;         // [3C]: a, b, c with dx = a*dz + b*x + c
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
// 8 channels of one row through a buffer descriptor (voff: per-thread bytes, soff: uniform)
template <typename T>
__device__ __forceinline__ Bf8 bld8(__amdgpu_buffer_rsrc_t r, int voff, int soff);
template <>
__device__ __forceinline__ Bf8 bld8<float>(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16, soff, 0);
  Bf8 o;
  o.v[0] = __uint_as_float(a.x); o.v[1] = __uint_as_float(a.y); o.v[2] = __uint_as_float(a.z); o.v[3] = __uint_as_float(a.w);
  o.v[4] = __uint_as_float(b.x); o.v[5] = __uint_as_float(b.y); o.v[6] = __uint_as_float(b.z); o.v[7] = __uint_as_float(b.w);
  return o;
}
template <>
__device__ __forceinline__ Bf8 bld8<uint16_t>(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  Bf8 o;
  o.v[0] = __uint_as_float(u.x << 16); o.v[1] = __uint_as_float(u.x & 0xffff0000u);
  o.v[2] = __uint_as_float(u.y << 16); o.v[3] = __uint_as_float(u.y & 0xffff0000u);
  o.v[4] = __uint_as_float(u.z << 16); o.v[5] = __uint_as_float(u.z & 0xffff0000u);
  o.v[6] = __uint_as_float(u.w << 16); o.v[7] = __uint_as_float(u.w & 0xffff0000u);
  return o;
}

// DY2: the layer's output fed two consumers (a block output -> the next block's conv and its
// shortcut) and autograd hands the two gradient contributions over separately
// (ops/bnact.py `dual`): dy = dy + dy2 is summed here instead of in a separate add kernel.
template <typename T>
__device__ __forceinline__ void add8(Bf8& d, const T* p) {
  const Bf8 e = ld8(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) d.v[j] += e.v[j];
}

// RX (with RELU): no saved mask -- the ReLU mask is recomputed from x as fmaf(x, scale, shift)
// > 0, the exact expression the forward apply thresholds (the fused stem's forward writes no
// mask: ops/bnact.py bn_relu_maxpool).
// WDZ: also store dz = [y > 0] (dy + dy2) (the residual input's gradient of a block-output BN):
// the dx pass then reads dz and x only (bn_dx_dz_kernel) and dz IS d(residual) -- 7 activation
// passes per layer instead of 8 (dy, dy2 and the mask read once, d(residual) not rewritten).
template <typename T, bool RELU, bool DY2, bool RX = false, bool WDZ = false>
__global__ __launch_bounds__(kB) void bn_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                       const T* __restrict__ x,
                                                       const uint8_t* __restrict__ mask, Red R, GradOut o,
                                                       T* __restrict__ dzout = nullptr, float* atot = nullptr) {
  float s1[8], s2[8], mu[8], rsc[8], rsh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = mu[j] = rsc[j] = rsh[j] = 0.f;
  {
    const int cg = threadIdx.x % R.tprp;
    if (cg < R.CT / 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mu[j] = o.save[blockIdx.y * R.CT + cg * 8 + j];
        if constexpr (RX) {
          rsc[j] = o.save[2 * R.C + blockIdx.y * R.CT + cg * 8 + j];
          rsh[j] = o.save[3 * R.C + blockIdx.y * R.CT + cg * 8 + j];
        }
      }
    }
  }
  auto acc = [&](const Bf8& d, const Bf8& v, uint32_t mb, T* dzp) {
    float z[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float dz = d.v[j];
      if constexpr (RELU && RX) dz = fmaf(v.v[j], rsc[j], rsh[j]) > 0.f ? dz : 0.f;
      else if constexpr (RELU) dz = (mb >> j) & 1u ? dz : 0.f;
      z[j] = dz;
      s1[j] += dz;
      s2[j] = fmaf(dz, v.v[j] - mu[j], s2[j]);
    }
    if constexpr (WDZ) st8(dzp, z);
  };
  // The 4-row batches address every operand through a buffer descriptor based at the block's
  // first row: one 32-bit VGPR offset per thread, the row step as a wave-uniform soffset.  With
  // flat 64-bit addresses each of the (up to) 24 in-flight 16-B loads of the two-gradient fp32
  // variant held its own VGPR pair and hipcc serialised the loads to stay within 128 VGPRs.
  const int64_t blk0 = (int64_t)blockIdx.x * R.rows_per_blk * R.C;  // element offset of the chunk
  const int64_t left = (R.M * (int64_t)R.C - blk0) * (int64_t)sizeof(T);
  const int nrec = (int)(left < 0x7fffffff ? left : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t rdy = brsrc(dy + blk0, nrec), rx = brsrc(x + blk0, nrec);
  const __amdgpu_buffer_rsrc_t rdy2 = brsrc(DY2 ? dy2 + blk0 : dy + blk0, nrec);
  for_rows(R, [&](int64_t e, int64_t step, int n) {
    if (n == 4) {
      const int vo = (int)((e - blk0) * (int64_t)sizeof(T));
      const int so = (int)(step * (int64_t)sizeof(T));
      Bf8 d[4], v[4];
      uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        d[u] = bld8<T>(rdy, vo, u * so);
        v[u] = bld8<T>(rx, vo, u * so);
        if constexpr (RELU && !RX) w[u] = mask[(e + u * step) >> 3];
      }
      if constexpr (DY2) {
        Bf8 d2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) d2[u] = bld8<T>(rdy2, vo, u * so);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) d[u].v[j] += d2[u].v[j];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc(d[u], v[u], w[u], WDZ ? dzout + e + u * step : nullptr);
    } else {
      Bf8 d = ld8(dy + e);
      const Bf8 v = ld8(x + e);
      if constexpr (DY2) add8(d, dy2 + e);
      uint32_t w = 0;
      if constexpr (RELU && !RX) w = mask[e >> 3];
      acc(d, v, w, WDZ ? dzout + e : nullptr);
    }
  });
  if (!block_reduce_tree(R, s1, s2, atot)) return;
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

// A dx pass's per-channel coefficients (dx = a*dz + b*x + c), written by the reduce kernel's
// finisher (tree or atomic totals), plus the forward's save (the RX variant's scale / shift).
struct CoefSrc {
  const float* coef;  // [3C]
  const float* save;  // [6C] forward save: mean, invstd, scale, shift, atomic totals [2C]
};

__device__ __forceinline__ void get_coef(const CoefSrc& s, int C, int c0, float* ca, float* cb, float* cc) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ca[j] = s.coef[c0 + j];
    cb[j] = s.coef[C + c0 + j];
    cc[j] = s.coef[2 * C + c0 + j];
  }
}

template <typename T, bool RELU, bool RES, bool DY2, bool RX = false>
__global__ __launch_bounds__(kB) void bn_dx_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                   const T* __restrict__ x,
                                                   const uint8_t* __restrict__ mask, CoefSrc cs,
                                                   T* __restrict__ dx, T* __restrict__ dres,
                                                   int64_t n_vec, int C) {
  const int tpr = C >> 3;
  const int64_t stride = (int64_t)gridDim.x * kB;
  int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int cg = (int)(i % tpr);
  float ca[8], cb[8], cc[8], rsc[8], rsh[8];
  get_coef(cs, C, cg * 8, ca, cb, cc);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    rsc[j] = RX ? cs.save[2 * C + cg * 8 + j] : 0.f;
    rsh[j] = RX ? cs.save[3 * C + cg * 8 + j] : 0.f;
  }
  for (; i < n_vec; i += stride) {
    Bf8 d = ld8(dy + i * 8);
    const Bf8 v = ld8(x + i * 8);
    if constexpr (DY2) add8(d, dy2 + i * 8);
    float dz[8], o[8];
    if constexpr (RELU && RX) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = fmaf(v.v[j], rsc[j], rsh[j]) > 0.f ? d.v[j] : 0.f;
    } else if constexpr (RELU) {
      const uint32_t mb = mask[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = (mb >> j) & 1u ? d.v[j] : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = d.v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(ca[j], dz[j], fmaf(cb[j], v.v[j], cc[j]));
    st8(dx + i * 8, o);
    if constexpr (RES) st8(dres + i * 8, dz);
  }
}


// dx = a*dz + b*x + c with dz already masked and summed (written by bn_reduce_kernel<WDZ>)
template <typename T>
__global__ __launch_bounds__(kB) void bn_dx_dz_kernel(const T* __restrict__ dz, const T* __restrict__ x,
                                                      CoefSrc cs, T* __restrict__ dx, int64_t n_vec, int C) {
  const int tpr = C >> 3;
  const int64_t stride = (int64_t)gridDim.x * kB;
  int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int cg = (int)(i % tpr);
  float ca[8], cb[8], cc[8];
  get_coef(cs, C, cg * 8, ca, cb, cc);
  for (; i < n_vec; i += stride) {
    const Bf8 d = ld8(dz + i * 8);
    const Bf8 v = ld8(x + i * 8);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(ca[j], d.v[j], fmaf(cb[j], v.v[j], cc[j]));
    st8(dx + i * 8, o);
  }
}

// ---------------------------------------------------------------- conv bias (+ ReLU)
// VGG's conv -> bias -> ReLU (MIOpen returns the conv without its bias: PyTorch then runs a
// broadcast add, a ReLU, and in backward threshold_backward plus a bias-gradient reduction --
// four full activation passes and three launches around every conv).  Here: forward = one
// streaming pass y = act(x + b); backward = ONE pass that writes dz = dy * [y > 0] and reduces
// Σdz per channel into the bias gradient through the same two-level arrival tree as the BN
// statistics (deterministic fp64 fold).
template <typename T, bool RELU>
__global__ __launch_bounds__(kB) void bias_act_fwd_kernel(const T* __restrict__ x, const float* __restrict__ bias,
                                                          T* __restrict__ y, int64_t n_vec, int C) {
  const int tpr = C >> 3;
  const int64_t stride = (int64_t)gridDim.x * kB;
  int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
  const int cg = (int)(i % tpr);  // stride % tpr == 0 (apply_grid)
  float b[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = bias[cg * 8 + j];
  for (; i < n_vec; i += stride) {
    const Bf8 v = ld8(x + i * 8);
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = RELU ? fmaxf(v.v[j] + b[j], 0.f) : v.v[j] + b[j];
    st8(y + i * 8, o);
  }
}

template <typename T, bool RELU>
__global__ __launch_bounds__(kB) void bias_act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                          T* __restrict__ dz, Red R, float* __restrict__ dbias) {
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  auto one = [&](const Bf8& d, const Bf8& v, T* out) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = (!RELU || v.v[j] > 0.f) ? d.v[j] : 0.f;
      s[j] += o[j];
    }
    st8(out, o);
  };
  for_rows(R, [&](int64_t e, int64_t step, int n) {
    if (n == 4) {
      Bf8 d[4], v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        d[u] = ld8(dy + e + u * step);
        if constexpr (RELU) v[u] = ld8(y + e + u * step);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) one(d[u], v[u], dz + e + u * step);
    } else {
      const Bf8 d = ld8(dy + e);
      Bf8 v{};
      if constexpr (RELU) v = ld8(y + e);
      one(d, v, dz + e);
    }
  });
  if (!block_reduce_tree(R, s, s, R.ftot)) return;  // atomic totals (self-cleaning slot) or the tree
  const double* total = R.total + (size_t)blockIdx.y * 2 * R.CT;
  for (int cl = threadIdx.x; cl < R.CT; cl += kB) dbias[blockIdx.y * R.CT + cl] = (float)total[cl];
}

// ---------------------------------------------------------------- BN + ReLU + max pool (stem)
// The ResNet stem runs conv -> BN -> ReLU -> 3x3/2 max pool: the BN output (the largest
// activation of the network, 103 MB fp32 at batch 32) is written only to be re-read by the pool,
// Fused forward = stats + ONE pass that normalises, applies the ReLU and pools straight from x
// (writes the pooled tensor and a 1-byte in-window argmax per pooled element; no BN output, no
// ReLU mask).  Backward = the gather max-pool backward (pool.hip) + the two BN passes with the
// ReLU mask recomputed from x (RX).  (Gathering dz inside the BN passes instead was measured
// slower: 159 vs 94 us -- per-row dependent code/gradient loads serialise the reduction.)
// Pool semantics as ops/pool.py.
struct PoolShape {
  int H, W, OH, OW, k, s, pad;
};

template <typename T>
__global__ __launch_bounds__(kB) void bn_pool_apply_kernel(const T* __restrict__ x, const float* __restrict__ save,
                                                           T* __restrict__ y, uint8_t* __restrict__ code, PoolShape g,
                                                           int C, int64_t n_vec) {
  const int cv = C >> 3;
  for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n_vec; i += (int64_t)gridDim.x * kB) {
    const int c8 = (int)(i % cv);
    const int64_t pix = i / cv;
    const int ow = (int)(pix % g.OW);
    const int oh = (int)((pix / g.OW) % g.OH);
    const int64_t n = pix / ((int64_t)g.OW * g.OH);
    float sc[8], sh[8], m[8];
    uint32_t arg[8];
    const int h0 = oh * g.s - g.pad, w0 = ow * g.s - g.pad;
    const uint32_t first = (uint32_t)(max(0, -h0) * g.k + max(0, -w0));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = save[2 * C + c8 * 8 + j];
      sh[j] = save[3 * C + c8 * 8 + j];
      m[j] = -INFINITY;
      arg[j] = first;
    }
    for (int kh = 0; kh < g.k; ++kh) {
      const int h = h0 + kh;
      if (h < 0 || h >= g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int w = w0 + kw;
        if (w < 0 || w >= g.W) continue;
        const Bf8 v = ld8(x + (((n * g.H + h) * g.W + w) * C + c8 * 8));
        const uint32_t pos = (uint32_t)(kh * g.k + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = fmaxf(fmaf(v.v[j], sc[j], sh[j]), 0.f);
          const bool take = (o > m[j]) || (o != o);
          m[j] = take ? o : m[j];
          arg[j] = take ? pos : arg[j];
        }
      }
    }
    st8(y + i * 8, m);
    uint2 packed;
    packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    *reinterpret_cast<uint2*>(code + i * 8) = packed;
  }
}

// ---------------------------------------------------------------- single-launch variants
// For the small/medium layers (ResNet-50 stages 2-4: 0.4-8 M elements) a BN pass is latency
// bound: two launches, each with a serial reduction tail, for a few MB of data.  The fused
// kernels keep the block's rows in REGISTERS (V 16-B vectors per thread per operand), run the
// same arrival tree, and then every block waits for its tile's finisher to publish the
// per-channel coefficients and finishes the elementwise pass from the registers: one launch,
// one read of every operand.
//
// The wait needs every block of a tile co-resident.  The host only picks this path when the
// whole grid fits in HALF of the device's occupancy for the kernel (hipOccupancy... x CUs), so
// it still fits next to a persistent RCCL kernel; the spin is additionally bounded (~0.5 s,
// s_sleep between polls) and a timed-out wait is counted in g_bn_spin_timeouts instead of
// hanging the device (the results of that launch are then wrong, and the test suite fails on
// the counter).
__device__ unsigned g_bn_spin_timeouts;

// Per-tile generation word (monotonic, never reset): every block reads it BEFORE its arrival in
// the tree, the tile's finisher bumps it after publishing, the others wait for it to move.  The
// hand-off follows cdna_hip_programming.md Guideline 16 R1 without fences: the finisher stores
// the coefficients write-through (sc1) and drains every wave before the bump; consumers read
// them with sc1 loads only, so no acquire (L1 invalidate) and no release (L2 writeback) is paid.
struct Flag {
  unsigned* gen;
  unsigned g0;  // value seen at entry (thread 0 only)
};

__device__ __forceinline__ Flag tile_flag(const Red& R) {
  Flag f;
  f.gen = R.cnt + kTreeWords + 2 * blockIdx.y;
  f.g0 = 0;
  if (threadIdx.x == 0) f.g0 = __hip_atomic_load(f.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the value must be back before this block's arrival add (arrive() drains vmcnt first)
  return f;
}

__device__ __forceinline__ void publish(const Flag& f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores are done
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(f.gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void wait_published(const Flag& f) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(f.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == f.g0) {
      __builtin_amdgcn_s_sleep(4);
      if (++spins > (1u << 22)) {
        atomicAdd(&g_bn_spin_timeouts, 1u);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: keep loads below the poll
  __syncthreads();
}

// published per-channel values: sc1 (agent-scope relaxed atomic) loads, never cached in L1
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Row addressing through buffer descriptors: the per-thread part (row phase + channel group) is
// one 32-bit VGPR offset, the per-vector part (block base + u * rpi rows) a scalar soffset, so
// holding V vectors in registers costs no per-vector address registers (flat 64-bit addresses
// kept live across the reduction for the final stores pushed the V = 16 variant to 255 VGPRs).
struct RowMap {
  int voff;    // bytes: (rs * C + col) * 2
  int sbase;   // bytes: block's first row * C * 2   (wave-uniform)
  int sstep;   // bytes: rpi * C * 2                (wave-uniform)
  int nvalid;  // vectors of this thread inside the tensor (<= V)
  int64_t row0;  // this thread's first row
  int64_t col;
  bool active;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ RowMap row_map(const Red& R, int V) {
  const int cg = threadIdx.x % R.tprp, rs = threadIdx.x / R.tprp;
  RowMap m;
  m.active = cg < R.CT / 8;
  m.col = (int64_t)blockIdx.y * R.CT + cg * 8;
  const int64_t b0 = (int64_t)blockIdx.x * R.rows_per_blk;
  m.voff = (int)(((int64_t)rs * R.C + m.col) * 2);
  m.sbase = (int)(b0 * R.C * 2);
  m.sstep = R.rpi * R.C * 2;
  m.row0 = b0 + rs;
  const int64_t left = R.M - (b0 + rs);  // rows from this thread's first row to the end
  int nv = left <= 0 ? 0 : (int)((left + R.rpi - 1) / R.rpi);
  m.nvalid = m.active ? (nv < V ? nv : V) : 0;
  return m;
}

// Vectors past the end of the tensor (u >= nvalid) are pushed out of the descriptor's range
// through the VGPR offset (+1 GiB; buffers here are < 2 GiB, so no 32-bit wrap): their loads
// return 0 and their stores are dropped by the hardware range check -- no per-vector branches.
__device__ __forceinline__ int voff_u(const RowMap& m, int u) { return u < m.nvalid ? m.voff : m.voff + 0x40000000; }

template <int V>
__device__ __forceinline__ void load_rows(const uint16_t* __restrict__ p, const Red& R, const RowMap& m, uint4 (&buf)[V]) {
  const __amdgpu_buffer_rsrc_t rs = rsrc(p, R.M * R.C * 2);
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff_u(m, u), m.sbase + u * m.sstep, 0);
    buf[u] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

// Stores take the whole offset in the VGPR and soffset = 0: with a REGISTER soffset hipcc
// (ROCm 7.2, gfx950) omits the wait state between a buffer_store_dwordx4 and a following VALU
// overwrite of its data VGPRs, and the store then writes the overwritten value (measured:
// d(residual) lanes corrupted exactly in the dword rewritten right after the store).
__device__ __forceinline__ void store_raw(__amdgpu_buffer_rsrc_t rs, const RowMap& m, int u, const uint4 w) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{w.x, w.y, w.z, w.w}, rs, voff_u(m, u) + m.sbase + u * m.sstep, 0, 0);
}

__device__ __forceinline__ void store_row(__amdgpu_buffer_rsrc_t rs, const RowMap& m, int u, const float* v) {
  uint4 o;
  o.x = (uint32_t)f32_to_bf16_rne(v[0]) | ((uint32_t)f32_to_bf16_rne(v[1]) << 16);
  o.y = (uint32_t)f32_to_bf16_rne(v[2]) | ((uint32_t)f32_to_bf16_rne(v[3]) << 16);
  o.z = (uint32_t)f32_to_bf16_rne(v[4]) | ((uint32_t)f32_to_bf16_rne(v[5]) << 16);
  o.w = (uint32_t)f32_to_bf16_rne(v[6]) | ((uint32_t)f32_to_bf16_rne(v[7]) << 16);
  store_raw(rs, m, u, o);
}

// Opaque to the optimiser: the second pass must re-unpack the packed bf16 registers instead of
// keeping the first pass's fp32 unpacked copies alive across the wait (2x the registers).
template <int V>
__device__ __forceinline__ void launder(uint4 (&b)[V]) {
#pragma unroll
  for (int u = 0; u < V; ++u) asm volatile("" : "+v"(b[u].x), "+v"(b[u].y), "+v"(b[u].z), "+v"(b[u].w));
}

__device__ __forceinline__ Bf8 unpack_bf8(const uint4 u) {
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

// stats finisher body shared by the two forward variants (store = how save[] is written)
template <typename Store>
__device__ __forceinline__ void finish_stats(const Red& R, const StatsOut& o, Store store) {
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
    store(o.save + c, (float)mean);
    store(o.save + C + c, invstd);
    store(o.save + 2 * C + c, scale);
    store(o.save + 3 * C + c, be - (float)mean * scale);
    store(o.save + 4 * C + c, 0.f);  // the backward's atomic totals
    store(o.save + 5 * C + c, 0.f);
    if (o.running_mean) {
      o.running_mean[c] = (1.f - o.momentum) * o.running_mean[c] + o.momentum * (float)mean;
      o.running_var[c] = (1.f - o.momentum) * o.running_var[c] + o.momentum * (float)(var * unbias);
    }
  }
  if (threadIdx.x == 0 && blockIdx.y == 0 && o.nbt) *o.nbt += 1;
}

template <int V, bool RELU, bool RES>
__global__ __launch_bounds__(kB) void bn_fwd_fused_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                          Red R, StatsOut o, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ mask) {
  const RowMap m = row_map(R, V);
  uint4 xb[V];
  uint4 rb[RES ? V : 1];
  load_rows<V>(x, R, m, xb);
  if constexpr (RES) load_rows<V>(res, R, m, rb);  // in flight across the reduction
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const Bf8 v = unpack_bf8(xb[u]);  // rows past the end are zeros: no effect on the sums
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += v.v[j];
      q[j] = fmaf(v.v[j], v.v[j], q[j]);
    }
  }
  const Flag f = tile_flag(R);
  if (block_reduce_tree(R, s, q)) {
    finish_stats(R, o, [](float* p, float v) { store_sc1(p, v); });
    publish(f);
  }
  wait_published(f);
  launder(xb);
  float sc[8], sh[8];
  if (m.active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = ld_sc1(o.save + 2 * R.C + m.col + j);
      sh[j] = ld_sc1(o.save + 3 * R.C + m.col + j);
    }
  }
  const __amdgpu_buffer_rsrc_t ys = rsrc(y, R.M * R.C * 2);
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const Bf8 v = unpack_bf8(xb[u]);
    float out[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = fmaf(v.v[j], sc[j], sh[j]);
    if constexpr (RES) {
      const Bf8 rr = unpack_bf8(rb[u]);
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] += rr.v[j];
    }
    if constexpr (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = fmaxf(out[j], 0.f);
    }
    const uint4 pk = pack_bf8(out);
    store_raw(ys, m, u, pk);
    if constexpr (RELU)
      if (u < m.nvalid) mask[(m.row0 + (int64_t)u * R.rpi) * (R.C >> 3) + (m.col >> 3)] = relu_byte(pk);
  }
}

template <int V, bool RELU, bool RES>
__global__ __launch_bounds__(kB) void bn_bwd_fused_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                          const uint8_t* __restrict__ mask, Red R, GradOut o,
                                                          uint16_t* __restrict__ dx, uint16_t* __restrict__ dres) {
  const RowMap m = row_map(R, V);
  uint4 db[V], xb[V];
  load_rows<V>(dy, R, m, db);
  load_rows<V>(x, R, m, xb);
  if constexpr (RELU) {  // db <- dz = dy * [y > 0], exact in bf16
    uint32_t mb[V];
#pragma unroll
    for (int u = 0; u < V; ++u)
      mb[u] = u < m.nvalid ? mask[(m.row0 + (int64_t)u * R.rpi) * (R.C >> 3) + (m.col >> 3)] : 0u;
#pragma unroll
    for (int u = 0; u < V; ++u) {
      db[u].x &= pair_mask(mb[u], 0);
      db[u].y &= pair_mask(mb[u], 1);
      db[u].z &= pair_mask(mb[u], 2);
      db[u].w &= pair_mask(mb[u], 3);
    }
  }
  float mu[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = m.active ? o.save[m.col + j] : 0.f;
    s1[j] = s2[j] = 0.f;
  }
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const Bf8 d = unpack_bf8(db[u]), v = unpack_bf8(xb[u]);  // zeros past the end
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[j] += d.v[j];
      s2[j] = fmaf(d.v[j], v.v[j] - mu[j], s2[j]);
    }
  }
  const Flag f = tile_flag(R);
  if (block_reduce_tree(R, s1, s2)) {
    const int CT = R.CT, C = R.C;
    const double* total = R.total + (size_t)blockIdx.y * 2 * CT;
    const double inv_m = 1.0 / (double)R.M;
    for (int cl = threadIdx.x; cl < CT; cl += kB) {
      const int c = blockIdx.y * CT + cl;
      const double S1 = total[cl], S2 = total[CT + cl];
      const float mean = o.save[c], invstd = o.save[C + c];
      const float ga = o.gamma ? o.gamma[c] : 1.f;
      const double dg = S2 * (double)invstd;
      if (o.dgamma) o.dgamma[c] = (float)dg;
      if (o.dbeta) o.dbeta[c] = (float)S1;
      const double a = (double)ga * invstd;
      const double b = -a * invstd * dg * inv_m;
      store_sc1(o.coef + c, (float)a);
      store_sc1(o.coef + C + c, (float)b);
      store_sc1(o.coef + 2 * C + c, (float)(-a * S1 * inv_m - b * mean));
    }
    publish(f);
  }
  wait_published(f);
  launder(db);
  launder(xb);
  float ca[8], cb[8], cc[8];
  if (m.active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ca[j] = ld_sc1(o.coef + m.col + j);
      cb[j] = ld_sc1(o.coef + R.C + m.col + j);
      cc[j] = ld_sc1(o.coef + 2 * R.C + m.col + j);
    }
  }
  const __amdgpu_buffer_rsrc_t dxs = rsrc(dx, R.M * R.C * 2);
  const __amdgpu_buffer_rsrc_t drs = rsrc(RES ? dres : dx, R.M * R.C * 2);
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const Bf8 d = unpack_bf8(db[u]), v = unpack_bf8(xb[u]);
    const float* dz = d.v;
    float out[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = fmaf(ca[j], dz[j], fmaf(cb[j], v.v[j], cc[j]));
    store_row(dxs, m, u, out);
    if constexpr (RES) store_raw(drs, m, u, db[u]);  // d(residual) = dz, already bf16-exact
  }
}

// ---------------------------------------------------------------- fp32 single-launch variants
// The fp32 step (the reference harness's precision) runs ~28 small BN layers per direction in
// ResNet-50 (stages 2-4 at batch 32: 1.6-13 MB per tensor) where the two-kernel path is bound by
// two launches and two serial reduction tails, not by bytes.  Same structure as the bf16
// kernels above -- the block's rows stay in REGISTERS (V 8-channel rows of 32 B per thread per
// operand: two 16-B buffer loads), the arrival tree publishes the coefficients, every block
// waits for its tile's finisher and finishes the elementwise pass from the registers -- with
// the fp32 numerics of the two-kernel path (fp64 fixed-order tree: deterministic).
// Backward variants: RELU (saved 1-bit mask), DY2 (dual output: dz = [y>0] (dy + dy2)), RES
// (write d(residual) = dz).  Buffers < 1 GiB (32-bit offsets with the +1 GiB out-of-range push).
__device__ __forceinline__ void ldf8(__amdgpu_buffer_rsrc_t rs, int voff, int soff, float* v) {
  const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
  const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16, soff, 0);
  v[0] = __uint_as_float(a.x); v[1] = __uint_as_float(a.y); v[2] = __uint_as_float(a.z); v[3] = __uint_as_float(a.w);
  v[4] = __uint_as_float(b.x); v[5] = __uint_as_float(b.y); v[6] = __uint_as_float(b.z); v[7] = __uint_as_float(b.w);
}

// whole offset in the VGPR, soffset 0 (see store_raw: the register-soffset store hazard)
__device__ __forceinline__ void stf8(__amdgpu_buffer_rsrc_t rs, int off, const float* v) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                               __float_as_uint(v[3])}, rs, off, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                                               __float_as_uint(v[7])}, rs, off + 16, 0, 0);
}

// fp32 row map: byte offsets of 4-byte elements (row_map is the bf16 one)
__device__ __forceinline__ RowMap row_map_f32(const Red& R, int V) {
  RowMap m = row_map(R, V);
  const int cg = threadIdx.x % R.tprp, rs = threadIdx.x / R.tprp;
  const int64_t b0 = (int64_t)blockIdx.x * R.rows_per_blk;
  m.voff = (int)(((int64_t)rs * R.C + m.col) * 4);
  m.sbase = (int)(b0 * R.C * 4);
  m.sstep = R.rpi * R.C * 4;
  (void)cg;
  return m;
}

template <int V>
__device__ __forceinline__ void load_rows_f32(const float* __restrict__ p, const Red& R, const RowMap& m,
                                              float (&buf)[V][8]) {
  const __amdgpu_buffer_rsrc_t rs = rsrc(p, R.M * R.C * 4);
#pragma unroll
  for (int u = 0; u < V; ++u) ldf8(rs, voff_u(m, u), m.sbase + u * m.sstep, buf[u]);
}

template <int V>
__device__ __forceinline__ void launder_f32(float (&b)[V][8]) {
#pragma unroll
  for (int u = 0; u < V; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(b[u][j]));
}

template <int V, bool RELU, bool RES>
__global__ __launch_bounds__(kB) void bn_fwd_fused_f32_kernel(const float* __restrict__ x, const float* __restrict__ res,
                                                              Red R, StatsOut o, float* __restrict__ y,
                                                              uint8_t* __restrict__ mask) {
  const RowMap m = row_map_f32(R, V);
  float xb[V][8];
  load_rows_f32<V>(x, R, m, xb);
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
#pragma unroll
  for (int u = 0; u < V; ++u)  // rows past the end load as zeros: no effect on the sums
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += xb[u][j];
      q[j] = fmaf(xb[u][j], xb[u][j], q[j]);
    }
  const Flag f = tile_flag(R);
  if (block_reduce_tree(R, s, q)) {
    finish_stats(R, o, [](float* p, float v) { store_sc1(p, v); });
    publish(f);
  }
  wait_published(f);
  launder_f32<V>(xb);
  float sc[8], sh[8];
  if (m.active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = ld_sc1(o.save + 2 * R.C + m.col + j);
      sh[j] = ld_sc1(o.save + 3 * R.C + m.col + j);
    }
  }
  const __amdgpu_buffer_rsrc_t ys = rsrc(y, R.M * R.C * 4);
  const __amdgpu_buffer_rsrc_t rr = rsrc(RES ? res : x, R.M * R.C * 4);
#pragma unroll
  for (int u = 0; u < V; ++u) {
    float out[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = fmaf(xb[u][j], sc[j], sh[j]);
    if constexpr (RES) {  // the residual is read only now (no registers held across the wait)
      float rv[8];
      ldf8(rr, voff_u(m, u), m.sbase + u * m.sstep, rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] += rv[j];
    }
    uint32_t b = 0;
    if constexpr (RELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        out[j] = fmaxf(out[j], 0.f);
        b |= (out[j] > 0.f ? 1u : 0u) << j;
      }
    }
    stf8(ys, voff_u(m, u) + m.sbase + u * m.sstep, out);
    if constexpr (RELU)
      if (u < m.nvalid) mask[(m.row0 + (int64_t)u * R.rpi) * (R.C >> 3) + (m.col >> 3)] = (uint8_t)b;
  }
}

template <int V, bool RELU, bool DY2, bool RES>
__global__ __launch_bounds__(kB) void bn_bwd_fused_f32_kernel(const float* __restrict__ dy, const float* __restrict__ dy2,
                                                              const float* __restrict__ x,
                                                              const uint8_t* __restrict__ mask, Red R, GradOut o,
                                                              float* __restrict__ dx, float* __restrict__ dres) {
  const RowMap m = row_map_f32(R, V);
  float db[V][8], xb[V][8];
  load_rows_f32<V>(dy, R, m, db);
  load_rows_f32<V>(x, R, m, xb);
  if constexpr (DY2) {
    const __amdgpu_buffer_rsrc_t r2 = rsrc(dy2, R.M * R.C * 4);
#pragma unroll
    for (int u = 0; u < V; ++u) {
      float e[8];
      ldf8(r2, voff_u(m, u), m.sbase + u * m.sstep, e);
#pragma unroll
      for (int j = 0; j < 8; ++j) db[u][j] += e[j];
    }
  }
  if constexpr (RELU) {  // db <- dz = dy * [y > 0]
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const uint32_t mb = u < m.nvalid ? mask[(m.row0 + (int64_t)u * R.rpi) * (R.C >> 3) + (m.col >> 3)] : 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j) db[u][j] = (mb >> j) & 1u ? db[u][j] : 0.f;
    }
  }
  float mu[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = m.active ? o.save[m.col + j] : 0.f;
    s1[j] = s2[j] = 0.f;
  }
#pragma unroll
  for (int u = 0; u < V; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[j] += db[u][j];
      s2[j] = fmaf(db[u][j], xb[u][j] - mu[j], s2[j]);
    }
  const Flag f = tile_flag(R);
  if (block_reduce_tree(R, s1, s2)) {
    const int CT = R.CT, C = R.C;
    const double* total = R.total + (size_t)blockIdx.y * 2 * CT;
    const double inv_m = 1.0 / (double)R.M;
    for (int cl = threadIdx.x; cl < CT; cl += kB) {
      const int c = blockIdx.y * CT + cl;
      const double S1 = total[cl], S2 = total[CT + cl];
      const float mean = o.save[c], invstd = o.save[C + c];
      const float ga = o.gamma ? o.gamma[c] : 1.f;
      const double dg = S2 * (double)invstd;
      if (o.dgamma) o.dgamma[c] = (float)dg;
      if (o.dbeta) o.dbeta[c] = (float)S1;
      const double a = (double)ga * invstd;
      const double b = -a * invstd * dg * inv_m;
      store_sc1(o.coef + c, (float)a);
      store_sc1(o.coef + C + c, (float)b);
      store_sc1(o.coef + 2 * C + c, (float)(-a * S1 * inv_m - b * mean));
    }
    publish(f);
  }
  wait_published(f);
  launder_f32<V>(db);
  launder_f32<V>(xb);
  float ca[8], cb[8], cc[8];
  if (m.active) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ca[j] = ld_sc1(o.coef + m.col + j);
      cb[j] = ld_sc1(o.coef + R.C + m.col + j);
      cc[j] = ld_sc1(o.coef + 2 * R.C + m.col + j);
    }
  }
  const __amdgpu_buffer_rsrc_t dxs = rsrc(dx, R.M * R.C * 4);
  const __amdgpu_buffer_rsrc_t drs = rsrc(RES ? dres : dx, R.M * R.C * 4);
#pragma unroll
  for (int u = 0; u < V; ++u) {
    float out[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = fmaf(ca[j], db[u][j], fmaf(cb[j], xb[u][j], cc[j]));
    const int off = voff_u(m, u) + m.sbase + u * m.sstep;
    stf8(dxs, off, out);
    if constexpr (RES) stf8(drs, off, db[u]);  // d(residual) = dz
  }
}

// ---------------------------------------------------------------- host-side geometry
// Arrival counters: a device pool of per-launch slots (kSlotWords counters each) taken
// round-robin; the final blocks re-arm their tile's counters, so graph replays reuse a slot and
// BN kernels running concurrently never share one.  Zeroed once at allocation.
constexpr int kSlots = 256;
struct Slots {
  unsigned* counters = nullptr;
  float* ftot = nullptr;
  int next = 0;
};
Slots g_slots[64];

unsigned* next_slot(hipStream_t stream, float** ftot = nullptr) {
  int dev = 0;
  GRACE_HIP_CHECK(hipGetDevice(&dev));
  Slots& p = g_slots[dev];
  if (!p.counters) {  // first use happens eagerly (warm-up), never inside a graph capture
    GRACE_HIP_CHECK(hipMalloc(&p.counters, (size_t)kSlots * kSlotWords * sizeof(unsigned)));
    GRACE_HIP_CHECK(hipMemsetAsync(p.counters, 0, (size_t)kSlots * kSlotWords * sizeof(unsigned), stream));
    // per-slot [2 kMaxC] fp32 totals of the atomic statistics: zero at allocation, re-zeroed by
    // every finisher that reads them (so each launch finds them clean)
    GRACE_HIP_CHECK(hipMalloc(&p.ftot, (size_t)kSlots * 2 * kMaxC * sizeof(float)));
    GRACE_HIP_CHECK(hipMemsetAsync(p.ftot, 0, (size_t)kSlots * 2 * kMaxC * sizeof(float), stream));
    GRACE_HIP_CHECK(hipStreamSynchronize(stream));
  }
  const int s = p.next;
  p.next = (s + 1) % kSlots;
  if (ftot) *ftot = p.ftot + (size_t)s * 2 * kMaxC;
  return p.counters + (size_t)s * kSlotWords;
}

// GRACE_BN_FWD_ATOMIC=1: the forward statistics' blocks meet in atomic fp32 totals with a
// totals-only finisher (as the backward).  Measured no faster than the fixed-order fp64 tree
// (2681-2706 vs 2700-2709 img/s, profiles/r3_bn_atomic_ab.txt), which also keeps the forward
// statistics deterministic and fp64-folded, so off by default.
bool bn_fwd_atomic() {
  static const bool on = [] {
    const char* e = std::getenv("GRACE_BN_FWD_ATOMIC");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

// Grid and tree shape.  Target ~512 blocks (2 per CU) with 8..32 row vectors per thread (knobs below).
// `fused_v` > 0: single-launch layout, exactly V row-vectors per thread (rows_per_blk = rpi*V).
// Grid-shape knobs for experiments (benchmarks/bnact_bench.py sweeps them on the box):
// GRACE_BN_TARGET_BLOCKS (default 512), GRACE_BN_VPT_MIN / _MAX (default 8 / 32 vectors per
// thread), GRACE_BN_ONE_LEVEL (fold every partial row in one level up to this many chunks;
// default 64).  Measured fp32 ResNet-50 (graph-replayed per shape): round-1 shape 4 / 16 / two
// levels always: fwd 1408 + bwd 1961 us per step; these defaults: 1343 + 1907 us.
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && *e) ? atoi(e) : dflt;
}
struct PlanKnobs {
  int target_blocks, vpt_min, vpt_max, one_level;
  PlanKnobs()
      : target_blocks(env_int("GRACE_BN_TARGET_BLOCKS", 512)),
        vpt_min(env_int("GRACE_BN_VPT_MIN", 8)),
        vpt_max(env_int("GRACE_BN_VPT_MAX", 32)),
        one_level(env_int("GRACE_BN_ONE_LEVEL", 64)) {}
};
const PlanKnobs& knobs() {
  static PlanKnobs k;
  return k;
}

// GRACE_BN_DZ=0 restores the 8-pass backward of the dual-gradient residual layers (A/B knob)
bool bn_dz_mode() {
  static const bool on = [] {
    const char* e = std::getenv("GRACE_BN_DZ");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

Red plan(int64_t M, int C, int fused_v = 0) {
  Red R{};
  R.M = M;
  R.C = C;
  R.CT = C < kTileC ? C : kTileC;
  const int tiles = C / R.CT;
  R.tprp = 1;
  while (R.tprp < R.CT / 8) R.tprp <<= 1;
  R.rpi = kB / R.tprp;
  int64_t rpb;
  if (fused_v > 0) {
    rpb = (int64_t)R.rpi * fused_v;
  } else {
    const int64_t n_vec = M * C / 8;
    const PlanKnobs& kn = knobs();
    int64_t vpt = n_vec / ((int64_t)kB * kn.target_blocks);
    if (vpt < kn.vpt_min) vpt = kn.vpt_min;
    if (vpt > kn.vpt_max) vpt = kn.vpt_max;
    const int64_t per_blk = R.rpi * vpt;
    int64_t nc = (M + per_blk - 1) / per_blk;
    if (nc * tiles > 2048) nc = (2048 + tiles - 1) / tiles;
    if (nc < 1) nc = 1;
    rpb = (M + nc - 1) / nc;
    rpb = (rpb + R.rpi - 1) / R.rpi * R.rpi;
  }
  const int64_t nc = (M + rpb - 1) / rpb;
  R.rows_per_blk = rpb;
  R.nchunks = (int)(nc < 1 ? 1 : nc);
  int gs = 1;
  while (gs * gs < R.nchunks) ++gs;
  if (R.nchunks <= knobs().one_level) gs = R.nchunks;  // one fold of every partial row
  int ng = (R.nchunks + gs - 1) / gs;
  while (ng > kMaxGroups) {
    ++gs;
    ng = (R.nchunks + gs - 1) / gs;
  }
  R.gsize = gs;
  R.ngroups = ng;
  return R;
}

// Single-launch eligibility: the smallest V in {2, 4, 8, 16 (forward only)} whose grid fits in
// half of the kernel's device-wide occupancy (see bn_fwd_fused_kernel); 0 = two-kernel path.
constexpr int kFusedVs[4] = {2, 4, 8, 16};

struct FusedCaps {
  int cap[2][4] = {};  // [bwd][v index] resident-block budget
  int target = 256;    // preferred maximum grid (= CUs)
  bool init = false;
};
FusedCaps g_caps[64];

template <typename K>
int half_occupancy(K kernel, int cus) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kB, 0) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return per_cu * cus / 2;
}

// Opt-in (GRACE_BN_FUSED=1 or bn_set_fused): on ResNet-50 the eligible layers gain 1.5-3.5 us
// per pass but the whole-step graph measured no net gain (4165 vs 4183 img/s, within noise),
// and the co-resident wait is the one place a BN launch could stall behind a persistent kernel.
int g_fused_mode = -1;  // -1: from GRACE_BN_FUSED (default off), 0 off, 1 on

template <int V>
int fwd_cap(int cus) {
  return std::min(std::min(half_occupancy(bn_fwd_fused_kernel<V, true, true>, cus),
                           half_occupancy(bn_fwd_fused_kernel<V, true, false>, cus)),
                  std::min(half_occupancy(bn_fwd_fused_kernel<V, false, true>, cus),
                           half_occupancy(bn_fwd_fused_kernel<V, false, false>, cus)));
}

template <int V>
int bwd_cap(int cus) {
  return std::min(std::min(half_occupancy(bn_bwd_fused_kernel<V, true, true>, cus),
                           half_occupancy(bn_bwd_fused_kernel<V, true, false>, cus)),
                  std::min(half_occupancy(bn_bwd_fused_kernel<V, false, true>, cus),
                           half_occupancy(bn_bwd_fused_kernel<V, false, false>, cus)));
}

bool fused_enabled() {
  if (g_fused_mode < 0) {
    const char* e = getenv("GRACE_BN_FUSED");
    g_fused_mode = (e && e[0] == '1') ? 1 : 0;
  }
  return g_fused_mode == 1;
}

const FusedCaps& caps() {
  int dev = 0;
  GRACE_HIP_CHECK(hipGetDevice(&dev));
  FusedCaps& c = g_caps[dev];
  if (!c.init) {
    int cus = 0;
    GRACE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    c.target = cus;
    // the most register-hungry instance of each (direction, V) bounds that V
    c.cap[0][0] = fwd_cap<2>(cus);
    c.cap[0][1] = fwd_cap<4>(cus);
    c.cap[0][2] = fwd_cap<8>(cus);
    c.cap[0][3] = fwd_cap<16>(cus);
    c.cap[1][0] = bwd_cap<2>(cus);
    c.cap[1][1] = bwd_cap<4>(cus);
    c.cap[1][2] = bwd_cap<8>(cus);
    c.cap[1][3] = 0;  // 3 operands x 16 vectors: too many registers
    c.init = true;
  }
  return c;
}

int pick_fused_v(int64_t M, int C, bool bwd) {
  if (!fused_enabled() || M * C * 2 >= ((int64_t)1 << 31)) return 0;  // 32-bit buffer offsets
  const FusedCaps& c = caps();
  const int tiles = C / (C < kTileC ? C : kTileC);
  for (int i = 0; i < 4; ++i) {
    const Red R = plan(M, C, kFusedVs[i]);
    const int64_t blocks = (int64_t)R.nchunks * tiles;
    // Only full blocks (V >= 8) at 1/2 - 1 block per CU pay for the hand-off: measured on MI355X
    // (benchmarks/bnact_bench.py, graph-replayed, ResNet-50 batch 32) V = 8/16 at 196-200 blocks
    // beat the two-kernel path by 1.5-3.5 us per pass; V = 2/4 grids (196-784 blocks of thin
    // blocks) lost 1-3 us, as did any grid of > 1 block per CU.
    if (kFusedVs[i] < 8) continue;
    if (c.cap[bwd][i] > 0 && blocks <= std::min(c.cap[bwd][i], c.target) && 2 * blocks >= c.target)
      return kFusedVs[i];
  }
  return 0;
}

// fp32 single-launch variants (bn_fwd_fused_f32_kernel / bn_bwd_fused_f32_kernel): opt-in
// (GRACE_BN_FUSED_F32=1 or bn_set_fused_f32(true)).  Measured SLOWER than the two-kernel path
// on MI355X (profiles/r4_bnfused_bench.txt, graph-replayed per shape: c256@14 fwd 17.2 vs 14.3 us,
// c512@7 fwd 13.8 vs 10.5 / bwd 19.6 vs 13.1 us; whole fp32 headline 2648 vs 2678 img/s): in a
// graph the second launch costs ~1.5 us while the in-kernel hand-off (tree -> publish -> every
// block's wait -> coefficient loads) serialises the elementwise pass behind the slowest block.
int g_fused32_mode = -1;
bool fused32_enabled() {
  if (g_fused32_mode < 0) {
    const char* e = getenv("GRACE_BN_FUSED_F32");
    g_fused32_mode = (e && e[0] == '1') ? 1 : 0;
  }
  return g_fused32_mode == 1;
}

template <int V>
int fwd_cap_f32(int cus) {
  return std::min(std::min(half_occupancy(bn_fwd_fused_f32_kernel<V, true, true>, cus),
                           half_occupancy(bn_fwd_fused_f32_kernel<V, true, false>, cus)),
                  std::min(half_occupancy(bn_fwd_fused_f32_kernel<V, false, true>, cus),
                           half_occupancy(bn_fwd_fused_f32_kernel<V, false, false>, cus)));
}
template <int V>
int bwd_cap_f32(int cus) {
  int c = half_occupancy(bn_bwd_fused_f32_kernel<V, true, true, true>, cus);
  c = std::min(c, half_occupancy(bn_bwd_fused_f32_kernel<V, true, false, false>, cus));
  c = std::min(c, half_occupancy(bn_bwd_fused_f32_kernel<V, false, false, false>, cus));
  c = std::min(c, half_occupancy(bn_bwd_fused_f32_kernel<V, false, false, true>, cus));
  c = std::min(c, half_occupancy(bn_bwd_fused_f32_kernel<V, true, true, false>, cus));
  return c;
}

struct FusedCaps32 {
  int cap[2][4] = {};  // [bwd][V index of kFusedVs]
  int target = 256;
  bool init = false;
};
FusedCaps32 g_caps32[64];

const FusedCaps32& caps32() {
  int dev = 0;
  GRACE_HIP_CHECK(hipGetDevice(&dev));
  FusedCaps32& c = g_caps32[dev];
  if (!c.init) {
    int cus = 0;
    GRACE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    c.target = cus;
    c.cap[0][0] = fwd_cap_f32<2>(cus);
    c.cap[0][1] = fwd_cap_f32<4>(cus);
    c.cap[0][2] = fwd_cap_f32<8>(cus);
    c.cap[0][3] = fwd_cap_f32<16>(cus);
    c.cap[1][0] = bwd_cap_f32<2>(cus);
    c.cap[1][1] = bwd_cap_f32<4>(cus);
    c.cap[1][2] = bwd_cap_f32<8>(cus);
    c.cap[1][3] = 0;  // 2-3 operands x 16 rows x 8 fp32: too many registers
    c.init = true;
  }
  return c;
}

// The V whose grid holds between half a block and one block per CU (and fits co-resident in
// half of the kernel's occupancy); 0 = the two-kernel path.  Largest V first (fuller blocks).
int pick_fused_v_f32(int64_t M, int C, bool bwd) {
  if (!fused32_enabled() || M * C * 4 >= ((int64_t)1 << 30)) return 0;
  const FusedCaps32& c = caps32();
  const int tiles = C / (C < kTileC ? C : kTileC);
  for (int i = 3; i >= 0; --i) {
    const Red R = plan(M, C, kFusedVs[i]);
    const int64_t blocks = (int64_t)R.nchunks * tiles;
    if (c.cap[bwd][i] > 0 && blocks <= std::min(c.cap[bwd][i], c.target) && 2 * blocks >= c.target)
      return kFusedVs[i];
  }
  return 0;
}

int64_t even(int64_t n) { return (n + 1) & ~(int64_t)1; }

int64_t ws_floats(const Red& R) {
  const int tiles = R.C / R.CT, C2 = 2 * R.CT;
  return even((int64_t)tiles * R.nchunks * C2) + 2 * (int64_t)tiles * (R.ngroups + 1) * C2;
}

void bind_ws(Red& R, float* ws, hipStream_t stream, bool atomic_stats = false) {
  const int tiles = R.C / R.CT, C2 = 2 * R.CT;
  R.part = ws;
  R.gpart = reinterpret_cast<double*>(ws + even((int64_t)tiles * R.nchunks * C2));  // 8-B aligned
  R.total = R.gpart + (size_t)tiles * R.ngroups * C2;
  float* ft = nullptr;
  R.cnt = next_slot(stream, &ft);
  R.ftot = atomic_stats ? ft : nullptr;
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

int64_t bn_workspace_floats(int64_t M, int C) {
  int64_t w = ws_floats(plan(M, C));
  for (int v : kFusedVs) w = std::max(w, ws_floats(plan(M, C, v)));
  return w;
}

int bn_fused_v(int64_t M, int C, bool bwd) { return pick_fused_v(M, C, bwd); }

void bn_set_fused(bool on) { g_fused_mode = on ? 1 : 0; }

void bn_set_fused_f32(bool on) { g_fused32_mode = on ? 1 : 0; }

int bn_fused_v_f32(int64_t M, int C, bool bwd) { return pick_fused_v_f32(M, C, bwd); }

void bn_set_deterministic(bool on);

unsigned bn_spin_timeouts() {
  unsigned h = 0;
  GRACE_HIP_CHECK(hipMemcpyFromSymbol(&h, HIP_SYMBOL(g_bn_spin_timeouts), sizeof(h), 0, hipMemcpyDeviceToHost));
  return h;
}

namespace {

bool bn_deterministic_env();

template <typename T>
void forward_2k(const T* x, const T* res, int64_t M, int C, const StatsOut& o, bool relu, float* save, float* ws,
                T* y, uint8_t* mask, hipStream_t stream) {
  Red R = plan(M, C);
  bind_ws(R, ws, stream, bn_fwd_atomic() && !bn_deterministic_env());
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(R.nchunks, C / R.CT), dim3(kB), 0, stream, x, R, o);
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  if (relu && res)
    hipLaunchKernelGGL((bn_apply_kernel<T, true, true>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<T, true, false>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
  else if (res)
    hipLaunchKernelGGL((bn_apply_kernel<T, false, true>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
  else
    hipLaunchKernelGGL((bn_apply_kernel<T, false, false>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
}

// First level of a two-level fold of GEMM-epilogue partials [tiles][2][C] (fp32) into
// [S][2][C] fp64 rows: a (C/32) x S grid instead of C/32 workgroups walking every tile -- a
// ResNet-50 stage-1 layer has 1568 64-row tiles, which one 32-channel workgroup folded in ~28 us.
// Fixed order inside each slice and across slices (deterministic).
constexpr int kFoldSlice = 32;  // tiles per first-level workgroup
__global__ __launch_bounds__(kB) void bn_fold_l1_kernel(const float* __restrict__ part, int tiles, int C,
                                                        double* __restrict__ out) {
  const int cl = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const int t0 = blockIdx.y * kFoldSlice, t1 = min(tiles, t0 + kFoldSlice);
  double s1 = 0.0, s2 = 0.0;
  if (c < C)
    for (int t = t0 + ph; t < t1; t += 8) {
      s1 += (double)part[(int64_t)t * 2 * C + c];
      s2 += (double)part[(int64_t)t * 2 * C + C + c];
    }
  __shared__ double l1[8][32], l2[8][32];
  l1[ph][cl] = s1;
  l2[ph][cl] = s2;
  __syncthreads();
  if (ph == 0 && c < C) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a += l1[i][cl];
      b += l2[i][cl];
    }
    out[(int64_t)blockIdx.y * 2 * C + c] = a;
    out[(int64_t)blockIdx.y * 2 * C + C + c] = b;
  }
}

// BN statistics from the producing GEMM's epilogue partials (csrc/kernels/gemm_f32.hip p.stats:
// per (row tile, channel) [sum | sum of squares] of the output as stored): the statistics pass
// over the activation disappears; this fold reads tiles x 2C floats.  Block = 32 channels x 8
// tile phases, fp64 accumulation in fixed order (deterministic), finish as bn_stats_kernel.
template <typename P>
__global__ __launch_bounds__(kB) void bn_stats_fold_kernel(const P* __restrict__ part, int tiles, int64_t M,
                                                           int C, StatsOut o) {
  const int cl = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double sx = 0.0, sq = 0.0;
  if (c < C)
    for (int t = ph; t < tiles; t += 8) {
      sx += (double)part[(int64_t)t * 2 * C + c];
      sq += (double)part[(int64_t)t * 2 * C + C + c];
    }
  __shared__ double ls[8][32], lq[8][32];
  ls[ph][cl] = sx;
  lq[ph][cl] = sq;
  __syncthreads();
  if (ph == 0 && c < C) {
    double S = 0.0, Q = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      S += ls[i][cl];
      Q += lq[i][cl];
    }
    const double inv_m = 1.0 / (double)M;
    const double unbias = M > 1 ? (double)M / (double)(M - 1) : 1.0;
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
    o.save[4 * C + c] = 0.f;  // the backward's atomic totals
    o.save[5 * C + c] = 0.f;
    if (o.running_mean) {
      o.running_mean[c] = (1.f - o.momentum) * o.running_mean[c] + o.momentum * (float)mean;
      o.running_var[c] = (1.f - o.momentum) * o.running_var[c] + o.momentum * (float)(var * unbias);
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0 && o.nbt) *o.nbt += 1;
}

// BN backward totals from the consuming conv's data-grad GEMM epilogue (gemm_f32.hip bx / bmask:
// per (row tile, channel) [sum dz | sum dz (x - mean)]): the reduction pass over (dy, x)
// disappears; this fold reads tiles x 2C floats (fp64, fixed order: deterministic) and writes the
// dx pass's coefficients and the parameter gradients exactly as bn_reduce_kernel's finisher.
template <typename P>
__global__ __launch_bounds__(kB) void bn_grad_fold_kernel(const P* __restrict__ part, int tiles, int64_t M,
                                                          int C, GradOut o) {
  const int cl = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  double s1 = 0.0, s2 = 0.0;
  if (c < C)
    for (int t = ph; t < tiles; t += 8) {
      s1 += (double)part[(int64_t)t * 2 * C + c];
      s2 += (double)part[(int64_t)t * 2 * C + C + c];
    }
  __shared__ double l1[8][32], l2[8][32];
  l1[ph][cl] = s1;
  l2[ph][cl] = s2;
  __syncthreads();
  if (ph == 0 && c < C) {
    double S1 = 0.0, S2 = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      S1 += l1[i][cl];
      S2 += l2[i][cl];
    }
    const double inv_m = 1.0 / (double)M;
    const float mean = o.save[c], invstd = o.save[C + c];
    const float ga = o.gamma ? o.gamma[c] : 1.f;
    const double dg = S2 * (double)invstd;  // dgamma = sum dz x^
    if (o.dgamma) o.dgamma[c] = (float)dg;
    if (o.dbeta) o.dbeta[c] = (float)S1;
    const double a = (double)ga * invstd;
    const double b = -a * invstd * dg * inv_m;
    o.coef[c] = (float)a;
    o.coef[C + c] = (float)b;
    o.coef[2 * C + c] = (float)(-a * S1 * inv_m - b * mean);
  }
}

// ATOMIC mode (default; GRACE_BN_ATOMIC_CHUNKS bounds it by chunk count, GRACE_BN_DETERMINISTIC=1
// or a repeated backward of one forward select the fixed-order tree): the reduce kernel adds its blocks' partial rows into save[4C..6C) (zeroed by
// the forward's statistics finisher) and the dx kernel derives the coefficients (CoefSrc).
// GRACE_BN_ATOMIC_CHUNKS: the largest per-tile chunk count whose backward uses the atomic totals
// (default: every layer -- fp32 ResNet-50 headline 2669 -> 2716 img/s, profiles/r3_bn_atomic_ab.txt;
// 0 = the fixed-order tree everywhere, as GRACE_BN_DETERMINISTIC=1)
int g_atomic_chunks = -1;
int bn_atomic_max_chunks() {
  if (g_atomic_chunks < 0) g_atomic_chunks = env_int("GRACE_BN_ATOMIC_CHUNKS", 1 << 30);
  return g_atomic_chunks;
}

int g_det_mode = -1;  // -1: from GRACE_BN_DETERMINISTIC (default off), 0 atomic, 1 deterministic tree
bool bn_deterministic_env() {
  if (g_det_mode < 0) {
    const char* e = std::getenv("GRACE_BN_DETERMINISTIC");
    g_det_mode = (e != nullptr && e[0] == '1') ? 1 : 0;
  }
  return g_det_mode == 1;
}

CoefSrc coef_src(const GradOut& o, int64_t M, bool atomic) {
  (void)M;
  (void)atomic;  // both modes' finishers write coef
  return CoefSrc{o.coef, o.save};
}

float* atot_of(const GradOut& o, int C, bool atomic) {
  return atomic ? const_cast<float*>(o.save) + 4 * (int64_t)C : nullptr;
}

template <typename T, bool DY2>
void backward_2k_t(const T* dy, const T* dy2, const T* x, const uint8_t* mask, int64_t M, int C, const GradOut& o,
                   bool relu, bool atomic, float* ws, T* dx, T* dres, hipStream_t stream) {
  Red R = plan(M, C);
  bind_ws(R, ws, stream);
  const dim3 grid(R.nchunks, C / R.CT);
  float* at = atot_of(o, C, atomic);
  if (relu)
    hipLaunchKernelGGL((bn_reduce_kernel<T, true, DY2>), grid, dim3(kB), 0, stream, dy, dy2, x, mask, R, o, nullptr, at);
  else
    hipLaunchKernelGGL((bn_reduce_kernel<T, false, DY2>), grid, dim3(kB), 0, stream, dy, dy2, x, mask, R, o, nullptr, at);
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  const CoefSrc cs = coef_src(o, M, atomic);
  if (relu && dres)
    hipLaunchKernelGGL((bn_dx_kernel<T, true, true, DY2>), dim3(gb), dim3(kB), 0, stream, dy, dy2, x, mask, cs, dx,
                       dres, n_vec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_dx_kernel<T, true, false, DY2>), dim3(gb), dim3(kB), 0, stream, dy, dy2, x, mask, cs, dx,
                       dres, n_vec, C);
  else if (dres)
    hipLaunchKernelGGL((bn_dx_kernel<T, false, true, DY2>), dim3(gb), dim3(kB), 0, stream, dy, dy2, x, mask, cs, dx,
                       dres, n_vec, C);
  else
    hipLaunchKernelGGL((bn_dx_kernel<T, false, false, DY2>), dim3(gb), dim3(kB), 0, stream, dy, dy2, x, mask, cs,
                       dx, dres, n_vec, C);
}

// ReLU without a saved mask (recomputed from x and the forward's scale / shift in o.save)
template <typename T>
void backward_2k_rx(const T* dy, const T* x, int64_t M, int C, const GradOut& o, bool atomic, float* ws, T* dx,
                    T* dres, hipStream_t stream) {
  Red R = plan(M, C);
  bind_ws(R, ws, stream);
  hipLaunchKernelGGL((bn_reduce_kernel<T, true, false, true>), dim3(R.nchunks, C / R.CT), dim3(kB), 0, stream, dy,
                     (const T*)nullptr, x, (const uint8_t*)nullptr, R, o, nullptr, atot_of(o, C, atomic));
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  const CoefSrc cs = coef_src(o, M, atomic);
  if (dres)
    hipLaunchKernelGGL((bn_dx_kernel<T, true, true, false, true>), dim3(gb), dim3(kB), 0, stream, dy, (const T*)nullptr,
                       x, (const uint8_t*)nullptr, cs, dx, dres, n_vec, C);
  else
    hipLaunchKernelGGL((bn_dx_kernel<T, true, false, false, true>), dim3(gb), dim3(kB), 0, stream, dy,
                       (const T*)nullptr, x, (const uint8_t*)nullptr, cs, dx, dres, n_vec, C);
}

// Two gradients (dual output) AND a residual gradient wanted: the reduce pass stores dz (it is
// d(residual)) and the dx pass reads dz + x -- see bn_reduce_kernel WDZ.
template <typename T>
void backward_2k_dz(const T* dy, const T* dy2, const T* x, const uint8_t* mask, int64_t M, int C, const GradOut& o,
                    bool relu, bool atomic, float* ws, T* dx, T* dres, hipStream_t stream) {
  Red R = plan(M, C);
  bind_ws(R, ws, stream);
  const dim3 grid(R.nchunks, C / R.CT);
  float* at = atot_of(o, C, atomic);
  if (relu)
    hipLaunchKernelGGL((bn_reduce_kernel<T, true, true, false, true>), grid, dim3(kB), 0, stream, dy, dy2, x, mask,
                       R, o, dres, at);
  else
    hipLaunchKernelGGL((bn_reduce_kernel<T, false, true, false, true>), grid, dim3(kB), 0, stream, dy, dy2, x, mask,
                       R, o, dres, at);
  const int64_t n_vec = M * C / 8;
  hipLaunchKernelGGL(bn_dx_dz_kernel<T>, dim3(apply_grid(n_vec, C)), dim3(kB), 0, stream, (const T*)dres, x,
                     coef_src(o, M, atomic), dx, n_vec, C);
}

template <typename T>
void backward_2k(const T* dy, const T* dy2, const T* x, const uint8_t* mask, int64_t M, int C, const GradOut& o,
                 bool relu, bool atomic, float* ws, T* dx, T* dres, hipStream_t stream) {
  if (relu && mask == nullptr && dy2 == nullptr)
    backward_2k_rx<T>(dy, x, M, C, o, atomic, ws, dx, dres, stream);
  else if (std::is_same<T, float>::value && dy2 && dres && bn_dz_mode())  // fp32: dz stored exactly
    backward_2k_dz<T>(dy, dy2, x, mask, M, C, o, relu, atomic, ws, dx, dres, stream);
  else if (dy2)
    backward_2k_t<T, true>(dy, dy2, x, mask, M, C, o, relu, atomic, ws, dx, dres, stream);
  else
    backward_2k_t<T, false>(dy, dy2, x, mask, M, C, o, relu, atomic, ws, dx, dres, stream);
}

}  // namespace

void bn_act_forward(const void* xv, const void* resv, bool fp32, int64_t M, int C, const float* gamma,
                    const float* beta, float* running_mean, float* running_var, int64_t* nbt, float momentum,
                    float eps, bool relu, float* save, float* ws, void* yv, uint8_t* mask, hipStream_t stream) {
  StatsOut o{gamma, beta, running_mean, running_var, nbt, momentum, eps, save};
  if (fp32) {
    const float* xf = static_cast<const float*>(xv);
    const float* rf = static_cast<const float*>(resv);
    float* yf = static_cast<float*>(yv);
    if (const int v = pick_fused_v_f32(M, C, false)) {
      Red R = plan(M, C, v);
      bind_ws(R, ws, stream);
      const dim3 grid(R.nchunks, C / R.CT);
#define GRACE_BN_FWD32(V)                                                                                         \
  if (v == V) {                                                                                                   \
    if (relu && rf)                                                                                               \
      hipLaunchKernelGGL((bn_fwd_fused_f32_kernel<V, true, true>), grid, dim3(kB), 0, stream, xf, rf, R, o, yf, mask);   \
    else if (relu)                                                                                                \
      hipLaunchKernelGGL((bn_fwd_fused_f32_kernel<V, true, false>), grid, dim3(kB), 0, stream, xf, rf, R, o, yf, mask);  \
    else if (rf)                                                                                                  \
      hipLaunchKernelGGL((bn_fwd_fused_f32_kernel<V, false, true>), grid, dim3(kB), 0, stream, xf, rf, R, o, yf, mask);  \
    else                                                                                                          \
      hipLaunchKernelGGL((bn_fwd_fused_f32_kernel<V, false, false>), grid, dim3(kB), 0, stream, xf, rf, R, o, yf, mask); \
    return;                                                                                                       \
  }
      GRACE_BN_FWD32(2)
      GRACE_BN_FWD32(4)
      GRACE_BN_FWD32(8)
      GRACE_BN_FWD32(16)
#undef GRACE_BN_FWD32
    }
    forward_2k(xf, rf, M, C, o, relu, save, ws, yf, mask, stream);
    return;
  }
  const uint16_t* x = static_cast<const uint16_t*>(xv);
  const uint16_t* res = static_cast<const uint16_t*>(resv);
  uint16_t* y = static_cast<uint16_t*>(yv);
  if (const int v = pick_fused_v(M, C, false)) {
    Red R = plan(M, C, v);
    bind_ws(R, ws, stream);
    const dim3 grid(R.nchunks, C / R.CT);
#define GRACE_BN_FWD(V)                                                                                        \
  if (v == V) {                                                                                                \
    if (relu && res)                                                                                           \
      hipLaunchKernelGGL((bn_fwd_fused_kernel<V, true, true>), grid, dim3(kB), 0, stream, x, res, R, o, y, mask);    \
    else if (relu)                                                                                             \
      hipLaunchKernelGGL((bn_fwd_fused_kernel<V, true, false>), grid, dim3(kB), 0, stream, x, res, R, o, y, mask);   \
    else if (res)                                                                                              \
      hipLaunchKernelGGL((bn_fwd_fused_kernel<V, false, true>), grid, dim3(kB), 0, stream, x, res, R, o, y, mask);   \
    else                                                                                                       \
      hipLaunchKernelGGL((bn_fwd_fused_kernel<V, false, false>), grid, dim3(kB), 0, stream, x, res, R, o, y, mask);  \
    return;                                                                                                    \
  }
    GRACE_BN_FWD(2)
    GRACE_BN_FWD(4)
    GRACE_BN_FWD(8)
    GRACE_BN_FWD(16)
#undef GRACE_BN_FWD
  }
  forward_2k(x, res, M, C, o, relu, save, ws, y, mask, stream);
}

// Statistics fold of [tiles][2][C] epilogue partials: one level up to 2 slices, else two (ws:
// >= ceil(tiles / kFoldSlice) * 2C doubles).
void fold_stats(const float* part, int tiles, int64_t M, int C, const StatsOut& o, double* ws, hipStream_t stream) {
  // forward folds: the extra launch of the two-level form measured slower for the headline's
  // statistics folds (21 folds 0.162 ms vs 18 one-level 0.115 ms per step); only very long ones split
  if (tiles > 32 * kFoldSlice && ws != nullptr) {
    const int S = (tiles + kFoldSlice - 1) / kFoldSlice;
    hipLaunchKernelGGL(bn_fold_l1_kernel, dim3((C + 31) / 32, S), dim3(kB), 0, stream, part, tiles, C, ws);
    hipLaunchKernelGGL(bn_stats_fold_kernel<double>, dim3((C + 31) / 32), dim3(kB), 0, stream, (const double*)ws, S,
                       M, C, o);
  } else {
    hipLaunchKernelGGL(bn_stats_fold_kernel<float>, dim3((C + 31) / 32), dim3(kB), 0, stream, part, tiles, M, C, o);
  }
}

// Forward from GEMM-epilogue statistics (fp32): fold + apply, no statistics pass over x.
void bn_act_forward_from_partials(const float* x, const float* res, const float* part, int tiles, int64_t M, int C,
                                  const float* gamma, const float* beta, float* running_mean, float* running_var,
                                  int64_t* nbt, float momentum, float eps, bool relu, float* save, float* y,
                                  uint8_t* mask, hipStream_t stream, double* ws) {
  StatsOut o{gamma, beta, running_mean, running_var, nbt, momentum, eps, save};
  fold_stats(part, tiles, M, C, o, ws, stream);
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  if (relu && res)
    hipLaunchKernelGGL((bn_apply_kernel<float, true, true>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<float, true, false>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
  else if (res)
    hipLaunchKernelGGL((bn_apply_kernel<float, false, true>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
  else
    hipLaunchKernelGGL((bn_apply_kernel<float, false, false>), dim3(gb), dim3(kB), 0, stream, x, res, save, y, mask, n_vec, C);
}

void bn_stats_only(const float* x, int64_t M, int C, const float* gamma, const float* beta, float* running_mean,
                   float* running_var, int64_t* nbt, float momentum, float eps, float* save, float* ws,
                   hipStream_t stream) {
  StatsOut o{gamma, beta, running_mean, running_var, nbt, momentum, eps, save};
  Red R = plan(M, C);
  bind_ws(R, ws, stream, bn_fwd_atomic() && !bn_deterministic_env());
  hipLaunchKernelGGL(bn_stats_kernel<float>, dim3(R.nchunks, C / R.CT), dim3(kB), 0, stream, x, R, o);
}

void bn_fold_partials(const float* part, int tiles, int64_t M, int C, const float* gamma, const float* beta,
                      float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps, float* save,
                      hipStream_t stream, double* ws) {
  StatsOut o{gamma, beta, running_mean, running_var, nbt, momentum, eps, save};
  fold_stats(part, tiles, M, C, o, ws, stream);
}

void bn_act_backward_from_partials(const float* dy, const float* x, const uint8_t* mask, const float* part, int tiles,
                                   int64_t M, int C, const float* gamma, const float* save, bool relu, float* dgamma,
                                   float* dbeta, float* coef, float* dx, hipStream_t stream, double* ws) {
  GradOut o{gamma, save, dgamma, dbeta, coef};
  if (tiles > 2 * kFoldSlice && ws != nullptr) {
    const int S = (tiles + kFoldSlice - 1) / kFoldSlice;
    hipLaunchKernelGGL(bn_fold_l1_kernel, dim3((C + 31) / 32, S), dim3(kB), 0, stream, part, tiles, C, ws);
    hipLaunchKernelGGL(bn_grad_fold_kernel<double>, dim3((C + 31) / 32), dim3(kB), 0, stream, (const double*)ws, S, M,
                       C, o);
  } else {
    hipLaunchKernelGGL(bn_grad_fold_kernel<float>, dim3((C + 31) / 32), dim3(kB), 0, stream, part, tiles, M, C, o);
  }
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  const CoefSrc cs = CoefSrc{coef, save};
  if (relu && mask != nullptr)
    hipLaunchKernelGGL((bn_dx_kernel<float, true, false, false>), dim3(gb), dim3(kB), 0, stream, dy, (const float*)nullptr,
                       x, mask, cs, dx, (float*)nullptr, n_vec, C);
  else if (relu)  // no saved mask (the BN output was never materialised): recomputed from x, scale, shift
    hipLaunchKernelGGL((bn_dx_kernel<float, true, false, false, true>), dim3(gb), dim3(kB), 0, stream, dy,
                       (const float*)nullptr, x, (const uint8_t*)nullptr, cs, dx, (float*)nullptr, n_vec, C);
  else
    hipLaunchKernelGGL((bn_dx_kernel<float, false, false, false>), dim3(gb), dim3(kB), 0, stream, dy,
                       (const float*)nullptr, x, (const uint8_t*)nullptr, cs, dx, (float*)nullptr, n_vec, C);
}

void bn_set_deterministic(bool on) { g_det_mode = on ? 1 : 0; }
void bn_set_atomic_chunks(int n) { g_atomic_chunks = n < 0 ? 0 : n; }
int bn_atomic_chunks() { return bn_atomic_max_chunks(); }

void bn_act_backward(const void* dyv, const void* dy2v, const void* xv, bool fp32, const uint8_t* mask, int64_t M,
                     int C, const float* gamma, const float* save, bool relu, float* dgamma, float* dbeta,
                     float* coef, float* ws, void* dxv, void* dresv, bool deterministic, hipStream_t stream) {
  GradOut o{gamma, save, dgamma, dbeta, coef};
  // atomic totals (one arrival + a totals-only finisher) up to the chunk-count threshold
  const bool atomic = !deterministic && !bn_deterministic_env() && plan(M, C).nchunks <= bn_atomic_max_chunks();
  if (fp32) {
    const float* dyf = static_cast<const float*>(dyv);
    const float* dy2f = static_cast<const float*>(dy2v);
    const float* xf = static_cast<const float*>(xv);
    float* dxf = static_cast<float*>(dxv);
    float* drf = static_cast<float*>(dresv);
    // the single-launch variant needs the saved mask for a ReLU (the stem's RX form stays 2-kernel)
    const int v = (relu && mask == nullptr) ? 0 : pick_fused_v_f32(M, C, true);
    if (v) {
      Red R = plan(M, C, v);
      bind_ws(R, ws, stream);
      const dim3 grid(R.nchunks, C / R.CT);
#define GRACE_BN_BWD32_K(V, RL, D2, RS) \
  hipLaunchKernelGGL((bn_bwd_fused_f32_kernel<V, RL, D2, RS>), grid, dim3(kB), 0, stream, dyf, dy2f, xf, mask, R, o, dxf, drf)
#define GRACE_BN_BWD32(V)                                                   \
  if (v == V) {                                                             \
    if (relu) {                                                             \
      if (dy2f && drf) GRACE_BN_BWD32_K(V, true, true, true);               \
      else if (dy2f) GRACE_BN_BWD32_K(V, true, true, false);                \
      else if (drf) GRACE_BN_BWD32_K(V, true, false, true);                 \
      else GRACE_BN_BWD32_K(V, true, false, false);                         \
    } else {                                                                \
      if (dy2f && drf) GRACE_BN_BWD32_K(V, false, true, true);              \
      else if (dy2f) GRACE_BN_BWD32_K(V, false, true, false);               \
      else if (drf) GRACE_BN_BWD32_K(V, false, false, true);                \
      else GRACE_BN_BWD32_K(V, false, false, false);                        \
    }                                                                       \
    return;                                                                 \
  }
      GRACE_BN_BWD32(2)
      GRACE_BN_BWD32(4)
      GRACE_BN_BWD32(8)
#undef GRACE_BN_BWD32
#undef GRACE_BN_BWD32_K
    }
    // atomic totals contend on 2C addresses from every block: for C <= 64 (one narrow tile) the
    // fixed-order tree is faster (benchmarks/bnact_bench.py fp32, profiles/r4_bnbench.txt)
    backward_2k(dyf, dy2f, xf, mask, M, C, o, relu, atomic && C > 64, ws, dxf, drf, stream);
    return;
  }
  const uint16_t* dy = static_cast<const uint16_t*>(dyv);
  const uint16_t* dy2 = static_cast<const uint16_t*>(dy2v);
  const uint16_t* x = static_cast<const uint16_t*>(xv);
  uint16_t* dx = static_cast<uint16_t*>(dxv);
  uint16_t* dres = static_cast<uint16_t*>(dresv);
  // the single-launch variant reads one dy and a saved mask
  const int v = (dy2 || (relu && mask == nullptr)) ? 0 : pick_fused_v(M, C, true);
  if (v) {
    Red R = plan(M, C, v);
    bind_ws(R, ws, stream);
    const dim3 grid(R.nchunks, C / R.CT);
#define GRACE_BN_BWD(V)                                                                                           \
  if (v == V) {                                                                                                   \
    if (relu && dres)                                                                                             \
      hipLaunchKernelGGL((bn_bwd_fused_kernel<V, true, true>), grid, dim3(kB), 0, stream, dy, x, mask, R, o, dx, dres);   \
    else if (relu)                                                                                                \
      hipLaunchKernelGGL((bn_bwd_fused_kernel<V, true, false>), grid, dim3(kB), 0, stream, dy, x, mask, R, o, dx, dres);  \
    else if (dres)                                                                                                \
      hipLaunchKernelGGL((bn_bwd_fused_kernel<V, false, true>), grid, dim3(kB), 0, stream, dy, x, mask, R, o, dx, dres);  \
    else                                                                                                          \
      hipLaunchKernelGGL((bn_bwd_fused_kernel<V, false, false>), grid, dim3(kB), 0, stream, dy, x, mask, R, o, dx, dres); \
    return;                                                                                                       \
  }
    GRACE_BN_BWD(2)
    GRACE_BN_BWD(4)
    GRACE_BN_BWD(8)
#undef GRACE_BN_BWD
  }
  backward_2k(dy, dy2, x, mask, M, C, o, relu, atomic, ws, dx, dres, stream);
}

namespace {
template <typename T>
void bias_fwd_t(const T* x, const float* bias, int64_t M, int C, bool relu, T* y, hipStream_t stream) {
  const int64_t n_vec = M * C / 8;
  const int gb = apply_grid(n_vec, C);
  if (relu)
    hipLaunchKernelGGL((bias_act_fwd_kernel<T, true>), dim3(gb), dim3(kB), 0, stream, x, bias, y, n_vec, C);
  else
    hipLaunchKernelGGL((bias_act_fwd_kernel<T, false>), dim3(gb), dim3(kB), 0, stream, x, bias, y, n_vec, C);
}
template <typename T>
void bias_bwd_t(const T* dy, const T* y, int64_t M, int C, bool relu, float* dbias, float* ws, T* dz,
                hipStream_t stream) {
  Red R = plan(M, C);
  // the bias gradient's blocks meet in the slot's self-cleaning atomic totals, like the BN backward
  bind_ws(R, ws, stream, !bn_deterministic_env() && plan(M, C).nchunks <= bn_atomic_max_chunks());
  const dim3 grid(R.nchunks, C / R.CT);
  if (relu)
    hipLaunchKernelGGL((bias_act_bwd_kernel<T, true>), grid, dim3(kB), 0, stream, dy, y, dz, R, dbias);
  else
    hipLaunchKernelGGL((bias_act_bwd_kernel<T, false>), grid, dim3(kB), 0, stream, dy, y, dz, R, dbias);
}
}  // namespace

void bias_act_forward(const void* x, const float* bias, bool fp32, int64_t M, int C, bool relu, void* y,
                      hipStream_t stream) {
  if (fp32)
    bias_fwd_t(static_cast<const float*>(x), bias, M, C, relu, static_cast<float*>(y), stream);
  else
    bias_fwd_t(static_cast<const uint16_t*>(x), bias, M, C, relu, static_cast<uint16_t*>(y), stream);
}

void bias_act_backward(const void* dy, const void* y, bool fp32, int64_t M, int C, bool relu, float* dbias, float* ws,
                       void* dz, hipStream_t stream) {
  if (fp32)
    bias_bwd_t(static_cast<const float*>(dy), static_cast<const float*>(y), M, C, relu, dbias, ws,
               static_cast<float*>(dz), stream);
  else
    bias_bwd_t(static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(y), M, C, relu, dbias, ws,
               static_cast<uint16_t*>(dz), stream);
}

namespace {
template <typename T>
void pool_fwd_t(const T* x, int64_t M, int C, const StatsOut& o, float* save, float* ws, const PoolShape& g, int N,
                T* y, uint8_t* code, hipStream_t stream) {
  Red R = plan(M, C);
  bind_ws(R, ws, stream, bn_fwd_atomic() && !bn_deterministic_env());
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(R.nchunks, C / R.CT), dim3(kB), 0, stream, x, R, o);
  const int64_t n_vec = (int64_t)N * g.OH * g.OW * (C / 8);
  const int gb = (int)std::min<int64_t>((n_vec + kB - 1) / kB, 8192);
  hipLaunchKernelGGL(bn_pool_apply_kernel<T>, dim3(gb), dim3(kB), 0, stream, x, save, y, code, g, C, n_vec);
}
}  // namespace

void bn_act_pool_forward(const void* x, bool fp32, int N, int H, int W, int C, const float* gamma, const float* beta,
                         float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps, int k,
                         int s, int pad, int OH, int OW, float* save, float* ws, void* y, uint8_t* code,
                         hipStream_t stream) {
  StatsOut o{gamma, beta, running_mean, running_var, nbt, momentum, eps, save};
  const PoolShape g{H, W, OH, OW, k, s, pad};
  const int64_t M = (int64_t)N * H * W;
  if (fp32)
    pool_fwd_t(static_cast<const float*>(x), M, C, o, save, ws, g, N, static_cast<float*>(y), code, stream);
  else
    pool_fwd_t(static_cast<const uint16_t*>(x), M, C, o, save, ws, g, N, static_cast<uint16_t*>(y), code, stream);
}


}  // namespace grace
