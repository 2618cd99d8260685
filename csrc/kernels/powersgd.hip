// PowerSGD power iteration on CDNA4: bandwidth-shaped VALU tall-skinny products + an MFMA Gram
// (fp32-in/fp32-acc v_mfma_f32_16x16x4_f32, exact fp32) for the r > 4 orthonormalisation.
//
// Reference per matrix (/root/reference/grace_dl/dist/compressor/powersgd.py:30-65):
//   P = M Q ; orthogonalize(P) ; Q = M^T P ; decompress P Q^T     (M: n x m, Q: m x r, r <= 4 typ.)
// Here every matrix of a bucket is processed by ONE launch per product:
//
//  ps_mq / ps_mtp     P = M Q / Q = M^T P: bandwidth-shaped VALU kernels (see below) -- with
//                     r <= 16 the products are 2r FLOP per element, far below the MFMA break-even;
//                     the round-1 MFMA versions (r padded to the 16-wide N tile) measured 0.25-1.8 %
//                     matrix-core utilisation and 2.6-4.4 TB/s.
//  gram_orthonormalize  r <= 4: one workgroup per matrix, one launch (fp64 Gram, MGS in the Gram
//                     metric, in-place A <- A T, twice for CholQR2); r > 4: Gram tiles on MFMA
//                     (all tiles of all matrices in one launch, v_mfma_f32_16x16x4_f32 on the
//                     r x r Gram), per-matrix fix, apply -- see below
//  ps_pqt             out = s P Q^T (s = 1/W: the average of the SUM-all-reduced Q folded in),
//                     optionally fused with the residual update r = x - out
//  philox_normal      N(0,1) via Philox4x32 + Box-Muller (Q identical on every rank)
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kBlock = 256;
constexpr int kT = 64;          // LDS sub-tile edge
constexpr int kLd = kT + 1;     // padded LDS row stride (floats)
constexpr int kStrip = 1024;    // strip length along the reduction dimension
constexpr int kRPad = 16;       // r padded to the MFMA N dimension

using f32x4 = __attribute__((ext_vector_type(4))) float;

struct Mat {
  int64_t x_off, n, m, r, p_off, q_off;
};

__device__ __forceinline__ Mat load_mat(const int64_t* __restrict__ mats, int i) {
  const int64_t* p = mats + 6 * (int64_t)i;
  return Mat{p[0], p[1], p[2], p[3], p[4], p[5]};
}

// ---- Bandwidth-shaped tall-skinny products for the PowerSGD ranks (r <= 16), VALU.
// With r = 4 a product is 8 FLOP per 4-byte element of M: ~0.5 ms of VALU for all of VGG-16 at
// the chip's fp32 rate against ~0.1 ms of HBM time -- it is the BYTES that set the speed, so
// these kernels read M exactly once with 16-B loads (rows whose start is not 16-B aligned use
// the 4-B path), keep the small operand in registers / scalar loads, and write each result once:
//   ps_mq    P[i,:] = sum_k M[i,k] Q[k,:]   block = 16 rows (4 per wave) x 2048-column strip;
//            per-wave row sums reduced with cross-lane adds, one atomic per (row, j) per strip;
//            COMP fuses the PowerSGD error-feedback compensate (M = beta*r + gamma*x -> xout)
//   ps_mtp   Q[k,:] = sum_i M[i,k] P[i,:]   thread = 4 columns (1 unaligned), block = 256-row strip;
//            P rows are wave-uniform (scalar loads), one atomic per (column, j) per strip
//   ps_pqt   out = s P Q^T, resid -= out       thread = 4 columns, Q rows in registers, 32-row strip
// (The MFMA versions of these -- 64x64 LDS-staged tiles with r padded to the 16-wide MFMA N --
// ran at 2.6-4.4 TB/s; MFMA utilisation 0.25-1.8 %, profiles/r1_pmc_powersgd.txt.)
constexpr int kRB0 = 16, kCS0 = 2048;     // ps_mq: rows per block, columns per strip
constexpr int kCBV = 1024, kCBS = 256;    // ps_mtp / ps_pqt: columns per block (16-B / 4-B path)
constexpr int kRSP = 32;                  // rows per strip, at most: ps_pqt (the tile gives its strip; ps_mtp: per-matrix)
constexpr int kPB = 8;                    // rows per batch: independent 16-B loads in flight per thread


__device__ __forceinline__ bool mat_vec(const Mat& mt) { return ((mt.x_off | mt.m) & 3) == 0; }

template <int R>
__device__ __forceinline__ void load_small_row(const float* __restrict__ S, int64_t row, int r, float (&v)[R]) {
  if constexpr (R == 4) {
    if (r == 4 && (reinterpret_cast<uintptr_t>(S) & 15) == 0) {
      const float4 q = *reinterpret_cast<const float4*>(S + row * 4);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      return;
    }
  }
  {
#pragma unroll
    for (int j = 0; j < R; ++j) v[j] = j < r ? S[row * r + j] : 0.f;
  }
}

// COMP 3 (deferred residual): cr holds the previous step's compensated M, and the residual
// r = cr - ls * Pp Qp^T of that step (Pp / Qp: its final P and summed Q, ls = 1/W) is formed here,
// with the float ops of ps_pqt's residual update, instead of being written by ps_pqt and read back.
struct Lazy {
  const float* p;
  const float* q;
  float s;
};

// the 1-D segments of a bucket (biases) travel uncompressed: packed into vec by the P = M Q launch,
// scattered back (times scale) by the P Q^T launch -- no gather / scatter launches of their own
struct VecMove {
  float* vec;
  const int64_t* idx;
  int64_t n;
  float scale;
};

template <int R, int COMP>
__global__ __launch_bounds__(kBlock) void ps_mq_kernel(const float* __restrict__ x, const float* __restrict__ Qall,
                                                       float* __restrict__ Pall, const int64_t* __restrict__ mats,
                                                       const int32_t* __restrict__ tiles, const float* cr, float beta,
                                                       float gamma, float* xout, Lazy lz, int64_t* bump,
                                                       VecMove vm) {
  // the caller's device step counter advances here (read by the philox launch that produced Q,
  // which has completed: stream order) -- one launch fewer per bucket than a separate add
  if (bump != nullptr && blockIdx.x == 0 && threadIdx.x == 0) bump[0] = bump[0] + 1;
  // the bucket's 1-D segments packed for the communicator: vec[e] = x[idx[e]] (grid-stride over
  // every block: replaces a separate gather launch)
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < vm.n; e += (int64_t)gridDim.x * kBlock)
    vm.vec[e] = x[vm.idx[e]];
  const int* tl = tiles + 3 * blockIdx.x;
  const Mat mt = load_mat(mats, tl[0]);
  const int64_t n = mt.n, m = mt.m;
  const int r = (int)mt.r;
  const float* Q = Qall + mt.q_off;
  const int lane = lane_id(), w = wave_id();
  const int64_t row0 = (int64_t)tl[1] * kRB0 + 4 * w;
  // tl[2] = strip index | log2(strip columns) << 24 (0: kCS0) -- the strip length is a host choice
  const int lg = tl[2] >> 24;
  const int64_t cs = lg ? (int64_t(1) << lg) : kCS0;
  const int64_t c0 = (int64_t)(tl[2] & 0xffffff) * cs;
  const int64_t c1 = c0 + cs < m ? c0 + cs : m;
  float acc[4][R];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int j = 0; j < R; ++j) acc[a][j] = 0.f;
  float lp[COMP == 3 ? 4 : 1][R];  // the previous P rows of this wave's 4 rows (wave-uniform)
  if constexpr (COMP == 3) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      if (row0 + rr < n)
        load_small_row<R>(lz.p + mt.p_off, row0 + rr, r, lp[rr]);
      else
#pragma unroll
        for (int j = 0; j < R; ++j) lp[rr][j] = 0.f;
    }
  }
  // residual of the previous step at (row rr, column c + t): cr - ls * sum_j Pp[row, j] Qp[c + t, j]
  auto lazy_o = [&](int rr, const float (&lq)[R]) -> float {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < R; ++j) v = fmaf(lp[rr][j], lq[j], v);
    return v * lz.s;
  };
  // r = 4 (the BASELINE rank): the iteration's 512 Q (and Q') rows are staged through LDS by the
  // whole block -- coalesced 16-B loads, transposed to [j][column] so each lane then takes its 4
  // columns' values with one conflict-free ds_read_b128 per j.  Direct per-lane loads of those
  // rows (4 x 16 B at a 64-B lane stride, the same rows re-fetched by all 4 waves) were half of
  // the kernel's vector loads and left it latency-bound (profiles/r5_powersgd_pmc.txt).
  constexpr int kStage = 512;  // columns per iteration (kCU * 4 * kWave)
  __shared__ __align__(16) float sq[(R == 4) ? (COMP == 3 ? 2 : 1) * 4 * kStage : 1];
  const bool staged = R == 4 && r == 4 && (reinterpret_cast<uintptr_t>(Q) & 15) == 0 &&
                      (COMP != 3 || (reinterpret_cast<uintptr_t>(lz.q + mt.q_off) & 15) == 0);
  if (mat_vec(mt)) {
    constexpr int kCU = 2;  // column chunks per iteration: 4 rows x 2 chunks (x2 with COMP 2) loads in flight
    // the trip count is block-uniform (iterations step the uniform chunk start; lanes past the
    // strip's end load nothing): the staged path's barriers are reached by every thread
    for (int64_t base = c0; base < c1; base += 4 * kWave * kCU) {
      const int64_t cb = base + 4 * lane;
      float4 mv[kCU][4], rv[kCU][4];
#pragma unroll
      for (int k = 0; k < kCU; ++k)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int64_t c = cb + (int64_t)k * 4 * kWave, row = row0 + rr;
          mv[k][rr] = make_float4(0.f, 0.f, 0.f, 0.f);
          rv[k][rr] = mv[k][rr];
          if (row < n && c < c1) {
            const int64_t gi = mt.x_off + row * m + c;
            mv[k][rr] = *reinterpret_cast<const float4*>(x + gi);
            if (COMP >= 2) rv[k][rr] = *reinterpret_cast<const float4*>(cr + gi);
          }
        }
      if constexpr (R == 4) {
        if (staged) {
          const float* lqg = COMP == 3 ? lz.q + mt.q_off : nullptr;
          for (int u = threadIdx.x; u < kStage; u += kBlock) {
            const int64_t col = base + u;
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
            if (col < c1) {
              a = *reinterpret_cast<const float4*>(Q + col * 4);
              if (COMP == 3) b = *reinterpret_cast<const float4*>(lqg + col * 4);
            }
            sq[0 * kStage + u] = a.x;
            sq[1 * kStage + u] = a.y;
            sq[2 * kStage + u] = a.z;
            sq[3 * kStage + u] = a.w;
            if (COMP == 3) {
              sq[4 * kStage + u] = b.x;
              sq[5 * kStage + u] = b.y;
              sq[6 * kStage + u] = b.z;
              sq[7 * kStage + u] = b.w;
            }
          }
          __syncthreads();
        }
      }
#pragma unroll
      for (int k = 0; k < kCU; ++k) {
        const int64_t c = cb + (int64_t)k * 4 * kWave;
        if (c >= c1) break;
        float q[4][R];
        // the 4 columns' rows: from the LDS image (staged, r = 4) or straight from memory
        auto rows4 = [&](int which, const float* g, float (&o)[4][R]) {
          if constexpr (R == 4) {
            if (staged) {
              const int u = (int)(c - base);
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const float4 w4 = *reinterpret_cast<const float4*>(sq + (which * 4 + j) * kStage + u);
                o[0][j] = w4.x;
                o[1][j] = w4.y;
                o[2][j] = w4.z;
                o[3][j] = w4.w;
              }
              return;
            }
          }
#pragma unroll
          for (int t = 0; t < 4; ++t) load_small_row<R>(g, c + t, r, o[t]);
        };
        rows4(0, Q, q);
        if constexpr (COMP == 3) {
          float lq[4][R];
          rows4(1, lz.q + mt.q_off, lq);
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            float4& rv4 = rv[k][rr];
            rv4 = make_float4(rv4.x - lazy_o(rr, lq[0]), rv4.y - lazy_o(rr, lq[1]), rv4.z - lazy_o(rr, lq[2]),
                              rv4.w - lazy_o(rr, lq[3]));
          }
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          float4 v = mv[k][rr];
          if (COMP >= 2)
            v = make_float4(fmaf(beta, rv[k][rr].x, gamma * v.x), fmaf(beta, rv[k][rr].y, gamma * v.y),
                            fmaf(beta, rv[k][rr].z, gamma * v.z), fmaf(beta, rv[k][rr].w, gamma * v.w));
          const int64_t row = row0 + rr;
          if (COMP != 0 && row < n) *reinterpret_cast<float4*>(xout + mt.x_off + row * m + c) = v;
          const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int j = 0; j < R; ++j) acc[rr][j] = fmaf(e[t], q[t][j], acc[rr][j]);
        }
      }
      if constexpr (R == 4) {
        if (staged) __syncthreads();  // the next iteration rewrites the LDS image
      }
    }
  } else {
    for (int64_t c = c0 + lane; c < c1; c += kWave) {
      float q[R], lq[R];
      load_small_row<R>(Q, c, r, q);
      if constexpr (COMP == 3) load_small_row<R>(lz.q + mt.q_off, c, r, lq);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int64_t row = row0 + rr;
        if (row < n) {
          const int64_t gi = mt.x_off + row * m + c;
          float v = x[gi];
          if (COMP == 2) v = fmaf(beta, cr[gi], gamma * v);
          if constexpr (COMP == 3) v = fmaf(beta, cr[gi] - lazy_o(rr, lq), gamma * v);
          if (COMP != 0) xout[gi] = v;
#pragma unroll
          for (int j = 0; j < R; ++j) acc[rr][j] = fmaf(v, q[j], acc[rr][j]);
        }
      }
    }
  }
  float* P = Pall + mt.p_off;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
#pragma unroll
    for (int j = 0; j < R; ++j) acc[rr][j] = wave_sum(acc[rr][j]);
    const int64_t row = row0 + rr;
    if (lane < r && row < n) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < R; ++j) v = lane == j ? acc[rr][j] : v;
      atomicAdd(&P[row * r + lane], v);
    }
  }
}

// ps_mtp geometry: a block owns 1024 contiguous columns (16-B path: 256 threads x 4; 4-B path:
// 256 columns) of a row strip whose length is chosen per matrix on the host (enough workgroups for
// every matrix); each thread accumulates its columns over the strip with kPB independent 16-B
// loads in flight, the block's partial Q is transposed through LDS into address order, and the
// strip's atomics go out as contiguous wave-wide runs (per-lane atomics 64 B apart measured 1.8
// TB/s for VGG-16 fc6; a block covering only 1 KB of each row read slower than one covering 4 KB).
template <int SR>
__device__ void gram_t_block(const float* __restrict__ A, int64_t len, int r, int passes, float* __restrict__ Tout,
                             float4* __restrict__ stage);

// gram: the first n_gram workgroups do not multiply -- workgroup i computes the orthonormalising
// transform T_i of P_i (r <= 4, gram_t_block) while the others stream M: the Gram work hides
// under this bandwidth-bound launch instead of idling the chip in a launch of its own.  Q is then
// M^T P_raw, and Q T / P T are formed where they are consumed (ps_pqt).
template <int R, int kPBm>  // kPBm: rows per batch (independent 16-B loads in flight per thread)
__global__ __launch_bounds__(kBlock) void ps_mtp_kernel(const float* __restrict__ x, const float* __restrict__ Pall,
                                                        float* __restrict__ Qall, const int64_t* __restrict__ mats,
                                                        const int32_t* __restrict__ tiles, int n_gram,
                                                        float* __restrict__ Tout, int passes) {
  __shared__ __align__(16) float red[kCBV * R];
  if ((int)blockIdx.x < n_gram) {  // block-uniform; red doubles as its row staging buffer
    const Mat g = load_mat(mats, blockIdx.x);
    gram_t_block<(kCBV * R) / (kBlock * 4)>(Pall + g.p_off, g.n, (int)g.r, passes, Tout + 16 * (int64_t)blockIdx.x,
                                            reinterpret_cast<float4*>(red));
    return;
  }
  const int* tl = tiles + 3 * (blockIdx.x - n_gram);
  const Mat mt = load_mat(mats, tl[0]);
  const int64_t n = mt.n, m = mt.m;
  const int r = (int)mt.r;
  const float* P = Pall + mt.p_off;
  float* Q = Qall + mt.q_off;
  // tl[2] = (first row / 32) << 16 | (rows / 32)
  const int64_t r0 = (int64_t)(tl[2] >> 16) * 32;
  const int64_t r1 = r0 + (int64_t)(tl[2] & 0xffff) * 32 < n ? r0 + (int64_t)(tl[2] & 0xffff) * 32 : n;
  if (mat_vec(mt)) {  // block-uniform branch
    const int64_t cb = (int64_t)tl[1] * kCBV;
    const int64_t c = cb + 4 * threadIdx.x;
    const bool act = c < m;
    float acc[4][R];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < R; ++j) acc[t][j] = 0.f;
    for (int64_t rb = r0; rb < r1; rb += kPBm) {
      float4 mv[kPBm];
#pragma unroll
      for (int u = 0; u < kPBm; ++u)
        mv[u] = (act && rb + u < r1) ? *reinterpret_cast<const float4*>(x + mt.x_off + (rb + u) * m + c)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < kPBm; ++u) {
        if (rb + u >= r1) break;
        float p[R];
        load_small_row<R>(P, rb + u, r, p);
        const float e[4] = {mv[u].x, mv[u].y, mv[u].z, mv[u].w};
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < R; ++j) acc[t][j] = fmaf(e[t], p[j], acc[t][j]);
      }
    }
    // LDS image of the block's Q rows in address order: (local column, j) at local_col * r + j
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j < r) red[(4 * threadIdx.x + t) * r + j] = acc[t][j];
    __syncthreads();
    const int64_t ncols = m - cb < kCBV ? m - cb : kCBV;
    for (int e = threadIdx.x; e < ncols * r; e += kBlock) atomicAdd(&Q[cb * r + e], red[e]);
  } else {
    const int64_t c = (int64_t)tl[1] * kCBS + threadIdx.x;
    if (c >= m) return;
    float acc[R];
#pragma unroll
    for (int j = 0; j < R; ++j) acc[j] = 0.f;
    for (int64_t row = r0; row < r1; ++row) {
      const float v = x[mt.x_off + row * m + c];
      float p[R];
      load_small_row<R>(P, row, r, p);
#pragma unroll
      for (int j = 0; j < R; ++j) acc[j] = fmaf(v, p[j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (j < r) atomicAdd(&Q[c * r + j], acc[j]);
  }
}

template <int R>
__global__ __launch_bounds__(kBlock) void ps_pqt_kernel(const float* __restrict__ Pall, const float* __restrict__ Qall,
                                                        float* out, const int64_t* __restrict__ mats,
                                                        const int32_t* __restrict__ tiles, float* __restrict__ resid,
                                                        float scale, float* __restrict__ save_p,
                                                        float* __restrict__ save_q, VecMove vm,
                                                        const float* __restrict__ Tall) {  // out == nullptr: residual update only
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < vm.n; e += (int64_t)gridDim.x * kBlock)
    out[vm.idx[e]] = vm.vec[e] * vm.scale;
  const int* tl = tiles + 3 * blockIdx.x;
  const Mat mt = load_mat(mats, tl[0]);
  // Tall (r <= 4): the orthonormalising transform of matrix tl[0] (ps_mtp's gram workgroups): the
  // P / Q rows read here are P_raw / M^T P_raw, and P T / (M^T P_raw) T = M^T (P T) are formed in
  // registers
  float tt[(R <= 4) ? 4 : 1][(R <= 4) ? 4 : 1];
  const bool use_t = R <= 4 && Tall != nullptr;
  if constexpr (R <= 4) {
    if (use_t) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) tt[i][j] = Tall[16 * (int64_t)tl[0] + 4 * i + j];
    }
  }
  auto xform = [&](float (&v)[R]) {
    if constexpr (R <= 4) {
      if (use_t) {
        float o[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < R; ++i) a = fmaf(v[i], tt[i][j], a);
          o[j] = a;
        }
#pragma unroll
        for (int j = 0; j < R; ++j) v[j] = o[j];
      }
    }
  };
  const int64_t n = mt.n, m = mt.m;
  const int r = (int)mt.r;
  const float* P = Pall + mt.p_off;
  const float* Q = Qall + mt.q_off;
  // tl[1] = first row, tl[2] = column block | rows in the strip (<= kRSP) << 20: short strips
  // (more workgroups) for buckets of small matrices, chosen on the host
  const int64_t rows = tl[2] >> 20;
  const int64_t r0 = tl[1];
  const int64_t r1 = r0 + rows < n ? r0 + rows : n;
  const int cblk = tl[2] & 0xfffff;
  // save_p / save_q (the deferred residual's copies of this step's P and Q, same offsets): the
  // first column block of every row strip stores the strip's P rows, the first row strip stores
  // Q below (each element exactly once; replaces two copy launches per bucket)
  if (save_p != nullptr && cblk == 0)
    for (int64_t row = r0 + threadIdx.x; row < r1; row += kBlock) {
      float p[R];
      load_small_row<R>(P, row, r, p);
      xform(p);
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j < r) save_p[mt.p_off + row * r + j] = p[j];
    }
  const bool save_q_here = save_q != nullptr && tl[1] == 0;
  if (mat_vec(mt)) {
    const int64_t c = (int64_t)cblk * kCBV + 4 * threadIdx.x;
    if (c >= m) return;
    float q[4][R];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      load_small_row<R>(Q, c + t, r, q[t]);
      xform(q[t]);
    }
    if (save_q_here)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < R; ++j)
          if (j < r) save_q[mt.q_off + (c + t) * r + j] = q[t][j];
    for (int64_t rb = r0; rb < r1; rb += kPB) {
      float4 rv[kPB];
      if (resid != nullptr) {
#pragma unroll
        for (int u = 0; u < kPB; ++u)
          if (rb + u < r1) rv[u] = *reinterpret_cast<const float4*>(resid + mt.x_off + (rb + u) * m + c);
      }
#pragma unroll
      for (int u = 0; u < kPB; ++u) {
        const int64_t row = rb + u;
        if (row >= r1) break;
        float p[R];
        load_small_row<R>(P, row, r, p);
        xform(p);
        float o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float v = 0.f;
#pragma unroll
          for (int j = 0; j < R; ++j) v = fmaf(p[j], q[t][j], v);
          o[t] = v * scale;
        }
        const int64_t gi = mt.x_off + row * m + c;
        if (out != nullptr) *reinterpret_cast<float4*>(out + gi) = make_float4(o[0], o[1], o[2], o[3]);
        if (resid != nullptr)
          *reinterpret_cast<float4*>(resid + gi) =
              make_float4(rv[u].x - o[0], rv[u].y - o[1], rv[u].z - o[2], rv[u].w - o[3]);
      }
    }
  } else {
    const int64_t c = (int64_t)cblk * kCBS + threadIdx.x;
    if (c >= m) return;
    float q[R];
    load_small_row<R>(Q, c, r, q);
    xform(q);
    if (save_q_here)
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j < r) save_q[mt.q_off + c * r + j] = q[j];
    for (int64_t row = r0; row < r1; ++row) {
      float p[R];
      load_small_row<R>(P, row, r, p);
      xform(p);
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < R; ++j) v = fmaf(p[j], q[j], v);
      v *= scale;
      const int64_t gi = mt.x_off + row * m + c;
      if (out != nullptr) out[gi] = v;
      if (resid != nullptr) resid[gi] -= v;
    }
  }
}

// ---- Orthonormalisation of the r columns of every (len x r) block: Gram-matrix MGS.
// The reference runs modified Gram-Schmidt column by column (dist/compressor/powersgd.py:7-18);
// a one-workgroup-per-matrix MGS leaves the chip idle (VGG-16's 25088 x 4 Q took 77 us).  Here:
//   gram_partial  G_tile = A_tile^T A_tile with one v_mfma_f32_16x16x4_f32 per 4 rows (A is both
//                 MFMA operands), all tiles of all matrices in one launch -> fp64 partials;
//   gram_fix      per matrix: fold the partials in tile order (fp64, deterministic), then MGS
//                 expressed in the Gram metric on the r x r coefficient matrix T (columns of
//                 A*T stay orthonormal; zero columns stay zero, as in the MGS kernel it replaces);
//   gram_apply    A <- A T row by row.
// Run twice (CholQR2): the second pass restores fp32-level orthogonality for ill-conditioned P.
constexpr int kGRows = 256;  // rows per Gram tile (64 per wave: short dependent MFMA chains)

__device__ __forceinline__ int64_t blk_len(const Mat& mt, int which) { return which == 0 ? mt.n : mt.m; }
__device__ __forceinline__ int64_t blk_off(const Mat& mt, int which) { return which == 0 ? mt.p_off : mt.q_off; }

// gtiles: int32 [n][2] = (matrix, tile); part: fp64 [n][16*16]
__global__ __launch_bounds__(kBlock) void gram_partial_kernel(const float* __restrict__ buf,
                                                              const int64_t* __restrict__ mats,
                                                              const int32_t* __restrict__ gtiles, int which,
                                                              double* __restrict__ part) {
  const int* tl = gtiles + 2 * blockIdx.x;
  const Mat mt = load_mat(mats, tl[0]);
  const int64_t len = blk_len(mt, which);
  const int r = (int)mt.r;
  const float* A = buf + blk_off(mt, which);
  const int lane = lane_id(), w = wave_id();
  const int64_t r0 = (int64_t)tl[1] * kGRows + (int64_t)w * (kGRows / 4);
  int64_t r1 = r0 + kGRows / 4;
  if (r1 > len) r1 = len;
  const int col = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int64_t k0 = r0; k0 < r1; k0 += 4) {
    const int64_t row = k0 + (lane >> 4);
    const float a = (row < r1 && col < r) ? A[row * r + col] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, acc, 0, 0, 0);  // C[i][j] += A[k][i] A[k][j]
  }
  __shared__ double red[kBlock / kWave][256];
#pragma unroll
  for (int q = 0; q < 4; ++q) red[w][((lane >> 4) * 4 + q) * 16 + col] = (double)acc[q];
  __syncthreads();
  double* o = part + (int64_t)blockIdx.x * 256;
  for (int e = threadIdx.x; e < 256; e += kBlock) o[e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
}

// Modified Gram-Schmidt expressed in the Gram metric: on entry Tm = I, G = A^T A; on exit the
// columns of A*Tm are orthonormal (zero columns stay zero).  One thread (r <= 16).
__device__ void mgs_gram_metric(const double (*G)[16], double (*Tm)[16], int r) {
  for (int i = 0; i < r; ++i) {
    double nn = 0.0;  // ||A t_i||^2 = t_i^T G t_i
    for (int a = 0; a <= i; ++a)
      for (int b = 0; b <= i; ++b) nn += Tm[a][i] * G[a][b] * Tm[b][i];
    // a column (numerically) inside the span of the previous ones -- residual norm below 1e-5 of
    // its own original norm (||A e_i||^2 = G[i][i]) -- becomes ZERO instead of normalised noise
    // (a rank-deficient P, e.g. dead ReLU rows, would otherwise gain a spurious direction and
    // P-hat P-hat^T would no longer be a projection); zero columns stay zero
    const double nrm = nn > 1e-10 * G[i][i] && nn > 0.0 ? sqrt(nn) : 0.0;
    const double inv = nrm > 1e-30 ? 1.0 / nrm : 0.0;
    for (int a = 0; a <= i; ++a) Tm[a][i] *= inv;
    for (int j = i + 1; j < r; ++j) {
      double pr = 0.0;  // <A t_i, A t_j> = t_i^T G t_j
      for (int a = 0; a <= i; ++a)
        for (int b = 0; b <= j; ++b) pr += Tm[a][i] * G[a][b] * Tm[b][j];
      for (int a = 0; a <= i; ++a) Tm[a][j] -= pr * Tm[a][i];
    }
  }
}

// mgs_gram_metric for r <= 4 with register arrays (unrolled, predicated on the runtime r)
__device__ __forceinline__ void mgs_gram_metric_reg(const double (&G)[4][4], double (&Tm)[4][4], int r) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= r) break;
    double nn = 0.0;
#pragma unroll
    for (int a = 0; a <= i; ++a)
#pragma unroll
      for (int b = 0; b <= i; ++b) nn += Tm[a][i] * G[a][b] * Tm[b][i];
    const double nrm = nn > 1e-10 * G[i][i] && nn > 0.0 ? sqrt(nn) : 0.0;  // as mgs_gram_metric
    const double inv = nrm > 1e-30 ? 1.0 / nrm : 0.0;
#pragma unroll
    for (int a = 0; a <= i; ++a) Tm[a][i] *= inv;
#pragma unroll
    for (int j = i + 1; j < 4; ++j) {
      if (j >= r) break;
      double pr = 0.0;
#pragma unroll
      for (int a = 0; a <= i; ++a)
#pragma unroll
        for (int b = 0; b <= j; ++b) pr += Tm[a][i] * G[a][b] * Tm[b][j];
#pragma unroll
      for (int a = 0; a <= i; ++a) Tm[a][j] -= pr * Tm[a][i];
    }
  }
}

// The orthonormalising transform of one n x r block A (r <= 4) WITHOUT rewriting A: T = T_1 T_2
// (CholQR2 in the Gram metric, fp64 Gram sums, as gram_small_kernel) such that A T has orthonormal
// columns; pass 2's rows fl(A T_1) are formed on the fly from A.  Tout: fp32 4 x 4, row-major,
// zero outside r x r.  Whole workgroup; block-uniform control flow.
template <int SR>  // rows per thread staged per round (the stage holds kBlock * SR rows of 16 B)
__device__ void gram_t_block(const float* __restrict__ A, int64_t len, int r, int passes, float* __restrict__ Tout,
                             float4* __restrict__ stage) {
  __shared__ double red[kBlock / kWave][10];
  __shared__ float tcur[4][4];
  __shared__ double tacc[4][4];
  __shared__ double gG[8][4], gT[4][4];
  const bool vec = r == 4 && (reinterpret_cast<uintptr_t>(A) & 15) == 0;
  if (threadIdx.x < 16) {
    const int i = threadIdx.x >> 2, j = threadIdx.x & 3;
    tcur[i][j] = i == j ? 1.f : 0.f;
    tacc[i][j] = i == j ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int pass = 0; pass < passes; ++pass) {
    float t[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) t[i][j] = tcur[i][j];
    double s[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) s[k] = 0.0;
    // rounds of kBlock * SR rows: the SR 16-B loads of a thread go out together and land in the
    // thread's own slots of the stage (no barrier: each thread reads back only what it wrote),
    // then the rows are consumed one at a time -- latency of one round trip per round while the
    // fp64 math stays rolled (VGPRs: this workgroup's register budget is the whole launch's)
#pragma unroll 1
    for (int64_t base = 0; base < len; base += (int64_t)kBlock * SR) {
      if (vec) {
#pragma unroll
        for (int u = 0; u < SR; ++u) {
          const int64_t row = base + (int64_t)u * kBlock + threadIdx.x;
          stage[u * kBlock + threadIdx.x] =
              row < len ? reinterpret_cast<const float4*>(A)[row] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll 1
    for (int u = 0; u < SR; ++u) {
      const int64_t row = base + (int64_t)u * kBlock + threadIdx.x;
      float a[4];
      if (vec) {
        const float4 v = stage[u * kBlock + threadIdx.x];
        a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = i < r && row < len ? A[row * r + i] : 0.f;
      }
      float o[4];
      if (pass == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = a[j];
      } else {  // the row of A T_acc, with gram_small_kernel's apply float ops
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) v = fmaf(a[i], t[i][j], v);
          o[j] = v;
        }
      }
      int k = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i; j < 4; ++j) s[k++] += (double)o[i] * (double)o[j];
    }
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) s[k] = wave_sum(s[k]);
    if (lane_id() == 0)
#pragma unroll
      for (int k = 0; k < 10; ++k) red[wave_id()][k] = s[k];
    __syncthreads();
    if (threadIdx.x == 0) {
      // the Gram and the MGS coefficients in LDS (mgs_gram_metric, runtime loops): this workgroup
      // runs beside the bandwidth-bound product, so its latency is hidden, while register arrays
      // here (mgs_gram_metric_reg) would set the WHOLE launch's VGPR budget (200, occupancy 2)
      // (loops kept rolled: unrolled, this one lane's fp64 temporaries set the register budget)
#pragma unroll 1
      for (int e = 0; e < 16; ++e) {
        const int i = e >> 2, j = e & 3, lo = i < j ? i : j, hi = i < j ? j : i;
        const int k = lo * 4 - (lo * (lo - 1)) / 2 + (hi - lo);  // packed upper-triangle index
        double v = 0.0;
#pragma unroll 1
        for (int w = 0; w < kBlock / kWave; ++w) v += red[w][k];  // fixed order: deterministic
        gG[i][j] = v;
        gT[i][j] = i == j ? 1.0 : 0.0;
      }
#pragma unroll 1
      for (int i = 0; i < r; ++i) {  // mgs_gram_metric on the 4 x 4 corner
        double nn = 0.0;
#pragma unroll 1
        for (int a = 0; a <= i; ++a)
#pragma unroll 1
          for (int b = 0; b <= i; ++b) nn += gT[a][i] * gG[a][b] * gT[b][i];
        const double nrm = nn > 1e-10 * gG[i][i] && nn > 0.0 ? sqrt(nn) : 0.0;
        const double inv = nrm > 1e-30 ? 1.0 / nrm : 0.0;
#pragma unroll 1
        for (int a = 0; a <= i; ++a) gT[a][i] *= inv;
#pragma unroll 1
        for (int j = i + 1; j < r; ++j) {
          double pr = 0.0;
#pragma unroll 1
          for (int a = 0; a <= i; ++a)
#pragma unroll 1
            for (int b = 0; b <= j; ++b) pr += gT[a][i] * gG[a][b] * gT[b][j];
#pragma unroll 1
          for (int a = 0; a <= i; ++a) gT[a][j] -= pr * gT[a][i];
        }
      }
#pragma unroll 1
      for (int e = 0; e < 16; ++e) {  // T_acc <- T_acc T_pass (fp64; gG reused as scratch)
        const int i = e >> 2, j = e & 3;
        double v = 0.0;
#pragma unroll 1
        for (int l = 0; l < 4; ++l) v += tacc[i][l] * gT[l][j];
        gG[4 + i][j] = v;
      }
#pragma unroll 1
      for (int e = 0; e < 16; ++e) {
        const int i = e >> 2, j = e & 3;
        tacc[i][j] = gG[4 + i][j];
        tcur[i][j] = (float)gG[4 + i][j];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x < 16) {
    const int i = threadIdx.x >> 2, j = threadIdx.x & 3;
    Tout[threadIdx.x] = i < r && j < r ? tcur[i][j] : 0.f;
  }
}

// one 64-thread workgroup per matrix; T: fp32 [n_mat][16*16] (row i, col j: A_new[:, j] = sum_i A[:, i] T[i][j])
__global__ __launch_bounds__(kWave) void gram_fix_kernel(const int64_t* __restrict__ mats,
                                                         const int32_t* __restrict__ gtile_begin,
                                                         const double* __restrict__ part, float* __restrict__ T) {
  const int mi = blockIdx.x;
  const Mat mt = load_mat(mats, mi);
  const int r = (int)mt.r;
  __shared__ double G[16][16];
  __shared__ double Tm[16][16];
  const int t0 = gtile_begin[mi], t1 = gtile_begin[mi + 1];
  for (int e = threadIdx.x; e < 256; e += kWave) {
    double v = 0.0;
#pragma unroll 4
    for (int t = t0; t < t1; ++t) v += part[(int64_t)t * 256 + e];
    G[e >> 4][e & 15] = v;
    Tm[e >> 4][e & 15] = (e >> 4) == (e & 15) ? 1.0 : 0.0;
  }
  __syncthreads();
  if (threadIdx.x == 0) mgs_gram_metric(G, Tm, r);
  __syncthreads();
  for (int e = threadIdx.x; e < 256; e += kWave) T[(int64_t)mi * 256 + e] = (float)Tm[e >> 4][e & 15];
}

__global__ __launch_bounds__(kBlock) void gram_apply_kernel(float* __restrict__ buf, const int64_t* __restrict__ mats,
                                                            const int32_t* __restrict__ gtiles, int which,
                                                            const float* __restrict__ T) {
  const int* tl = gtiles + 2 * blockIdx.x;
  const int mi = tl[0];
  const Mat mt = load_mat(mats, mi);
  const int64_t len = blk_len(mt, which);
  const int r = (int)mt.r;
  float* A = buf + blk_off(mt, which);
  __shared__ float Ts[256];
  Ts[threadIdx.x] = T[(int64_t)mi * 256 + threadIdx.x];
  __syncthreads();
  const int64_t rb = (int64_t)tl[1] * kGRows;
  int64_t re = rb + kGRows;
  if (re > len) re = len;
  for (int64_t row = rb + threadIdx.x; row < re; row += kBlock) {
    float a[16], o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = i < r ? A[row * r + i] : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) v = fmaf(a[i], Ts[i * 16 + j], v);
      o[j] = v;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < r) A[row * r + j] = o[j];
  }
}

// r <= 4 (the PowerSGD ranks in use): the whole orthonormalisation of a matrix in ONE workgroup
// and ONE launch for all matrices -- every pass is a Gram matrix from 16-B row loads (fp64 sums
// of the 10 distinct products), MGS in the Gram metric, and the in-place A <- A T.  The
// three-kernel form above costs 3 launches per pass (CholQR2: 6) of ~10 us each for matrices
// of at most a few hundred KB; here the largest (VGG-16 fc6's 25088 x 4 Q) is one workgroup
// streaming 400 KB per pass, the others run beside it.
constexpr int kSmallR = 4;
constexpr int kGramLds = 16384;  // floats of a block staged in LDS (64 KB)
__global__ __launch_bounds__(kBlock) void gram_small_kernel(float* __restrict__ buf, const int64_t* __restrict__ mats,
                                                            int which, int passes, float* __restrict__ zero,
                                                            int64_t zn) {
  // zero[0, zn): the Q arena the following M^T P launches accumulate into (their memsets folded
  // into this launch, which precedes them)
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < zn; e += (int64_t)gridDim.x * kBlock) zero[e] = 0.f;
  const Mat mt = load_mat(mats, blockIdx.x);
  const int64_t len = blk_len(mt, which);
  const int r = (int)mt.r;
  float* A = buf + blk_off(mt, which);
  __shared__ double Tm[kSmallR][kSmallR];
  __shared__ double red[kBlock / kWave][10];
  const bool vec = r == 4 && (reinterpret_cast<uintptr_t>(A) & 15) == 0;
  auto load_row = [&](int64_t row, float (&a)[kSmallR]) {
    if (vec) {
      const float4 v = reinterpret_cast<const float4*>(A)[row];
      a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    } else {
#pragma unroll
      for (int i = 0; i < kSmallR; ++i) a[i] = i < r ? A[row * r + i] : 0.f;
    }
  };
  // A block of <= 64 KB (every P of VGG-16 / ResNet-50) is staged in LDS once: the passes then
  // run on LDS instead of re-streaming the rows with one dependent global load per thread per
  // 256 rows (latency bound: 37 us per call for VGG-16 before)
  __shared__ float4 sA[kGramLds / 4];
  const bool in_lds = vec && len * 4 <= kGramLds;
  if (in_lds) {  // all of a thread's rows (<= 16) in flight at once, then into LDS
    float4 st[kGramLds / 4 / kBlock];
#pragma unroll
    for (int k = 0; k < kGramLds / 4 / kBlock; ++k) {
      const int64_t row = threadIdx.x + (int64_t)k * kBlock;
      st[k] = row < len ? reinterpret_cast<const float4*>(A)[row] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < kGramLds / 4 / kBlock; ++k) {
      const int64_t row = threadIdx.x + (int64_t)k * kBlock;
      if (row < len) sA[row] = st[k];
    }
    __syncthreads();
  }
  auto row_of = [&](int64_t row, float (&a)[kSmallR]) {
    if (in_lds) {
      const float4 v = sA[row];
      a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    } else {
      load_row(row, a);
    }
  };
  for (int pass = 0; pass < passes; ++pass) {
    double s[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) s[k] = 0.0;
#pragma unroll 4
    for (int64_t row = threadIdx.x; row < len; row += kBlock) {
      float a[kSmallR];
      row_of(row, a);
      int k = 0;
#pragma unroll
      for (int i = 0; i < kSmallR; ++i)
#pragma unroll
        for (int j = i; j < kSmallR; ++j) s[k++] += (double)a[i] * (double)a[j];
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) s[k] = wave_sum(s[k]);
    if (lane_id() == 0)
#pragma unroll
      for (int k = 0; k < 10; ++k) red[wave_id()][k] = s[k];
    __syncthreads();
    if (threadIdx.x == 0) {
      // the 4 x 4 Gram and the MGS coefficients in REGISTERS (fully unrolled): the LDS-resident
      // version ran ~8 us per pass of dependent LDS round trips in this single thread
      double g[kSmallR][kSmallR], tm[kSmallR][kSmallR];
      int k = 0;
#pragma unroll
      for (int i = 0; i < kSmallR; ++i)
#pragma unroll
        for (int j = i; j < kSmallR; ++j, ++k) {
          double v = 0.0;
#pragma unroll
          for (int w = 0; w < kBlock / kWave; ++w) v += red[w][k];  // fixed order: deterministic
          g[i][j] = g[j][i] = v;
        }
#pragma unroll
      for (int i = 0; i < kSmallR; ++i)
#pragma unroll
        for (int j = 0; j < kSmallR; ++j) tm[i][j] = i == j ? 1.0 : 0.0;
      mgs_gram_metric_reg(g, tm, r);
#pragma unroll
      for (int i = 0; i < kSmallR; ++i)
#pragma unroll
        for (int j = 0; j < kSmallR; ++j) Tm[i][j] = tm[i][j];
    }
    __syncthreads();
    float t[kSmallR][kSmallR];
#pragma unroll
    for (int i = 0; i < kSmallR; ++i)
#pragma unroll
      for (int j = 0; j < kSmallR; ++j) t[i][j] = (float)Tm[i][j];
#pragma unroll 4
    for (int64_t row = threadIdx.x; row < len; row += kBlock) {
      float a[kSmallR], o[kSmallR];
      row_of(row, a);
#pragma unroll
      for (int j = 0; j < kSmallR; ++j) {
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < kSmallR; ++i) v = fmaf(a[i], t[i][j], v);
        o[j] = v;
      }
      if (in_lds && pass + 1 < passes) {
        sA[row] = make_float4(o[0], o[1], o[2], o[3]);  // the next pass reads LDS
      } else if (vec) {
        reinterpret_cast<float4*>(A)[row] = make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int j = 0; j < kSmallR; ++j)
          if (j < r) A[row * r + j] = o[j];
      }
    }
    __syncthreads();  // the next pass reads what this one wrote (same workgroup)
  }
}

__global__ __launch_bounds__(kBlock) void philox_normal_kernel(float* __restrict__ out, int64_t n, SeedArg sa,
                                                              float* __restrict__ zero, int64_t zn) {
  // zero[0, zn): the P buffer the following M Q launch accumulates into (its memset folded here)
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < zn; e += (int64_t)gridDim.x * kBlock) zero[e] = 0.f;
  const uint64_t seed = sa.get();
  const int64_t stride = (int64_t)gridDim.x * kBlock * 4;
  for (int64_t base = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4; base < n; base += stride) {
    const uint4 r = Philox::gen(seed, (uint64_t)base >> 2, 0x6e6f726du);
    const float u1 = (r.x >> 8) * (1.0f / 16777216.0f) + (0.5f / 16777216.0f);
    const float u2 = (r.y >> 8) * (1.0f / 16777216.0f);
    const float u3 = (r.z >> 8) * (1.0f / 16777216.0f) + (0.5f / 16777216.0f);
    const float u4 = (r.w >> 8) * (1.0f / 16777216.0f);
    const float r1 = sqrtf(-2.f * logf(u1)), r2 = sqrtf(-2.f * logf(u3));
    float s1, c1, s2, c2;
    sincosf(6.283185307179586f * u2, &s1, &c1);
    sincosf(6.283185307179586f * u4, &s2, &c2);
    const float v[4] = {r1 * c1, r1 * s1, r2 * c2, r2 * s2};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (base + k < n) out[base + k] = v[k];
  }
}

}  // namespace

template <int R>
void launch_mq(const float* x, const float* small, float* out, const int64_t* mats, const int32_t* tiles, int n_tiles,
               int mode, const float* comp_r, float beta, float gamma, float* xout, Lazy lz, int64_t* bump,
               VecMove vm, hipStream_t stream) {
  const Lazy none{nullptr, nullptr, 0.f};
  if (mode == 1)  // (16 rows per batch measured slower: 0.855 vs 0.755 ms VGG-16 exchange)
    ps_mtp_kernel<R, kPB><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, 0, nullptr, 0);
  else if (xout == nullptr)
    ps_mq_kernel<R, 0><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, nullptr, 0.f, 0.f, nullptr, none,
                                                       bump, vm);
  else if (comp_r == nullptr)
    ps_mq_kernel<R, 1><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, nullptr, 0.f, 0.f, xout, none, bump,
                                                       vm);
  else if (lz.p == nullptr)
    ps_mq_kernel<R, 2><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, comp_r, beta, gamma, xout, none,
                                                       bump, vm);
  else
    ps_mq_kernel<R, 3><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, comp_r, beta, gamma, xout, lz, bump,
                                                       vm);
}

void powersgd_mq(const float* x, const float* small, float* out, int64_t out_len, const int64_t* mats,
                 const int32_t* tiles, int n_tiles, int mode, const float* comp_r, float beta, float gamma,
                 float* xout, int max_r, hipStream_t stream, const float* lazy_p, const float* lazy_q,
                 float lazy_scale, bool zeroed, int64_t* bump, float* vec, const int64_t* vec_idx,
                 int64_t n_vec) {
  // zeroed: an earlier launch on this stream (philox Q / the Gram launch) already cleared out
  if (!zeroed) GRACE_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(float) * out_len, stream));
  if (n_tiles <= 0) return;  // (the binding refuses a step counter without tiles to advance it)
  const Lazy lz{lazy_p, lazy_q, lazy_scale};
  const VecMove vm{vec, vec_idx, vec != nullptr ? n_vec : 0, 1.f};
  if (max_r <= 1) launch_mq<1>(x, small, out, mats, tiles, n_tiles, mode, comp_r, beta, gamma, xout, lz, bump, vm, stream);
  else if (max_r <= 2) launch_mq<2>(x, small, out, mats, tiles, n_tiles, mode, comp_r, beta, gamma, xout, lz, bump, vm, stream);
  else if (max_r <= 4) launch_mq<4>(x, small, out, mats, tiles, n_tiles, mode, comp_r, beta, gamma, xout, lz, bump, vm, stream);
  else if (max_r <= 8) launch_mq<8>(x, small, out, mats, tiles, n_tiles, mode, comp_r, beta, gamma, xout, lz, bump, vm, stream);
  else launch_mq<16>(x, small, out, mats, tiles, n_tiles, mode, comp_r, beta, gamma, xout, lz, bump, vm, stream);
}

void powersgd_mtp_gram(const float* x, const float* P, float* Q, const int64_t* mats, const int32_t* tiles,
                       int n_tiles, int n_mat, float* T, int passes, int max_r, hipStream_t stream) {
  const int nb = n_tiles + n_mat;
  if (nb <= 0) return;
  if (max_r <= 1) ps_mtp_kernel<1, kPB><<<nb, kBlock, 0, stream>>>(x, P, Q, mats, tiles, n_mat, T, passes);
  else if (max_r <= 2) ps_mtp_kernel<2, kPB><<<nb, kBlock, 0, stream>>>(x, P, Q, mats, tiles, n_mat, T, passes);
  else ps_mtp_kernel<4, kPB><<<nb, kBlock, 0, stream>>>(x, P, Q, mats, tiles, n_mat, T, passes);
}

void gram_orthonormalize(float* buf, const int64_t* mats, int n_mat, int which, const int32_t* gtiles,
                         int n_gtiles, const int32_t* gtile_begin, double* partials, float* T, int passes,
                         int max_r, float* zero, int64_t zn, hipStream_t stream) {
  if (n_mat <= 0 || n_gtiles <= 0) {
    if (zn > 0) GRACE_HIP_CHECK(hipMemsetAsync(zero, 0, sizeof(float) * zn, stream));
    return;
  }
  if (max_r <= kSmallR) {
    gram_small_kernel<<<n_mat, kBlock, 0, stream>>>(buf, mats, which, passes, zero, zn);
    return;
  }
  if (zn > 0) GRACE_HIP_CHECK(hipMemsetAsync(zero, 0, sizeof(float) * zn, stream));
  for (int p = 0; p < passes; ++p) {
    gram_partial_kernel<<<n_gtiles, kBlock, 0, stream>>>(buf, mats, gtiles, which, partials);
    gram_fix_kernel<<<n_mat, kWave, 0, stream>>>(mats, gtile_begin, partials, T);
    gram_apply_kernel<<<n_gtiles, kBlock, 0, stream>>>(buf, mats, gtiles, which, T);
  }
}

void powersgd_pqt(const float* P, const float* Q, float* out, const int64_t* mats, const int32_t* tiles, int n_tiles,
                  float* resid, float scale, int max_r, float* save_p, float* save_q, const float* vec,
                  const int64_t* vec_idx, int64_t n_vec, float vec_scale, const float* T, hipStream_t stream) {
  if (n_tiles <= 0) return;  // (the binding refuses vector segments without tiles)
  const VecMove vm{const_cast<float*>(vec), vec_idx, vec != nullptr ? n_vec : 0, vec_scale};
  if (max_r <= 1) ps_pqt_kernel<1><<<n_tiles, kBlock, 0, stream>>>(P, Q, out, mats, tiles, resid, scale, save_p, save_q, vm, T);
  else if (max_r <= 2) ps_pqt_kernel<2><<<n_tiles, kBlock, 0, stream>>>(P, Q, out, mats, tiles, resid, scale, save_p, save_q, vm, T);
  else if (max_r <= 4) ps_pqt_kernel<4><<<n_tiles, kBlock, 0, stream>>>(P, Q, out, mats, tiles, resid, scale, save_p, save_q, vm, T);
  else if (max_r <= 8) ps_pqt_kernel<8><<<n_tiles, kBlock, 0, stream>>>(P, Q, out, mats, tiles, resid, scale, save_p, save_q, vm, T);
  else ps_pqt_kernel<16><<<n_tiles, kBlock, 0, stream>>>(P, Q, out, mats, tiles, resid, scale, save_p, save_q, vm, T);
}

void philox_normal(float* out, int64_t n, SeedArg seed, hipStream_t stream, float* zero, int64_t zn) {
  if (n <= 0) {
    if (zn > 0) GRACE_HIP_CHECK(hipMemsetAsync(zero, 0, sizeof(float) * zn, stream));
    return;
  }
  int64_t b = (n + 4 * kBlock - 1) / (4 * kBlock);
  if (b > 2048) b = 2048;
  philox_normal_kernel<<<(int)b, kBlock, 0, stream>>>(out, n, seed, zero, zn);
}

}  // namespace grace
