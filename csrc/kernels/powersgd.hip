// PowerSGD power iteration on CDNA4 matrix cores (fp32-in/fp32-acc MFMA, exact fp32).
//
// Reference per matrix (/root/reference/grace_dl/dist/compressor/powersgd.py:30-65):
//   P = M Q ; orthogonalize(P) ; Q = M^T P ; decompress P Q^T     (M: n x m, Q: m x r, r <= 4 typ.)
// Here every matrix of a bucket is processed by ONE launch per product:
//
//  powersgd_mq<MODE>  MODE 0: P = M Q    MODE 1: Q = M^T P
//      Work list of 64 x 1024 (MODE 0) / 1024 x 64 (MODE 1) strips of M.  A 256-thread workgroup
//      stages 64x64 fp32 sub-tiles of M in LDS (coalesced 256-B row reads, +1 padding against
//      bank conflicts), each wave runs v_mfma_f32_16x16x4_f32 on a 16-row (MODE 0) or 16-column
//      (MODE 1) slice: 16 MFMAs per sub-tile, the small operand (Q or P, r padded to 16) comes
//      from a second LDS tile.  Strip partial sums are combined with fp32 atomics (the output
//      is only n*r or m*r floats).  Tall-skinny with r=4 is bandwidth bound (2 FLOP/byte):
//      the MFMA work is ~25% utilised by construction but still ~3x faster than HBM needs.
//  gram_orthonormalize  r <= 4: one workgroup per matrix, one launch (fp64 Gram, MGS in the Gram
//                     metric, in-place A <- A T, twice for CholQR2); r > 4: Gram tiles on MFMA
//                     (all tiles of all matrices in one launch), per-matrix fix, apply -- see below
//  powersgd_pqt       out = P Q^T: exactly one 16x16x4 MFMA per 16x16 output tile when r <= 4,
//                     optionally fused with the residual update  r = x - P Q^T
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

// tiles: int32 [n_tiles][3] = (matrix, block index along the output dim, strip index)
// COMP (MODE 0 only; every element of M is staged by exactly one workgroup there):
//   0: M = x      1: M = x, stored to xout      2: M = beta*r + gamma*x, stored to xout
// i.e. the PowerSGD error-feedback compensate (memory/powersgd.py) fused into the first
// product instead of a separate read-read-write pass over the bucket.
template <int MODE, int COMP>
__global__ __launch_bounds__(kBlock) void mq_kernel(const float* __restrict__ x, const float* __restrict__ small,
                                                    float* __restrict__ out, const int64_t* __restrict__ mats,
                                                    const int32_t* __restrict__ tiles, const float* cr, float beta,
                                                    float gamma, float* xout) {
  __shared__ float ms[kT * kLd];
  __shared__ float ss[kT * kRPad];
  const int* tl = tiles + 3 * blockIdx.x;
  const Mat mt = load_mat(mats, tl[0]);
  const int64_t n = mt.n, m = mt.m, r = mt.r;
  const int lane = lane_id(), w = wave_id();
  // MODE 0: output rows [ob, ob+64), reduce over cols [s0, s1)
  // MODE 1: output cols [ob, ob+64), reduce over rows [s0, s1)
  const int64_t ob = (int64_t)tl[1] * kT;
  const int64_t red_len = MODE == 0 ? m : n;
  const int64_t s0 = (int64_t)tl[2] * kStrip;
  const int64_t s1 = s0 + kStrip < red_len ? s0 + kStrip : red_len;
  const float* S = small + (MODE == 0 ? mt.q_off : mt.p_off);  // [red_len][r]
  // Software pipeline: the global loads of sub-tile k+1 are issued into registers before the
  // MFMAs of sub-tile k run, so HBM latency overlaps the matrix-core work.
  constexpr int kPer = kT * kT / kBlock;  // 16 elements of M per thread per sub-tile
  float pg[kPer], pr[kPer];
  auto elem = [&](int64_t sb, int it, int64_t& gi) -> bool {
    const int idx = it * kBlock + threadIdx.x;
    const int64_t gr = (MODE == 0 ? ob : sb) + (idx >> 6), gc = (MODE == 0 ? sb : ob) + (idx & 63);
    gi = mt.x_off + gr * m + gc;
    return gr < n && gc < m;
  };
  auto fetch = [&](int64_t sb) {
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      int64_t gi;
      const bool ok = elem(sb, it, gi);
      pg[it] = ok ? x[gi] : 0.f;
      if (COMP == 2) pr[it] = ok ? cr[gi] : 0.f;
    }
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  fetch(s0);
  for (int64_t sb = s0; sb < s1; sb += kT) {
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int idx = it * kBlock + threadIdx.x;
      float v = pg[it];
      if (COMP == 2) v = fmaf(beta, pr[it], gamma * v);
      if (COMP != 0) {
        int64_t gi;
        if (elem(sb, it, gi)) xout[gi] = v;
      }
      ms[(idx >> 6) * kLd + (idx & 63)] = v;
    }
    // small operand rows [sb, sb+64) of S, r padded to 16 with zeros
    for (int it = 0; it < kT * kRPad / kBlock; ++it) {
      const int idx = it * kBlock + threadIdx.x;
      const int kk = idx >> 4, j = idx & 15;
      const int64_t gk = sb + kk;
      ss[idx] = (j < r && gk < s1) ? S[gk * r + j] : 0.f;
    }
    __syncthreads();
    if (sb + kT < s1) fetch(sb + kT);
#pragma unroll 4
    for (int kk = 0; kk < kT; kk += 4) {
      const int ka = kk + (lane >> 4);
      float a;
      if (MODE == 0)
        a = ms[(16 * w + (lane & 15)) * kLd + ka];  // A[i][k] = M[row i][col k]
      else
        a = ms[ka * kLd + 16 * w + (lane & 15)];  // A[i][k] = M^T[col i][row k]
      const float bv = ss[ka * kRPad + (lane & 15)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
    }
  }
  // C/D: col j = lane & 15, row i = (lane >> 4) * 4 + reg
  const int j = lane & 15;
  if (j < r) {
    float* O = out + (MODE == 0 ? mt.p_off : mt.q_off);
    const int64_t olen = MODE == 0 ? n : m;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t oi = ob + 16 * w + (lane >> 4) * 4 + q;
      if (oi < olen) atomicAdd(&O[oi * r + j], acc[q]);
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
    const double nrm = nn > 0.0 ? sqrt(nn) : 0.0;
    const double inv = nrm > 1e-30 ? 1.0 / nrm : 0.0;  // zero column stays zero
    for (int a = 0; a <= i; ++a) Tm[a][i] *= inv;
    for (int j = i + 1; j < r; ++j) {
      double pr = 0.0;  // <A t_i, A t_j> = t_i^T G t_j
      for (int a = 0; a <= i; ++a)
        for (int b = 0; b <= j; ++b) pr += Tm[a][i] * G[a][b] * Tm[b][j];
      for (int a = 0; a <= i; ++a) Tm[a][j] -= pr * Tm[a][i];
    }
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
__global__ __launch_bounds__(kBlock) void gram_small_kernel(float* __restrict__ buf, const int64_t* __restrict__ mats,
                                                            int which, int passes) {
  const Mat mt = load_mat(mats, blockIdx.x);
  const int64_t len = blk_len(mt, which);
  const int r = (int)mt.r;
  float* A = buf + blk_off(mt, which);
  __shared__ double G[16][16];
  __shared__ double Tm[16][16];
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
  for (int pass = 0; pass < passes; ++pass) {
    double s[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) s[k] = 0.0;
#pragma unroll 4
    for (int64_t row = threadIdx.x; row < len; row += kBlock) {
      float a[kSmallR];
      load_row(row, a);
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
      for (int e = 0; e < 256; ++e) {
        G[e >> 4][e & 15] = 0.0;
        Tm[e >> 4][e & 15] = (e >> 4) == (e & 15) ? 1.0 : 0.0;
      }
      int k = 0;
      for (int i = 0; i < kSmallR; ++i)
        for (int j = i; j < kSmallR; ++j, ++k) {
          double v = 0.0;
          for (int w = 0; w < kBlock / kWave; ++w) v += red[w][k];  // fixed order: deterministic
          G[i][j] = G[j][i] = v;
        }
      mgs_gram_metric(G, Tm, r);
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
      load_row(row, a);
#pragma unroll
      for (int j = 0; j < kSmallR; ++j) {
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < kSmallR; ++i) v = fmaf(a[i], t[i][j], v);
        o[j] = v;
      }
      if (vec) {
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

// out[x_off + row*m + col] = sum_j P[row][j] Q[col][j]; tiles: (matrix, row block of 16, col block of 256).
// Each wave computes four 16x16 MFMA tiles (64 columns); the 16 x 256 workgroup tile is staged in
// LDS so every store instruction writes 64 consecutive floats of one row (256 B) instead of four
// 64-B row pieces.  With ``resid`` (holding x) the residual r = x - P Q^T is updated in the same pass.
constexpr int kPqtCols = 256;
__global__ __launch_bounds__(kBlock) void pqt_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                                     float* __restrict__ out, const int64_t* __restrict__ mats,
                                                     const int32_t* __restrict__ tiles, float* resid) {
  __shared__ float tile[16][kPqtCols + 1];
  const int* tl = tiles + 3 * blockIdx.x;
  const Mat mt = load_mat(mats, tl[0]);
  const int64_t n = mt.n, m = mt.m, r = mt.r;
  const float* Pm = P + mt.p_off;
  const float* Qm = Q + mt.q_off;
  const int lane = lane_id(), w = wave_id();
  const int64_t row0 = (int64_t)tl[1] * 16;
  const int64_t cbase = (int64_t)tl[2] * kPqtCols;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int lc0 = 64 * w + 16 * cb;  // local column of this 16x16 tile
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < r; k0 += 4) {
      const int k = k0 + (lane >> 4);
      const int64_t ar = row0 + (lane & 15), bc = cbase + lc0 + (lane & 15);
      const float a = (ar < n && k < r) ? Pm[ar * r + k] : 0.f;  // A[i][k] = P[row i][k]
      const float b = (bc < m && k < r) ? Qm[bc * r + k] : 0.f;  // B[k][j] = Q[col j][k]
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[(lane >> 4) * 4 + q][lc0 + (lane & 15)] = acc[q];
  }
  __syncthreads();
  const int64_t col = cbase + threadIdx.x;
  if (col < m) {
#pragma unroll 4
    for (int rr = 0; rr < 16; ++rr) {
      const int64_t row = row0 + rr;
      if (row < n) {
        const int64_t gi = mt.x_off + row * m + col;
        const float v = tile[rr][threadIdx.x];
        out[gi] = v;
        if (resid != nullptr) resid[gi] -= v;
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void philox_normal_kernel(float* __restrict__ out, int64_t n, SeedArg sa) {
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

void powersgd_mq(const float* x, const float* small, float* out, int64_t out_len, const int64_t* mats,
                 const int32_t* tiles, int n_tiles, int mode, const float* comp_r, float beta, float gamma,
                 float* xout, hipStream_t stream) {
  GRACE_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(float) * out_len, stream));
  if (n_tiles <= 0) return;
  if (mode == 1)
    mq_kernel<1, 0><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, nullptr, 0.f, 0.f, nullptr);
  else if (xout == nullptr)
    mq_kernel<0, 0><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, nullptr, 0.f, 0.f, nullptr);
  else if (comp_r == nullptr)
    mq_kernel<0, 1><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, nullptr, 0.f, 0.f, xout);
  else
    mq_kernel<0, 2><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles, comp_r, beta, gamma, xout);
}

void gram_orthonormalize(float* buf, const int64_t* mats, int n_mat, int which, const int32_t* gtiles,
                         int n_gtiles, const int32_t* gtile_begin, double* partials, float* T, int passes,
                         int max_r, hipStream_t stream) {
  if (n_mat <= 0 || n_gtiles <= 0) return;
  if (max_r <= kSmallR) {
    gram_small_kernel<<<n_mat, kBlock, 0, stream>>>(buf, mats, which, passes);
    return;
  }
  for (int p = 0; p < passes; ++p) {
    gram_partial_kernel<<<n_gtiles, kBlock, 0, stream>>>(buf, mats, gtiles, which, partials);
    gram_fix_kernel<<<n_mat, kWave, 0, stream>>>(mats, gtile_begin, partials, T);
    gram_apply_kernel<<<n_gtiles, kBlock, 0, stream>>>(buf, mats, gtiles, which, T);
  }
}

void powersgd_pqt(const float* P, const float* Q, float* out, const int64_t* mats, const int32_t* tiles, int n_tiles,
                  float* resid, hipStream_t stream) {
  if (n_tiles <= 0) return;
  pqt_kernel<<<n_tiles, kBlock, 0, stream>>>(P, Q, out, mats, tiles, resid);
}

void philox_normal(float* out, int64_t n, SeedArg seed, hipStream_t stream) {
  if (n <= 0) return;
  int64_t b = (n + 4 * kBlock - 1) / (4 * kBlock);
  if (b > 2048) b = 2048;
  philox_normal_kernel<<<(int)b, kBlock, 0, stream>>>(out, n, seed);
}

}  // namespace grace
