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
//  gram_schmidt       one workgroup per matrix, modified Gram-Schmidt over its r columns with
//                     workgroup reductions (columns normalised, later columns projected out)
//  powersgd_pqt       out = P Q^T: exactly one 16x16x4 MFMA per 16x16 output tile when r <= 4
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
template <int MODE>
__global__ __launch_bounds__(kBlock) void mq_kernel(const float* __restrict__ x, const float* __restrict__ small,
                                                    float* __restrict__ out, const int64_t* __restrict__ mats,
                                                    const int32_t* __restrict__ tiles) {
  __shared__ float ms[kT * kLd];
  __shared__ float ss[kT * kRPad];
  const int* tl = tiles + 3 * blockIdx.x;
  const Mat mt = load_mat(mats, tl[0]);
  const int64_t n = mt.n, m = mt.m, r = mt.r;
  const float* M = x + mt.x_off;
  const int lane = lane_id(), w = wave_id();
  // MODE 0: output rows [ob, ob+64), reduce over cols [s0, s1)
  // MODE 1: output cols [ob, ob+64), reduce over rows [s0, s1)
  const int64_t ob = (int64_t)tl[1] * kT;
  const int64_t red_len = MODE == 0 ? m : n;
  const int64_t s0 = (int64_t)tl[2] * kStrip;
  const int64_t s1 = s0 + kStrip < red_len ? s0 + kStrip : red_len;
  const float* S = small + (MODE == 0 ? mt.q_off : mt.p_off);  // [red_len][r]
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t sb = s0; sb < s1; sb += kT) {
    __syncthreads();
    // stage the 64x64 sub-tile: rows/cols of M depend on MODE
    const int64_t r0 = MODE == 0 ? ob : sb;
    const int64_t c0 = MODE == 0 ? sb : ob;
    for (int it = 0; it < kT * kT / kBlock; ++it) {
      const int idx = it * kBlock + threadIdx.x;
      const int rr = idx >> 6, cc = idx & 63;
      const int64_t gr = r0 + rr, gc = c0 + cc;
      ms[rr * kLd + cc] = (gr < n && gc < m) ? M[gr * m + gc] : 0.f;
    }
    // small operand rows [sb, sb+64) of S, r padded to 16 with zeros
    for (int it = 0; it < kT * kRPad / kBlock; ++it) {
      const int idx = it * kBlock + threadIdx.x;
      const int kk = idx >> 4, j = idx & 15;
      const int64_t gk = sb + kk;
      ss[idx] = (j < r && gk < s1) ? S[gk * r + j] : 0.f;
    }
    __syncthreads();
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

// Modified Gram-Schmidt on the r columns of a (len x r) row-major block; one workgroup/matrix.
__global__ __launch_bounds__(kBlock) void gram_schmidt_kernel(float* __restrict__ buf, const int64_t* __restrict__ mats,
                                                              int which) {
  const Mat mt = load_mat(mats, blockIdx.x);
  const int64_t len = which == 0 ? mt.n : mt.m;
  const int r = (int)mt.r;
  float* A = buf + (which == 0 ? mt.p_off : mt.q_off);
  __shared__ float red[kRPad][kBlock / kWave];
  __shared__ float coef[kRPad];
  for (int i = 0; i < r; ++i) {
    // norm of column i
    float s = 0.f;
    for (int64_t k = threadIdx.x; k < len; k += kBlock) {
      const float v = A[k * r + i];
      s += v * v;
    }
    s = wave_sum(s);
    if (lane_id() == 0) red[0][wave_id()] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int q = 0; q < kBlock / kWave; ++q) t += red[0][q];
      const float nrm = sqrtf(t);
      coef[0] = nrm > 1e-30f ? 1.f / nrm : 1e30f;  // zero column stays zero (reference: NaN)
    }
    __syncthreads();
    const float inv = coef[0];
    for (int64_t k = threadIdx.x; k < len; k += kBlock) A[k * r + i] *= inv;
    __syncthreads();
    if (i + 1 >= r) break;
    // projections of the normalised column on every later column
    float d[kRPad];
#pragma unroll
    for (int j = 0; j < kRPad; ++j) d[j] = 0.f;
    for (int64_t k = threadIdx.x; k < len; k += kBlock) {
      const float ci = A[k * r + i];
      for (int j = i + 1; j < r; ++j) d[j] += ci * A[k * r + j];
    }
    for (int j = i + 1; j < r; ++j) {
      const float v = wave_sum(d[j]);
      if (lane_id() == 0) red[j][wave_id()] = v;
    }
    __syncthreads();
    if (threadIdx.x < kRPad && (int)threadIdx.x > i && (int)threadIdx.x < r) {
      float t = 0.f;
      for (int q = 0; q < kBlock / kWave; ++q) t += red[threadIdx.x][q];
      coef[threadIdx.x] = t;
    }
    __syncthreads();
    for (int64_t k = threadIdx.x; k < len; k += kBlock) {
      const float ci = A[k * r + i];
      for (int j = i + 1; j < r; ++j) A[k * r + j] -= coef[j] * ci;
    }
    __syncthreads();
  }
}

// out[x_off + row*m + col] = sum_j P[row][j] Q[col][j]; tiles: (matrix, row block of 16, col block of 64)
__global__ __launch_bounds__(kBlock) void pqt_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                                     float* __restrict__ out, const int64_t* __restrict__ mats,
                                                     const int32_t* __restrict__ tiles) {
  const int* tl = tiles + 3 * blockIdx.x;
  const Mat mt = load_mat(mats, tl[0]);
  const int64_t n = mt.n, m = mt.m, r = mt.r;
  const float* Pm = P + mt.p_off;
  const float* Qm = Q + mt.q_off;
  const int lane = lane_id(), w = wave_id();
  const int64_t row0 = (int64_t)tl[1] * 16;
  const int64_t col0 = (int64_t)tl[2] * 64 + 16 * w;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < r; k0 += 4) {
    const int k = k0 + (lane >> 4);
    const int64_t ar = row0 + (lane & 15), bc = col0 + (lane & 15);
    const float a = (ar < n && k < r) ? Pm[ar * r + k] : 0.f;   // A[i][k] = P[row i][k]
    const float b = (bc < m && k < r) ? Qm[bc * r + k] : 0.f;   // B[k][j] = Q[col j][k]
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  const int64_t col = col0 + (lane & 15);
  if (col < m) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t row = row0 + (lane >> 4) * 4 + q;
      if (row < n) out[mt.x_off + row * m + col] = acc[q];
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
                 const int32_t* tiles, int n_tiles, int mode, hipStream_t stream) {
  GRACE_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(float) * out_len, stream));
  if (n_tiles <= 0) return;
  if (mode == 0)
    mq_kernel<0><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles);
  else
    mq_kernel<1><<<n_tiles, kBlock, 0, stream>>>(x, small, out, mats, tiles);
}

void gram_schmidt(float* buf, const int64_t* mats, int n_mat, int which, hipStream_t stream) {
  if (n_mat <= 0) return;
  gram_schmidt_kernel<<<n_mat, kBlock, 0, stream>>>(buf, mats, which);
}

void powersgd_pqt(const float* P, const float* Q, float* out, const int64_t* mats, const int32_t* tiles, int n_tiles,
                  hipStream_t stream) {
  if (n_tiles <= 0) return;
  pqt_kernel<<<n_tiles, kBlock, 0, stream>>>(P, Q, out, mats, tiles);
}

void philox_normal(float* out, int64_t n, SeedArg seed, hipStream_t stream) {
  if (n <= 0) return;
  int64_t b = (n + 4 * kBlock - 1) / (4 * kBlock);
  if (b > 2048) b = 2048;
  philox_normal_kernel<<<(int)b, kBlock, 0, stream>>>(out, n, seed);
}

}  // namespace grace
