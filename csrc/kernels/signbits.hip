// 1-bit sign compressors for CDNA4: SignSGD, Signum, EF-SignSGD, 1-bit SGD.
//
// Reference payloads store ONE BYTE per sign (uint8 0/1):
//   signsgd.py:11-16, signum.py:13-23, efsignsgd.py:12-21, onebit.py:8-25 (dist backend).
// Here a wave64 `__ballot` turns 64 comparisons into one 64-bit word: 1 bit per element
// (8x smaller than the reference payload, 32x smaller than fp32).  Words are laid out per
// segment: segment s owns words [word_off[s], word_off[s+1]) covering ceil(n_s / 64) groups.
//
// sign_pack   : bit = (x >= 0) [POS] or (x < 0) [NEG]; optionally
//               * Signum momentum m = (1-beta)*x + beta*m_prev, kept in `mom` (sign of m sent),
//               * fused error feedback: x = beta*r + gamma*g first, residual afterwards
//                 r = x - (bit ? vT[seg] : vF[seg])   (vT/vF = the decoded values).
// sign_unpack_aggregate : over W ranks' words (rank-strided rows, rank order fixed):
//               VOTE  : out = (2*#ones >= W) ? +1 : -1     -- majority vote (signsgd.py:25-30)
//               VALUE : out = scale * sum_r (bit_r ? vT_r[seg] : vF_r[seg])
//                       (EF-SignSGD: vT=mean, vF=-mean; 1-bit: vT=mean0, vF=mean1)
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

template <bool NEG, bool MOM, bool EF, bool RESID>
__global__ __launch_bounds__(kBlock) void sign_pack_kernel(ChunkTable ct, const int64_t* __restrict__ seg_start,
                                                           const int64_t* __restrict__ word_off, const float* g,
                                                           const float* r, float beta, float gamma, float* mom,
                                                           float mom_beta, int mom_valid,
                                                           const float* __restrict__ vT, const float* __restrict__ vF,
                                                           float* resid, uint64_t* __restrict__ words) {
  const int c = blockIdx.x;
  const int s = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const int64_t s0 = seg_start[s];
  const int64_t g0 = (b - s0) >> 6;  // first group of this chunk inside the segment
  const int64_t ngroups = (e - b + kWave - 1) / kWave;
  float t_val = 0.f, f_val = 0.f;
  if constexpr (RESID) {
    t_val = vT[s];
    f_val = vF[s];
  }
  for (int64_t q = wave_id(); q < ngroups; q += kWavesPerBlock) {
    const int64_t i = b + q * kWave + lane_id();
    const bool valid = i < e;
    float xv = 0.f, v = 0.f;  // xv: compensated gradient, v: value whose sign is sent
    if (valid) {
      xv = g[i];
      if constexpr (EF) xv = fmaf(beta, r[i], gamma * xv);
      v = xv;
      if constexpr (MOM) {
        if (mom_valid) v = fmaf(1.f - mom_beta, xv, mom_beta * mom[i]);
        mom[i] = v;
      }
    }
    const bool bit = valid && (NEG ? (v < 0.f) : (v >= 0.f));
    const unsigned long long m = __ballot(bit);
    if (lane_id() == 0) words[word_off[s] + g0 + q] = m;
    if constexpr (RESID) {
      if (valid) resid[i] = xv - (bit ? t_val : f_val);
    }
  }
}

template <bool VOTE>
__global__ __launch_bounds__(kBlock) void sign_unpack_kernel(ChunkTable ct, const int64_t* __restrict__ seg_start,
                                                             const int64_t* __restrict__ word_off,
                                                             const uint8_t* __restrict__ base, int64_t rank_stride,
                                                             int64_t words_off_bytes, int64_t vals_off_bytes,
                                                             int n_seg, int n_ranks, float scale,
                                                             float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x;
  const int s = ct.seg[c];
  const int64_t b = ct.begin[c], e = ct.end[c];
  const int64_t s0 = seg_start[s];
  const int64_t g0 = (b - s0) >> 6;
  const int64_t ngroups = (e - b + kWave - 1) / kWave;
  for (int64_t q = wave_id(); q < ngroups; q += kWavesPerBlock) {
    const int64_t i = b + q * kWave + lane_id();
    const int64_t w = word_off[s] + g0 + q;
    float acc = 0.f;
    int ones = 0;
    for (int rk = 0; rk < n_ranks; ++rk) {
      const uint8_t* rb = base + (int64_t)rk * rank_stride;
      const uint64_t word = reinterpret_cast<const uint64_t*>(rb + words_off_bytes)[w];
      const int bit = (int)((word >> lane_id()) & 1ull);
      if constexpr (VOTE) {
        ones += bit;
      } else {
        const float* vals = reinterpret_cast<const float*>(rb + vals_off_bytes);  // [vT_0, vF_0, vT_1, vF_1 ...]
        acc += bit ? vals[2 * s] : vals[2 * s + 1];
      }
    }
    if (i < e) {
      float res;
      if constexpr (VOTE)
        res = (2 * ones >= n_ranks) ? 1.f : -1.f;
      else
        res = acc * scale;
      out[i] = accumulate ? out[i] + res : res;
    }
  }
}

}  // namespace

void sign_pack(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const float* g,
               const float* r, int ef_mode, float beta, float gamma, float* mom, float mom_beta, int mom_valid,
               const float* vT, const float* vF, float* resid, bool neg, uint64_t* words, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  const bool ef = ef_mode == 1, m = mom != nullptr, rs = resid != nullptr;
#define GRACE_SIGN_LAUNCH(N, M, E, R)                                                                         \
  sign_pack_kernel<N, M, E, R><<<ct.n_chunks, kBlock, 0, stream>>>(ct, seg_start, word_off, g, r, beta, gamma, \
                                                                   mom, mom_beta, mom_valid, vT, vF, resid, words)
  if (neg) {
    if (rs) {
      if (ef) GRACE_SIGN_LAUNCH(true, false, true, true);
      else GRACE_SIGN_LAUNCH(true, false, false, true);
    } else {
      GRACE_SIGN_LAUNCH(true, false, false, false);
    }
  } else if (m) {
    if (rs) {
      if (ef) GRACE_SIGN_LAUNCH(false, true, true, true);
      else GRACE_SIGN_LAUNCH(false, true, false, true);
    } else {
      GRACE_SIGN_LAUNCH(false, true, false, false);
    }
  } else {
    if (rs) {
      if (ef) GRACE_SIGN_LAUNCH(false, false, true, true);
      else GRACE_SIGN_LAUNCH(false, false, false, true);
    } else {
      GRACE_SIGN_LAUNCH(false, false, false, false);
    }
  }
#undef GRACE_SIGN_LAUNCH
}

void sign_unpack(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const uint8_t* base,
                 int64_t rank_stride, int64_t words_off_bytes, int64_t vals_off_bytes, int n_seg, int n_ranks,
                 bool vote, float scale, float* out, bool accumulate, hipStream_t stream) {
  if (ct.n_chunks == 0) return;
  if (vote)
    sign_unpack_kernel<true><<<ct.n_chunks, kBlock, 0, stream>>>(ct, seg_start, word_off, base, rank_stride,
                                                                 words_off_bytes, vals_off_bytes, n_seg, n_ranks,
                                                                 scale, out, accumulate ? 1 : 0);
  else
    sign_unpack_kernel<false><<<ct.n_chunks, kBlock, 0, stream>>>(ct, seg_start, word_off, base, rank_stride,
                                                                  words_off_bytes, vals_off_bytes, n_seg, n_ranks,
                                                                  scale, out, accumulate ? 1 : 0);
}

}  // namespace grace
