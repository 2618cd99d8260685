// Host-side launcher declarations for every grace_amd HIP kernel.
// All launchers are asynchronous on `stream`, take raw device pointers and never allocate
// or synchronize (so they are safe inside hipGraph capture).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grace_common.h"

namespace grace {

// ---------------------------------------------------------------- topk.hip
struct TopkState {
  uint32_t prefix;  // radix prefix of the k-th largest |x| key (full key after the last digit)
  int32_t krem;     // elements still to take among keys that match `prefix`
};

void topk_select_bucket(const ChunkTable& ct, int n_seg, const float* g, const float* r, float* x,
                        float beta, float gamma, int mode, const int32_t* kseg, TopkState* st,
                        int32_t* hist, hipStream_t stream);
void topk_compact_bucket(const ChunkTable& ct, int n_seg, const float* x, const TopkState* st,
                         const int64_t* out_off, int32_t* counters, float* out_val,
                         int32_t* out_idx, float* resid, int64_t idx_base, hipStream_t stream);
// Two-pass Top-K with fused error feedback (the Top-K compressor): pass A compensates + digit-0
// histogram; pass B splits every chunk into definite takes (front of the chunk's slice of cand_*)
// and threshold-bin candidates (back of the slice); digits 1-2 run on the candidates; the
// assemble kernel writes the payload.  ctr = 3 * n_seg int32, ccnt = 3 * n_chunks int32, cand_*
// sized like x.  mode 0 -> x = g (copied when x != g), mode 1 -> x = beta * x + gamma * g;
// zero: emitted entries of x are set to 0 (the residual update).  g and x 16-B aligned.
void topk_ef_bucket(const ChunkTable& ct, const int32_t* seg_chunk_begin, int n_seg, const float* g, float* x,
                    int64_t total, float beta, float gamma, int mode, int zero, const int32_t* kseg, TopkState* st,
                    int32_t* hist, int32_t* ctr, int32_t* ccnt, const int64_t* out_off, float* out_val,
                    int32_t* out_idx, float* cand_val, int32_t* cand_idx, hipStream_t stream);
void sparse_scatter_add(const float* val, const int32_t* idx, int64_t K, float* out, float scale,
                        bool accumulate, hipStream_t stream);
// K = min(*count, cap) read on the device (capacity payloads with an in-band count);
// count_overflow: count *count > cap in the health words (the decode of this process's OWN payload)
void sparse_scatter_add_dev(const float* val, const int32_t* idx, const int32_t* count, int64_t cap, float* out,
                            float scale, bool accumulate, hipStream_t stream, bool count_overflow);

// ---------------------------------------------------------------- segstats.hip
// per segment: [sum, sumsq, max|x|, sum|x|, sum(x<0), count(x<0)]
constexpr int kSegStats = 6;
// g, r, mode, beta, gamma, xout: optional fused error-feedback compensate (see ef.hip)
void segment_stats(const ChunkTable& ct, int n_seg, const int32_t* seg_chunk_begin, const float* g,
                   const float* r, int mode, float beta, float gamma, float* xout, double* partials, float* stats,
                   hipStream_t stream);

// ---------------------------------------------------------------- sparsify.hip
void randk_gather(const float* x, int n_seg, const int64_t* seg_off, const int64_t* out_off,
                  const int64_t* seeds, const int64_t* step, int64_t K, float* vals, float* resid,
                  hipStream_t stream);
void randk_scatter(const float* vals, int64_t rank_stride, int n_ranks, int n_seg, const int64_t* seg_off,
                   const int64_t* out_off, const int64_t* seeds, const int64_t* step, int64_t K, float* out,
                   float scale, bool accumulate, hipStream_t stream);
void threshold_compact(const float* g, const float* r, int mode, float beta, float gamma, int64_t n, float thr,
                       float* out_val, int32_t* out_idx, int64_t cap, int32_t* counter, float* resid,
                       hipStream_t stream, int header_bytes = 4);

// ---------------------------------------------------------------- signbits.hip
void sign_pack(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const float* g,
               const float* r, int ef_mode, float beta, float gamma, float* mom, float mom_beta, int mom_valid,
               const float* vT, const float* vF, float* resid, bool neg, uint64_t* words, hipStream_t stream);
void sign_unpack(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const uint8_t* base,
                 int64_t rank_stride, int64_t words_off_bytes, int64_t vals_off_bytes, int n_seg, int n_ranks,
                 bool vote, float scale, float* out, bool accumulate, hipStream_t stream);

// ---------------------------------------------------------------- quant.hip
void qsgd_quantize(const ChunkTable& ct, const float* x, const float* norms, float s, SeedArg seed, void* codes,
                   int code_bytes, float* resid, hipStream_t stream);
// qsgd_aggregate code_bytes tags of the bit-packed small-s formats (2-bit: s = 1, 4-bit: s <= 7)
constexpr int kPacked2 = 0x102;
constexpr int kPacked4 = 0x104;
void qsgd_pack(const int8_t* codes, int64_t n, int s, int bits, uint8_t* out, hipStream_t stream);
void qsgd_aggregate(const ChunkTable& ct, const uint8_t* base, int64_t rank_stride, int64_t codes_off,
                    int64_t norms_off, const float* shared_norms, int code_bytes, int n_ranks, float s, float scale,
                    float* out, bool accumulate, hipStream_t stream);
void tern_quantize(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const float* x,
                   const float* clips, const float* scal, SeedArg seed, uint64_t* words, float* resid,
                   hipStream_t stream);
void tern_aggregate(const ChunkTable& ct, const int64_t* seg_start, const int64_t* word_off, const uint8_t* base,
                    int64_t rank_stride, int64_t words_off, int64_t scal_off, int n_ranks, float scale, float* out,
                    bool accumulate, hipStream_t stream);
void natural_encode(const float* x, int64_t n, SeedArg seed, uint8_t* codes, float* resid, hipStream_t stream);
void natural_aggregate(const uint8_t* base, int64_t rank_stride, int64_t n, int n_ranks, float scale, float* out,
                       bool accumulate, hipStream_t stream);
void u8_encode(const ChunkTable& ct, const float* x, const float* scales, int8_t* codes, float* resid,
               hipStream_t stream);
void u8_aggregate(const ChunkTable& ct, const uint8_t* base, int64_t rank_stride, int64_t codes_off, int64_t scal_off,
                  int n_ranks, float scale, float* out, bool accumulate, hipStream_t stream);

// ---------------------------------------------------------------- dgc.hip
// u / v non-null: x is the raw gradient and DgcMemory's compensate is applied on the fly (sample)
// and in place (the first refinement count pass writes u, v); count: int32 [32 n_seg]
void dgc_sample(const float* x, int n_seg, const int64_t* seg_off, const int64_t* samp_off, int64_t n_samples,
                SeedArg seed, float* samples, const float* u, const float* v, float momentum, int first,
                hipStream_t stream);
// ccnt: int32 [32 n_chunks] per-chunk tree counts; fnode: int32 [n_seg] final counted tree node
// (-1: uncounted) -- consumed by dgc_compact (coff: int32 [n_chunks] scratch)
void dgc_refine(const ChunkTable& ct, int n_seg, const float* x, const TopkState* st, const float* target,
                int max_iters, float* thr, int32_t* count, int32_t* done, float* u, float* v, float momentum,
                int first, int64_t n, int32_t* ccnt, int32_t* fnode, bool init, hipStream_t stream);
// exact k'-th largest |sample| per segment (one workgroup each) + the refinement state of
// dgc_refine (thr, count, done, fnode) -- dgc_refine(init = false) then skips its own init
void dgc_select_init(int n_seg, const float* samples, const int64_t* samp_off, const int32_t* kseg, TopkState* st,
                     float* thr, int32_t* count, int32_t* done, int32_t* fnode, hipStream_t stream);
void dgc_compact(const ChunkTable& ct, const float* x, const float* thr, float* out_val, int32_t* out_idx,
                 int64_t cap, int32_t* counter, float* vmask, float* umask, const int32_t* ccnt,
                 const int32_t* fnode, int32_t* coff, hipStream_t stream, int header_bytes = 4);
void dgc_compensate(const float* g, float* u, float* v, float momentum, int64_t n, bool first, hipStream_t stream);

// ---------------------------------------------------------------- powersgd.hip
// mats: int64 [n_mat][6] = (x_off, n, m, r, p_off, q_off); tiles: int32 [n_tiles][3]
void powersgd_mq(const float* x, const float* small, float* out, int64_t out_len, const int64_t* mats,
                 const int32_t* tiles, int n_tiles, int mode, const float* comp_r, float beta, float gamma,
                 float* xout, int max_r, hipStream_t stream, const float* lazy_p = nullptr,
                 const float* lazy_q = nullptr, float lazy_scale = 0.f, bool zeroed = false,
                 int64_t* bump = nullptr, float* vec = nullptr, const int64_t* vec_idx = nullptr,
                 int64_t n_vec = 0);  // lazy_*: deferred residual (mode 0 with comp_r): r = comp_r - s P Q^T;
                                      // zeroed: out already cleared; bump: step counter += 1 (mode 0);
                                      // vec[e] = x[vec_idx[e]] (mode 0: the 1-D segments, packed)
// max_r: largest rank r of the matrices (<= 4 selects the one-launch, one-workgroup-per-matrix form)
void gram_orthonormalize(float* buf, const int64_t* mats, int n_mat, int which, const int32_t* gtiles,
                         int n_gtiles, const int32_t* gtile_begin, double* partials, float* T, int passes,
                         int max_r, float* zero, int64_t zn, hipStream_t stream);  // also clears zero[0, zn)
// out may be null (resid only); save_p / save_q: copies of P and Q (same offsets), may be null
void powersgd_pqt(const float* P, const float* Q, float* out, const int64_t* mats, const int32_t* tiles, int n_tiles,
                  float* resid, float scale, int max_r, float* save_p, float* save_q, const float* vec,
                  const int64_t* vec_idx, int64_t n_vec, float vec_scale, const float* T,
                  hipStream_t stream);  // + out[vec_idx[e]] = vec_scale * vec[e]; T (r <= 4): P T, Q T
// Q = M^T P (P un-normalised) plus, in the same launch, T_i (fp32 [n_mat][16]) with P_i T_i orthonormal
// (r <= 4; n_mat workgroups ahead of the product tiles); Q must be cleared beforehand
void powersgd_mtp_gram(const float* x, const float* P, float* Q, const int64_t* mats, const int32_t* tiles,
                       int n_tiles, int n_mat, float* T, int passes, int max_r, hipStream_t stream);
void philox_normal(float* out, int64_t n, SeedArg seed, hipStream_t stream, float* zero = nullptr,
                   int64_t zn = 0);  // also clears zero[0, zn)

// ---------------------------------------------------------------- cast_sketch.hip
void cast16(const float* x, uint16_t* y, int64_t n, bool bf16, hipStream_t stream);
void decode16_sum(const uint8_t* base, int64_t rank_stride, int n_ranks, int64_t n, bool bf16, float scale, float* out,
                  hipStream_t stream);
void sketch_encode(const ChunkTable& ct, const float* x, const float* edges, int q, void* bins, int bin_bytes,
                   unsigned long long* sums, uint32_t* counts, int32_t* arrive, const int32_t* seg_chunk_begin,
                   float* means, hipStream_t stream);
// q > 1024: global fixed-point bin accumulators, torch.searchsorted's binary search
void sketch_encode_big(const ChunkTable& ct, int n_seg, const float* x, const float* edges, int q, void* bins,
                       int bin_bytes, unsigned long long* sums, uint32_t* counts, int32_t* arrive,
                       const int32_t* seg_chunk_begin, float* means, hipStream_t stream);
void sketch_decode(const ChunkTable& ct, const uint8_t* base, int64_t rank_stride, int64_t bins_off, int64_t means_off,
                   int q, int bin_bytes, int n_ranks, float scale, float* out, hipStream_t stream);

// ---------------------------------------------------------------- quantile.hip
// exact order statistics of every segment at the given sorted ranks + interpolated sketch edges
void quantile_select(const ChunkTable& ct, int n_seg, const float* x, int max_slots, const int32_t* ranks,
                     const int32_t* nrank, int32_t* h0, int32_t* h, uint32_t* st_pfx, int32_t* st_rank, int32_t* slot,
                     uint32_t* uniq, int32_t* nuniq, int q, const int32_t* lo_idx, const int32_t* hi_idx,
                     const float* w, float* edges, hipStream_t stream);

// ---------------------------------------------------------------- gemm_f32.hip
// C[m][n] (+)= sum_k A(m,k) B(n,k) on the f32 MFMA; X(r,k) = x[r*ld+k] (kcontig) or x[k*ld+r];
// splits > 1: split-K with f32 atomics into C (zeroed here; needs ldc == N)
// BatchNorm-backward epilogue operands (gemm_f32 / conv3x3_f32 data grad with stats): C is the
// gradient of a BN(+ReLU) output; x / mask / save are that BN's input, forward ReLU mask bits and
// save (mean, invstd); stats receives [tiles][2][N] = [sum dz | sum dz (x - mean)].
struct BnBwdEpi {
  const float* x;
  const uint8_t* mask;  // null with relu: the ReLU test is recomputed from x and save's scale / shift
  const float* save;
  int relu;
};
// BatchNorm-apply prologue (gemm_f32 / conv3x3_f32 forward and weight grad): the activation
// operand holds a BN input x of C channels; the GEMM consumes act(scale * x + shift) computed as
// it loads (scale / shift at save + 2C / + 3C).  op: 1 = A, 2 = B (gemm_f32; conv3x3_f32 picks).
struct BnApplyPro {
  const float* save;
  int C;
  int relu;
  int op;
};
int gemm_f32(const float* A, bool a_kcontig, int64_t lda, const float* B, bool b_kcontig, int64_t ldb, float* C,
              int64_t ldc, int M, int N, int K, int splits, hipStream_t stream, int tile = 0,
             float* stats = nullptr, const BnBwdEpi* bnb = nullptr, const BnApplyPro* xf = nullptr);
// 3x3 (pad 1) convolution of NHWC fp32 activations as an implicit GEMM on the same kernel (no
// im2col).  dir 0: C = y [N,Ho,Wo,Cout] from act = x, other = W [Cout][3][3][Cin] (+ stats as
// gemm_f32); dir 1 (stride 1): C = dx [N,H,W,Cin] from act = dY, other = W; dir 2: C = dW
// [Cout][3][3][Cin] from act = x, other = dY (splits 0 = auto split-K, C zeroed).  Cin % 32 == 0
// (dir 0), Cout % 32 == 0 (dir 1), Cin % 4 == 0 (dir 2), N*Ho*Wo and N*H*W < 2^24.  Returns the
// row tiles of C.
// ksize 1: a strided 1x1 (pad 0) convolution on the same path (one tap).
int conv3x3_f32(int dir, const float* act, const float* other, float* C, int N, int H, int W, int Cin, int Cout,
                int stride, int splits, int tile, float* stats, hipStream_t stream, int ksize = 3,
                const BnBwdEpi* bnb = nullptr, const BnApplyPro* xf = nullptr);

// ---------------------------------------------------------------- ef.hip (elementwise)
void axpby(const float* x, const float* y, float* out, int64_t n, float a, float b, hipStream_t stream);
void scale_inplace(float* x, int64_t n, float s, hipStream_t stream);

// ---------------------------------------------------------------- inceptionn.hip
int64_t inceptionn_tiles(int64_t n);
void inceptionn_count(const float* x, int64_t n, int e_b, int mid, int32_t* cnt, int32_t* totals, hipStream_t stream);
// totals (device, written by inceptionn_count) -> unified value stream of cap_bytes (drops the
// lowest classes first when they do not fit; cap_bytes >= 4 n never drops)
void inceptionn_encode(const float* x, int64_t n, int e_b, int mid, const int32_t* off, const int32_t* totals,
                       uint8_t* stream, int64_t cap_bytes, uint8_t* codes, hipStream_t stream_);
// W rank-strided payloads (stream at stream_off, codes at codes_off of each row) decoded + summed
void inceptionn_decode(const uint8_t* base, int64_t rank_stride, int64_t stream_off, int64_t codes_off, int n_ranks,
                       int64_t n, int32_t* cnt, int32_t* totals, float scale, float* out, bool accumulate,
                       hipStream_t stream);

// ---------------------------------------------------------------- adaq.hip
void adaq_sample(const float* x, int n_seg, const int64_t* seg_off, const int64_t* samp_off, int64_t n_samples,
                 SeedArg seed, float* samples, hipStream_t stream);
void adaq_prepare(const ChunkTable& ct, int n_seg, const float* x, const int64_t* seg_off, const int64_t* samp_off,
                  const float* stats, float ratio, int32_t* count, float* target, int32_t* kseg, float* fallback,
                  float* thr, int32_t* done, hipStream_t stream);
void adaq_refine(const ChunkTable& ct, int n_seg, const float* x, const TopkState* st, const float* fallback,
                 const float* target, int max_iters, float* thr, int32_t* count, int32_t* done, hipStream_t stream);
void adaq_offsets(int n_seg, const int32_t* count, int32_t* goff, int32_t* cursor, hipStream_t stream);
void adaq_compact(const ChunkTable& ct, int n_seg, const int32_t* seg_chunk_begin, const float* x, const float* thr,
                  const int32_t* goff, int32_t* cursor, int32_t* idx, int64_t cap, double* psum, float* means,
                  int32_t* counts, hipStream_t stream);
// one rank's capacity payload -> out (+)= means[group] * scale at its indices (goff_ws: n_groups+1)
void adaq_decode(int n_groups, const float* means, const int32_t* counts, const int32_t* idx, int64_t cap,
                 int32_t* goff_ws, float* out, float scale, hipStream_t stream);

// ---------------------------------------------------------------- ef.hip (bucket gather)
constexpr int kGatherSegs = 120;
void gather_segments(const void* const* src, bool bf16, const int64_t* dst_off, const int64_t* len, int n_seg,
                     float* dst, hipStream_t stream);
void cast_segments_bf16(const float* const* src, uint16_t* const* dst, const int64_t* len, int n_seg,
                        hipStream_t stream);

// ---------------------------------------------------------------- bnact.hip
// fused training-mode BatchNorm (+ residual) (+ ReLU), channels_last bf16 / fp32
bool bn_supported(int C);  // C % 8 == 0, C <= 2048, C % 256 == 0 above 256
int64_t bn_workspace_floats(int64_t M, int C);  // `ws` size (fp32 words, 8-B aligned base)
int bn_fused_v(int64_t M, int C, bool bwd);      // single-launch vectors/thread, 0 = two-kernel path
void bn_set_fused(bool on);                       // runtime switch (default: env GRACE_BN_FUSED == 1)
int bn_fused_v_f32(int64_t M, int C, bool bwd);  // fp32 single-launch rows/thread, 0 = two-kernel path
void bn_set_fused_f32(bool on);                   // runtime switch (default off; env GRACE_BN_FUSED_F32=1 on)
unsigned bn_spin_timeouts();                     // bounded co-residency waits that timed out (must stay 0)
// x/res/y/dy/dx/dres: bf16 (uint16_t) or fp32 (`fp32`) elements; fp32 uses the two-kernel path
void bn_act_forward(const void* x, const void* res, bool fp32, int64_t M, int C, const float* gamma,
                    const float* beta, float* running_mean, float* running_var, int64_t* nbt, float momentum,
                    float eps, bool relu, float* save, float* ws, void* y, uint8_t* relu_mask, hipStream_t stream);
// dy2 (may be nullptr): a second gradient contribution of the same layout, summed into dy
void bn_act_forward_from_partials(const float* x, const float* res, const float* part, int tiles, int64_t M, int C,
                                  const float* gamma, const float* beta, float* running_mean, float* running_var,
                                  int64_t* nbt, float momentum, float eps, bool relu, float* save, float* y,
                                  uint8_t* mask, hipStream_t stream, double* ws = nullptr);
// Statistics pass only (save, running statistics; no apply) over an fp32 [M][C] activation.
void bn_stats_only(const float* x, int64_t M, int C, const float* gamma, const float* beta, float* running_mean,
                   float* running_var, int64_t* nbt, float momentum, float eps, float* save, float* ws,
                   hipStream_t stream);
// Statistics only (no apply): the BN output is consumed by a GEMM's BnApplyPro prologue.
void bn_fold_partials(const float* part, int tiles, int64_t M, int C, const float* gamma, const float* beta,
                      float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps, float* save,
                      hipStream_t stream, double* ws = nullptr);
// Backward from the consuming conv's data-grad GEMM epilogue partials (BnBwdEpi): fold + dx pass.
void bn_act_backward_from_partials(const float* dy, const float* x, const uint8_t* mask, const float* part, int tiles,
                                   int64_t M, int C, const float* gamma, const float* save, bool relu, float* dgamma,
                                   float* dbeta, float* coef, float* dx, hipStream_t stream, double* ws = nullptr);
// doubles of the two-level fold workspace for `tiles` partial rows of C channels
inline int64_t bn_fold_ws_doubles(int64_t tiles, int64_t C) { return ((tiles + 31) / 32) * 2 * C; }
// fixed-order tree reductions in every BN backward (run-to-run bitwise reproducible) instead of
// the default atomic totals (GRACE_BN_DETERMINISTIC=1 at start-up does the same)
void bn_set_deterministic(bool on);
// layers with <= n row chunks per channel tile use the atomic backward totals (0: none)
void bn_set_atomic_chunks(int n);
int bn_atomic_chunks();
void bn_act_backward(const void* dy, const void* dy2, const void* x, bool fp32, const uint8_t* relu_mask, int64_t M,
                     int C, const float* gamma, const float* save, bool relu, float* dgamma, float* dbeta,
                     float* coef, float* ws, void* dx, void* dres, bool deterministic, hipStream_t stream);

// BN + ReLU + max pool (k x k, stride s, padding pad) over NHWC x: stats + one normalise/ReLU/pool
// pass (pooled y [N, OH, OW, C], 1-byte in-window argmax code per pooled element).  Backward:
// maxpool_backward, then bn_act_backward with relu_mask == nullptr (mask recomputed from x)
void bn_act_pool_forward(const void* x, bool fp32, int N, int H, int W, int C, const float* gamma, const float* beta,
                         float* running_mean, float* running_var, int64_t* nbt, float momentum, float eps, int k,
                         int s, int pad, int OH, int OW, float* save, float* ws, void* y, uint8_t* code,
                         hipStream_t stream);

// conv bias (+ ReLU) over [M, C] channels_last rows (same channel constraints as BN):
// y = act(x + bias); backward dz = dy * [y > 0] and dbias = Σ_rows dz in ONE pass (ws as BN)
void bias_act_forward(const void* x, const float* bias, bool fp32, int64_t M, int C, bool relu, void* y,
                      hipStream_t stream);
void bias_act_backward(const void* dy, const void* y, bool fp32, int64_t M, int C, bool relu, float* dbias, float* ws,
                       void* dz, hipStream_t stream);

// ---------------------------------------------------------------- pool.hip
// NHWC max pooling (C % 8 == 0, k <= 15) with a 1-byte in-window argmax code per output element
void maxpool_forward(const void* x, bool fp32, int N, int H, int W, int C, int OH, int OW, int k, int s, int pad,
                     void* y, uint8_t* code, hipStream_t stream);
void maxpool_backward(const void* dy, const uint8_t* code, bool fp32, int N, int H, int W, int C, int OH, int OW,
                      int k, int s, int pad, void* dx, hipStream_t stream,
                      const void* dy2 = nullptr);
// global average pool backward over channels_last: dx[n, h, w, c] = dy[n, c] / HW (C % 8 == 0)
void global_avgpool_backward(const void* dy, bool fp32, int N, int HW, int C, void* dx, hipStream_t stream);

// ---------------------------------------------------------------- optim.hip
constexpr int kSgdSegs = 64;
// buf[i] / w16[i] may be nullptr (no momentum / no bf16 working copy)
// Process-wide communication health words (csrc/comm/health.cpp): host-mapped copy (device
// writes it at system scope, the host reads it without a sync) + a device copy of the fault
// flag.  Null until health_init() (called before any capture by FusedSGD / XgmiComm).
constexpr int kHealthWords = 16;
constexpr int kHealthFault = 0;
constexpr int kHealthXgmiTimeouts = 1;
// capacity payloads (ops/cappayload.py) whose selection did not fit: the sent subset was cut
// (Threshold / DGC: spilled into the residual or dropped; INCEPTIONN: classes dropped).  Counted
// by the kernels themselves, so a lossy step is visible also inside a replayed HIP graph.
constexpr int kHealthCapOverflow = 2;
// host-mapped overflow counter (nullptr before health_init): one system-scope add per event
__device__ __forceinline__ void health_count_overflow(uint32_t* host_dev) {
  if (host_dev != nullptr)
    __hip_atomic_fetch_add(host_dev + kHealthCapOverflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr int kHealthMaxDevices = 64;
struct HealthWords {
  uint32_t* host;      // host pointer
  uint32_t* host_dev;  // device alias of the host words (portable: valid on every device)
  uint32_t* dev[kHealthMaxDevices];  // per-device copy of the fault flag, by device ordinal (null until init)
};
const HealthWords& health_words();
// allocates the host words once and the device words of `device` (-1: the current device)
void health_init(int device = -1);
// the fault words of `device` (nullptr when health_init never ran for it; never allocates, so
// it is safe while a stream is being captured)
uint32_t* health_dev(int device);

void sgd_step(float* const* p, const float* const* g, float* const* buf, uint16_t* const* w16, const int64_t* len,
              int n_seg, float lr, float momentum, float dampening, float wd, bool nesterov, bool maximize,
              bool first, hipStream_t stream);

}  // namespace grace
