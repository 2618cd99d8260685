// Python bindings for the grace_amd native library (module grace_amd._C).
//
// Every op validates device/dtype/contiguity on the host, then calls the raw-pointer launcher
// on PyTorch's *current* HIP stream so it orders correctly with surrounding torch work and
// can be captured into a HIP graph.
#include <array>

#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "grace_kernels.h"

namespace {

using at::Tensor;

// On ROCm PyTorch exposes GPUs as device type "cuda"; the *MasqueradingAsCUDA* guard/stream
// are the HIP implementations registered for that device type.
inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " must be " #dt)
// one statement each (safe under an unbraced `if`)
#define CHECK_F32(t)         \
  do {                       \
    CHECK_DEV(t);            \
    CHECK_CONTIG(t);         \
    CHECK_DT(t, at::kFloat); \
  } while (0)
#define CHECK_I32(t)       \
  do {                     \
    CHECK_DEV(t);          \
    CHECK_CONTIG(t);       \
    CHECK_DT(t, at::kInt); \
  } while (0)
#define CHECK_I64(t)        \
  do {                      \
    CHECK_DEV(t);           \
    CHECK_CONTIG(t);        \
    CHECK_DT(t, at::kLong); \
  } while (0)

inline const int64_t* opt_i64(const c10::optional<Tensor>& t) {
  if (!t.has_value()) return nullptr;
  CHECK_I64((*t));
  return t->data_ptr<int64_t>();
}

grace::ChunkTable make_ct(const Tensor& seg, const Tensor& cb, const Tensor& ce) {
  CHECK_I32(seg);
  CHECK_I64(cb);
  CHECK_I64(ce);
  TORCH_CHECK(seg.numel() == cb.numel() && cb.numel() == ce.numel(), "chunk table size mismatch");
  grace::ChunkTable ct;
  ct.seg = seg.data_ptr<int32_t>();
  ct.begin = cb.data_ptr<int64_t>();
  ct.end = ce.data_ptr<int64_t>();
  ct.n_chunks = (int32_t)seg.numel();
  return ct;
}

// ------------------------------------------------------------------------------ top-k
void topk_select(const Tensor& g, const c10::optional<Tensor>& r, const Tensor& x, double beta,
                 double gamma, int64_t mode, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                 const Tensor& kseg, const Tensor& state, const Tensor& hist) {
  CHECK_F32(g);
  CHECK_F32(x);
  CHECK_I32(kseg);
  CHECK_I32(state);
  CHECK_I32(hist);
  const int n_seg = (int)kseg.numel();
  TORCH_CHECK(state.numel() >= 2 * n_seg, "state too small");
  TORCH_CHECK(hist.numel() >= (int64_t)n_seg * 2048, "hist too small");
  TORCH_CHECK(x.numel() == g.numel(), "x/g size mismatch");
  const float* rp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(r.has_value(), "mode 1 needs a residual");
    CHECK_F32((*r));
    TORCH_CHECK(r->numel() == g.numel(), "r/g size mismatch");
    rp = r->data_ptr<float>();
  }
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(g.device());
  grace::topk_select_bucket(ct, n_seg, g.data_ptr<float>(), rp, x.data_ptr<float>(), (float)beta,
                            (float)gamma, (int)mode, kseg.data_ptr<int32_t>(),
                            reinterpret_cast<grace::TopkState*>(state.data_ptr<int32_t>()),
                            hist.data_ptr<int32_t>(), cur_stream());
}

void topk_compact(const Tensor& x, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                  const Tensor& state, const Tensor& out_off, const Tensor& counters,
                  const Tensor& out_val, const Tensor& out_idx, const c10::optional<Tensor>& resid,
                  int64_t idx_base) {
  CHECK_F32(x);
  CHECK_I32(state);
  CHECK_I64(out_off);
  CHECK_I32(counters);
  CHECK_F32(out_val);
  CHECK_I32(out_idx);
  const int n_seg = (int)out_off.numel() - 1;
  TORCH_CHECK(n_seg >= 1, "out_off must have n_seg+1 entries");
  TORCH_CHECK(counters.numel() >= 2 * n_seg, "counters too small");
  float* rp = nullptr;
  if (resid.has_value()) {
    CHECK_F32((*resid));
    TORCH_CHECK(resid->numel() == x.numel(), "resid size mismatch");
    rp = resid->data_ptr<float>();
  }
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::topk_compact_bucket(ct, n_seg, x.data_ptr<float>(),
                             reinterpret_cast<const grace::TopkState*>(state.data_ptr<int32_t>()),
                             out_off.data_ptr<int64_t>(), counters.data_ptr<int32_t>(),
                             out_val.data_ptr<float>(), out_idx.data_ptr<int32_t>(), rp, idx_base,
                             cur_stream());
}

// two-pass Top-K (csrc/kernels/topk.hip topk_ef_bucket); x may alias g (NoneMemory, mode 0)
void topk_ef(const Tensor& g, const Tensor& x, double beta, double gamma, int64_t mode, bool zero,
             const Tensor& seg, const Tensor& cb, const Tensor& ce, const Tensor& seg_chunk_begin,
             const Tensor& kseg, const Tensor& state, const Tensor& hist, const Tensor& ctr, const Tensor& ccnt,
             const Tensor& out_off, const Tensor& out_val, const Tensor& out_idx, const Tensor& cand_val,
             const Tensor& cand_idx) {
  CHECK_F32(g);
  CHECK_F32(x);
  CHECK_I32(seg_chunk_begin);
  CHECK_I32(kseg);
  CHECK_I32(state);
  CHECK_I32(hist);
  CHECK_I32(ctr);
  CHECK_I32(ccnt);
  CHECK_I64(out_off);
  CHECK_F32(out_val);
  CHECK_I32(out_idx);
  CHECK_F32(cand_val);
  CHECK_I32(cand_idx);
  const int n_seg = (int)kseg.numel();
  const int64_t n = g.numel();
  TORCH_CHECK(x.numel() == n, "x/g size mismatch");
  TORCH_CHECK(n < ((int64_t)1 << 31), "bucket too large for int32 indices");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(g.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0,
              "g and x must be 16-byte aligned");
  TORCH_CHECK(state.numel() >= 2 * n_seg && hist.numel() >= (int64_t)n_seg * 2048 && ctr.numel() >= 3 * n_seg,
              "state / hist / ctr too small");
  TORCH_CHECK(seg_chunk_begin.numel() == n_seg + 1 && ccnt.numel() >= 3 * seg.numel(), "chunk tables");
  TORCH_CHECK(out_off.numel() == n_seg + 1, "out_off size");
  TORCH_CHECK(cand_val.numel() >= n && cand_idx.numel() >= n, "candidate buffers must hold the bucket");
  TORCH_CHECK(mode == 0 || x.data_ptr() != g.data_ptr(), "mode 1 needs a residual distinct from g");
  TORCH_CHECK(!zero || x.data_ptr() != g.data_ptr(), "zeroing needs a residual distinct from g");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(g.device());
  grace::topk_ef_bucket(ct, seg_chunk_begin.data_ptr<int32_t>(), n_seg, g.data_ptr<float>(), x.data_ptr<float>(), n,
                        (float)beta, (float)gamma, (int)mode, zero ? 1 : 0, kseg.data_ptr<int32_t>(),
                        reinterpret_cast<grace::TopkState*>(state.data_ptr<int32_t>()), hist.data_ptr<int32_t>(),
                        ctr.data_ptr<int32_t>(), ccnt.data_ptr<int32_t>(), out_off.data_ptr<int64_t>(),
                        out_val.data_ptr<float>(), out_idx.data_ptr<int32_t>(), cand_val.data_ptr<float>(),
                        cand_idx.data_ptr<int32_t>(), cur_stream());
}

void sparse_scatter_add_dev(const Tensor& val, const Tensor& idx, const Tensor& count, const Tensor& out,
                            double scale, bool accumulate, bool count_overflow) {
  CHECK_F32(val);
  CHECK_I32(idx);
  CHECK_I32(count);
  CHECK_F32(out);
  TORCH_CHECK(val.numel() == idx.numel() && count.numel() >= 1, "val/idx size mismatch");
  DevGuard guard(out.device());
  grace::sparse_scatter_add_dev(val.data_ptr<float>(), idx.data_ptr<int32_t>(), count.data_ptr<int32_t>(),
                                val.numel(), out.data_ptr<float>(), (float)scale, accumulate, cur_stream(),
                                count_overflow);
}

void sparse_scatter_add(const Tensor& val, const Tensor& idx, const Tensor& out, double scale,
                        bool accumulate) {
  CHECK_F32(val);
  CHECK_I32(idx);
  CHECK_F32(out);
  TORCH_CHECK(val.numel() == idx.numel(), "val/idx size mismatch");
  DevGuard guard(out.device());
  grace::sparse_scatter_add(val.data_ptr<float>(), idx.data_ptr<int32_t>(), val.numel(),
                            out.data_ptr<float>(), (float)scale, accumulate, cur_stream());
}

// ------------------------------------------------------------------------------ random-k / threshold
void randk_gather(const Tensor& x, const Tensor& seg_off, const Tensor& out_off, const Tensor& seeds,
                  const c10::optional<Tensor>& step, const Tensor& vals, const c10::optional<Tensor>& resid) {
  CHECK_F32(x);
  CHECK_I64(seg_off);
  CHECK_I64(out_off);
  CHECK_I64(seeds);
  CHECK_F32(vals);
  const int n_seg = (int)seeds.numel();
  TORCH_CHECK(seg_off.numel() == n_seg + 1 && out_off.numel() == n_seg + 1, "offset tables must be n_seg+1");
  float* rp = nullptr;
  if (resid.has_value()) {
    CHECK_F32((*resid));
    TORCH_CHECK(resid->data_ptr() == x.data_ptr(), "residual zeroing requires x to be the residual buffer");
    rp = resid->data_ptr<float>();
  }
  DevGuard guard(x.device());
  grace::randk_gather(x.data_ptr<float>(), n_seg, seg_off.data_ptr<int64_t>(), out_off.data_ptr<int64_t>(),
                      seeds.data_ptr<int64_t>(), opt_i64(step), vals.numel(), vals.data_ptr<float>(), rp,
                      cur_stream());
}

// vals: [n_ranks, rank_stride] fp32 view (row r = rank r payload, first K entries used)
void randk_scatter(const Tensor& vals, int64_t rank_stride, int64_t n_ranks, int64_t K, const Tensor& seg_off,
                   const Tensor& out_off, const Tensor& seeds, const c10::optional<Tensor>& step, const Tensor& out,
                   double scale, bool accumulate) {
  CHECK_DEV(vals);
  CHECK_DT(vals, at::kFloat);
  CHECK_I64(seg_off);
  CHECK_I64(out_off);
  CHECK_I64(seeds);
  CHECK_F32(out);
  TORCH_CHECK(vals.storage().nbytes() >= (size_t)(vals.storage_offset() + (n_ranks - 1) * rank_stride + K) * 4,
              "vals view too small");
  DevGuard guard(out.device());
  grace::randk_scatter(vals.data_ptr<float>(), rank_stride, (int)n_ranks, (int)seeds.numel(),
                       seg_off.data_ptr<int64_t>(), out_off.data_ptr<int64_t>(), seeds.data_ptr<int64_t>(),
                       opt_i64(step), K, out.data_ptr<float>(), (float)scale, accumulate, cur_stream());
}

// Bytes of the in-band payload header to clear before a compaction: the whole 16-B
// [selected, capacity, 0, 0] header when the count word heads one (ops/cappayload.py
// sparse_payload), so no stale allocator bytes ride on the wire (payload bytes identical on every
// rank and run); else the count word alone.
static int header_bytes(const Tensor& counter) {
  const int64_t avail = (int64_t)counter.storage().nbytes() - counter.storage_offset() * (int64_t)sizeof(int32_t);
  return avail >= 16 ? 16 : 4;
}

int64_t threshold_compact(const Tensor& g, const c10::optional<Tensor>& r, int64_t mode, double beta, double gamma,
                          double thr, const Tensor& out_val, const Tensor& out_idx, const Tensor& counter,
                          const c10::optional<Tensor>& resid) {
  CHECK_F32(g);
  CHECK_F32(out_val);
  CHECK_I32(out_idx);
  CHECK_I32(counter);
  TORCH_CHECK(out_val.numel() == out_idx.numel() && counter.numel() >= 1, "capacity buffers / counter");
  TORCH_CHECK(g.numel() < ((int64_t)1 << 31), "int32 indices");
  const float* rp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(r.has_value(), "mode 1 needs r");
    CHECK_F32((*r));
    rp = r->data_ptr<float>();
  }
  float* wp = nullptr;
  if (resid.has_value()) {
    CHECK_F32((*resid));
    wp = resid->data_ptr<float>();
  }
  DevGuard guard(g.device());
  grace::threshold_compact(g.data_ptr<float>(), rp, (int)mode, (float)beta, (float)gamma, g.numel(), (float)thr,
                           out_val.data_ptr<float>(), out_idx.data_ptr<int32_t>(), out_val.numel(),
                           counter.data_ptr<int32_t>(), wp, cur_stream(), header_bytes(counter));
  return 0;
}

// ------------------------------------------------------------------------------ rank-strided payload rows
// `base` is a uint8 view whose row r starts at r*rank_stride; validate the furthest byte read.
void check_rows(const Tensor& base, int64_t rank_stride, int64_t n_ranks, int64_t last_byte) {
  CHECK_DEV(base);
  CHECK_DT(base, at::kByte);
  TORCH_CHECK(n_ranks >= 1, "n_ranks >= 1");
  const int64_t need = base.storage_offset() + (n_ranks - 1) * rank_stride + last_byte;
  TORCH_CHECK((int64_t)base.storage().nbytes() >= need, "payload rows out of bounds");
}

inline const float* opt_f32(const c10::optional<Tensor>& t) {
  if (!t.has_value()) return nullptr;
  CHECK_F32((*t));
  return t->data_ptr<float>();
}
inline grace::SeedArg seed_arg(int64_t seed, const c10::optional<Tensor>& step) {
  grace::SeedArg sa{(uint64_t)seed, nullptr};
  if (step.has_value()) {
    CHECK_I64((*step));
    sa.step = step->data_ptr<int64_t>();
  }
  return sa;
}
inline float* opt_f32_mut(const c10::optional<Tensor>& t) {
  if (!t.has_value()) return nullptr;
  CHECK_F32((*t));
  return t->data_ptr<float>();
}

// ------------------------------------------------------------------------------ sign bits
void sign_pack(const Tensor& g, const c10::optional<Tensor>& r, int64_t ef_mode, double beta, double gamma,
               const c10::optional<Tensor>& mom, double mom_beta, bool mom_valid, const c10::optional<Tensor>& vT,
               const c10::optional<Tensor>& vF, const c10::optional<Tensor>& resid, bool neg, const Tensor& words,
               const Tensor& seg, const Tensor& cb, const Tensor& ce, const Tensor& seg_start,
               const Tensor& word_off, int64_t n_words) {
  CHECK_F32(g);
  CHECK_DEV(words);
  CHECK_CONTIG(words);
  CHECK_DT(words, at::kLong);
  CHECK_I64(seg_start);
  CHECK_I64(word_off);
  TORCH_CHECK(words.numel() >= n_words, "words too small");
  if (ef_mode == 1) TORCH_CHECK(r.has_value(), "ef_mode 1 needs r");
  if (resid.has_value()) TORCH_CHECK(vT.has_value() && vF.has_value(), "residual needs vT/vF");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(g.device());
  grace::sign_pack(ct, seg_start.data_ptr<int64_t>(), word_off.data_ptr<int64_t>(), g.data_ptr<float>(), opt_f32(r),
                   (int)ef_mode, (float)beta, (float)gamma, opt_f32_mut(mom), (float)mom_beta, mom_valid ? 1 : 0,
                   opt_f32(vT), opt_f32(vF), opt_f32_mut(resid), neg,
                   reinterpret_cast<uint64_t*>(words.data_ptr<int64_t>()), cur_stream());
}

void sign_unpack(const Tensor& base, int64_t rank_stride, int64_t words_off, int64_t vals_off, int64_t n_ranks,
                 bool vote, double scale, const Tensor& out, bool accumulate, const Tensor& seg, const Tensor& cb,
                 const Tensor& ce, const Tensor& seg_start, const Tensor& word_off, int64_t nw) {
  CHECK_F32(out);
  CHECK_I64(seg_start);
  CHECK_I64(word_off);
  const int n_seg = (int)seg_start.numel() - 1;
  check_rows(base, rank_stride, n_ranks, std::max(words_off + nw * 8, vote ? (int64_t)0 : vals_off + 8 * n_seg));
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(out.device());
  grace::sign_unpack(ct, seg_start.data_ptr<int64_t>(), word_off.data_ptr<int64_t>(), base.data_ptr<uint8_t>(),
                     rank_stride, words_off, vals_off, n_seg, (int)n_ranks, vote, (float)scale, out.data_ptr<float>(),
                     accumulate, cur_stream());
}

// ------------------------------------------------------------------------------ quantizers
void qsgd_quantize(const Tensor& x, const Tensor& norms, double s, int64_t seed, const c10::optional<Tensor>& step,
                   const Tensor& codes,
                   const c10::optional<Tensor>& resid, const Tensor& seg, const Tensor& cb, const Tensor& ce) {
  CHECK_F32(x);
  CHECK_F32(norms);
  CHECK_DEV(codes);
  CHECK_CONTIG(codes);
  TORCH_CHECK(codes.numel() >= x.numel(), "codes too small");
  // 1 int8, 2 int16, 4 int32, 3 fp16 integer levels (quant.hip)
  const int cb_ = codes.scalar_type() == at::kHalf ? 3 : (int)codes.element_size();
  TORCH_CHECK(cb_ == 1 || cb_ == 2 || cb_ == 3 || cb_ == 4, "codes must be int8/int16/int32/fp16");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::qsgd_quantize(ct, x.data_ptr<float>(), norms.data_ptr<float>(), (float)s, seed_arg(seed, step), codes.data_ptr(),
                       cb_, opt_f32_mut(resid), cur_stream());
}

// shared_norms: [n_seg] norms used for every rank (shared-scale codes; the rows then hold codes only)
void qsgd_aggregate(const Tensor& base, int64_t rank_stride, int64_t codes_off, int64_t norms_off, int64_t code_bytes,
                    int64_t n_ranks, double s, double scale, const Tensor& out, bool accumulate, const Tensor& seg,
                    const Tensor& cb, const Tensor& ce, int64_t n_seg, const c10::optional<Tensor>& shared_norms) {
  CHECK_F32(out);
  // bytes of the code row: 3 = fp16 codes; kPacked2 / kPacked4 = 2- / 4-bit packed codes
  const int64_t code_row = code_bytes == grace::kPacked2   ? (out.numel() * 2 + 7) / 8
                           : code_bytes == grace::kPacked4 ? (out.numel() * 4 + 7) / 8
                           : out.numel() * (code_bytes == 3 ? 2 : code_bytes);
  const float* sn = nullptr;
  if (shared_norms.has_value()) {
    CHECK_F32((*shared_norms));
    TORCH_CHECK(shared_norms->numel() >= n_seg, "shared_norms too small");
    sn = shared_norms->data_ptr<float>();
    check_rows(base, rank_stride, n_ranks, codes_off + code_row);
  } else {
    check_rows(base, rank_stride, n_ranks, std::max(codes_off + code_row, norms_off + 4 * n_seg));
  }
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(out.device());
  grace::qsgd_aggregate(ct, base.data_ptr<uint8_t>(), rank_stride, codes_off, norms_off, sn, (int)code_bytes,
                        (int)n_ranks, (float)s, (float)scale, out.data_ptr<float>(), accumulate, cur_stream());
}

// int8 codes in [-s, s] -> `bits`-bit fields (code + s) of a uint8 row
void qsgd_pack(const Tensor& codes, int64_t s, int64_t bits, const Tensor& out) {
  TORCH_CHECK(codes.is_cuda() && codes.scalar_type() == at::kChar && codes.is_contiguous(), "codes: int8 GPU");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kByte && out.is_contiguous(), "out: uint8 GPU");
  TORCH_CHECK((bits == 2 && s == 1) || (bits == 4 && s >= 1 && s <= 7), "packing: 2 bits for s = 1, 4 bits for s <= 7");
  TORCH_CHECK(out.numel() >= (codes.numel() * bits + 7) / 8, "out too small");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0, "out must be 8-B aligned");
  DevGuard guard(out.device());
  grace::qsgd_pack(codes.data_ptr<int8_t>(), codes.numel(), (int)s, (int)bits, out.data_ptr<uint8_t>(), cur_stream());
}

void tern_quantize(const Tensor& x, const Tensor& clips, const Tensor& scal, int64_t seed,
                   const c10::optional<Tensor>& step, const Tensor& words,
                   const c10::optional<Tensor>& resid, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                   const Tensor& seg_start, const Tensor& word_off, int64_t n_words) {
  CHECK_F32(x);
  CHECK_F32(clips);
  CHECK_F32(scal);
  CHECK_DEV(words);
  CHECK_DT(words, at::kLong);
  CHECK_I64(seg_start);
  CHECK_I64(word_off);
  TORCH_CHECK(words.numel() >= 2 * n_words, "words too small");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::tern_quantize(ct, seg_start.data_ptr<int64_t>(), word_off.data_ptr<int64_t>(), x.data_ptr<float>(),
                       clips.data_ptr<float>(), scal.data_ptr<float>(), seed_arg(seed, step),
                       reinterpret_cast<uint64_t*>(words.data_ptr<int64_t>()), opt_f32_mut(resid), cur_stream());
}

void tern_aggregate(const Tensor& base, int64_t rank_stride, int64_t words_off, int64_t scal_off, int64_t n_ranks,
                    double scale, const Tensor& out, bool accumulate, const Tensor& seg, const Tensor& cb,
                    const Tensor& ce, const Tensor& seg_start, const Tensor& word_off, int64_t nw) {
  CHECK_F32(out);
  const int64_t n_seg = seg_start.numel() - 1;
  check_rows(base, rank_stride, n_ranks, std::max(words_off + 16 * nw, scal_off + 4 * n_seg));
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(out.device());
  grace::tern_aggregate(ct, seg_start.data_ptr<int64_t>(), word_off.data_ptr<int64_t>(), base.data_ptr<uint8_t>(),
                        rank_stride, words_off, scal_off, (int)n_ranks, (float)scale, out.data_ptr<float>(), accumulate,
                        cur_stream());
}

void natural_encode(const Tensor& x, int64_t seed, const c10::optional<Tensor>& step, const Tensor& codes,
                    const c10::optional<Tensor>& resid) {
  CHECK_F32(x);
  CHECK_DEV(codes);
  CHECK_DT(codes, at::kByte);
  TORCH_CHECK(codes.numel() >= x.numel(), "codes too small");
  DevGuard guard(x.device());
  grace::natural_encode(x.data_ptr<float>(), x.numel(), seed_arg(seed, step), codes.data_ptr<uint8_t>(), opt_f32_mut(resid),
                        cur_stream());
}

void natural_aggregate(const Tensor& base, int64_t rank_stride, int64_t n_ranks, double scale, const Tensor& out,
                       bool accumulate) {
  CHECK_F32(out);
  check_rows(base, rank_stride, n_ranks, out.numel());
  DevGuard guard(out.device());
  grace::natural_aggregate(base.data_ptr<uint8_t>(), rank_stride, out.numel(), (int)n_ranks, (float)scale,
                           out.data_ptr<float>(), accumulate, cur_stream());
}

void u8_encode(const Tensor& x, const Tensor& scales, const Tensor& codes, const c10::optional<Tensor>& resid,
               const Tensor& seg, const Tensor& cb, const Tensor& ce) {
  CHECK_F32(x);
  CHECK_F32(scales);
  CHECK_DEV(codes);
  CHECK_DT(codes, at::kChar);
  TORCH_CHECK(codes.numel() >= x.numel(), "codes too small");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::u8_encode(ct, x.data_ptr<float>(), scales.data_ptr<float>(), codes.data_ptr<int8_t>(), opt_f32_mut(resid),
                   cur_stream());
}

void u8_aggregate(const Tensor& base, int64_t rank_stride, int64_t codes_off, int64_t scal_off, int64_t n_ranks,
                  double scale, const Tensor& out, bool accumulate, const Tensor& seg, const Tensor& cb,
                  const Tensor& ce, int64_t n_seg) {
  CHECK_F32(out);
  check_rows(base, rank_stride, n_ranks, std::max(codes_off + out.numel(), scal_off + 4 * n_seg));
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(out.device());
  grace::u8_aggregate(ct, base.data_ptr<uint8_t>(), rank_stride, codes_off, scal_off, (int)n_ranks, (float)scale,
                      out.data_ptr<float>(), accumulate, cur_stream());
}

// ------------------------------------------------------------------------------ DGC
// u / v (optional, DgcMemory state of x's layout): x is the raw gradient, the samples are taken
// of the compensated v' = v + (m u + g) (first: g) without writing it
void dgc_sample(const Tensor& x, const Tensor& seg_off, const Tensor& samp_off, int64_t seed,
                const c10::optional<Tensor>& step, const Tensor& samples, const c10::optional<Tensor>& u,
                const c10::optional<Tensor>& v, double momentum, bool first) {
  CHECK_F32(x);
  CHECK_I64(seg_off);
  CHECK_I64(samp_off);
  CHECK_F32(samples);
  TORCH_CHECK(seg_off.numel() == samp_off.numel(), "offset tables");
  const bool comp = u.has_value() && u->defined();
  if (comp) {
    CHECK_F32(*u);
    CHECK_F32(*v);
    TORCH_CHECK(u->numel() == x.numel() && v->numel() == x.numel(), "dgc_sample: u / v like x");
  }
  DevGuard guard(x.device());
  grace::dgc_sample(x.data_ptr<float>(), (int)seg_off.numel() - 1, seg_off.data_ptr<int64_t>(),
                    samp_off.data_ptr<int64_t>(), samples.numel(), seed_arg(seed, step), samples.data_ptr<float>(),
                    comp ? u->data_ptr<float>() : nullptr, comp ? v->data_ptr<float>() : nullptr, (float)momentum,
                    first ? 1 : 0, cur_stream());
}

// u / v (optional): x is the raw gradient; the first count pass applies DgcMemory's compensate in
// place (u = m u + g; v = v + u; first: u = v = g) and later passes read v
void dgc_refine(const Tensor& x, const Tensor& state, const Tensor& target, int64_t max_iters, const Tensor& thr,
                const Tensor& count, const Tensor& done, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                const Tensor& ccnt, const Tensor& fnode, const c10::optional<Tensor>& u,
                const c10::optional<Tensor>& v, double momentum, bool first, bool init) {
  CHECK_F32(x);
  CHECK_I32(state);
  CHECK_F32(target);
  CHECK_F32(thr);
  CHECK_I32(count);
  CHECK_I32(done);
  const int n_seg = (int)target.numel();
  TORCH_CHECK(thr.numel() == n_seg && count.numel() >= 32 * n_seg && done.numel() == n_seg && state.numel() >= 2 * n_seg,
              "per-segment tables (count: 32 words per segment)");
  CHECK_I32(ccnt);
  CHECK_I32(fnode);
  TORCH_CHECK(ccnt.numel() >= 32 * seg.numel() && fnode.numel() >= n_seg, "dgc_refine: ccnt [32 n_chunks] / fnode [n_seg]");
  const bool comp = u.has_value() && u->defined();
  if (comp) {
    CHECK_F32(*u);
    CHECK_F32(*v);
    TORCH_CHECK(u->numel() == x.numel() && v->numel() == x.numel() && u->is_contiguous() && v->is_contiguous() &&
                    (reinterpret_cast<uintptr_t>(u->data_ptr()) - reinterpret_cast<uintptr_t>(x.data_ptr())) % 16 == 0 &&
                    (reinterpret_cast<uintptr_t>(v->data_ptr()) - reinterpret_cast<uintptr_t>(x.data_ptr())) % 16 == 0,
                "dgc_refine: u / v contiguous like x with x's 16-B alignment");
  }
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::dgc_refine(ct, n_seg, x.data_ptr<float>(), reinterpret_cast<const grace::TopkState*>(state.data_ptr<int32_t>()),
                    target.data_ptr<float>(), (int)max_iters, thr.data_ptr<float>(), count.data_ptr<int32_t>(),
                    done.data_ptr<int32_t>(), comp ? u->data_ptr<float>() : nullptr,
                    comp ? v->data_ptr<float>() : nullptr, (float)momentum, first ? 1 : 0, x.numel(),
                    ccnt.data_ptr<int32_t>(), fnode.data_ptr<int32_t>(), init, cur_stream());
}

void dgc_select_init(const Tensor& samples, const Tensor& samp_off, const Tensor& kseg, const Tensor& state,
                     const Tensor& thr, const Tensor& count, const Tensor& done, const Tensor& fnode) {
  CHECK_F32(samples);
  CHECK_I64(samp_off);
  CHECK_I32(kseg);
  CHECK_I32(state);
  CHECK_F32(thr);
  CHECK_I32(count);
  CHECK_I32(done);
  CHECK_I32(fnode);
  const int n_seg = (int)kseg.numel();
  TORCH_CHECK(samp_off.numel() == n_seg + 1 && state.numel() >= 2 * n_seg && thr.numel() == n_seg &&
                  count.numel() >= 32 * n_seg && done.numel() == n_seg && fnode.numel() >= n_seg,
              "dgc_select_init: per-segment tables");
  DevGuard guard(samples.device());
  grace::dgc_select_init(n_seg, samples.data_ptr<float>(), samp_off.data_ptr<int64_t>(), kseg.data_ptr<int32_t>(),
                         reinterpret_cast<grace::TopkState*>(state.data_ptr<int32_t>()), thr.data_ptr<float>(),
                         count.data_ptr<int32_t>(), done.data_ptr<int32_t>(), fnode.data_ptr<int32_t>(), cur_stream());
}

// capacity = out_val.numel(); vmask/umask (optional, DgcMemory fused): zeroed where sent
void dgc_compact(const Tensor& x, const Tensor& thr, const Tensor& out_val, const Tensor& out_idx,
                 const Tensor& counter, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                 const Tensor& ccnt, const Tensor& fnode, const Tensor& coff,
                 const c10::optional<Tensor>& vmask, const c10::optional<Tensor>& umask) {
  CHECK_F32(x);
  CHECK_F32(thr);
  CHECK_F32(out_val);
  CHECK_I32(out_idx);
  CHECK_I32(counter);
  TORCH_CHECK(out_val.numel() == out_idx.numel() && counter.numel() >= 1, "capacity buffers / counter");
  TORCH_CHECK(x.numel() < ((int64_t)1 << 31), "int32 indices");
  float* vp = nullptr;
  float* up = nullptr;
  if (vmask.has_value()) {
    CHECK_F32((*vmask));
    TORCH_CHECK(vmask->numel() == x.numel(), "vmask size");
    vp = vmask->data_ptr<float>();
  }
  if (umask.has_value()) {
    CHECK_F32((*umask));
    TORCH_CHECK(umask->numel() == x.numel(), "umask size");
    up = umask->data_ptr<float>();
  }
  CHECK_I32(ccnt);
  CHECK_I32(fnode);
  CHECK_I32(coff);
  TORCH_CHECK(ccnt.numel() >= 32 * seg.numel() && coff.numel() >= seg.numel() && fnode.numel() >= thr.numel(),
              "dgc_compact: ccnt [32 n_chunks] / coff [n_chunks] / fnode [n_seg]");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::dgc_compact(ct, x.data_ptr<float>(), thr.data_ptr<float>(), out_val.data_ptr<float>(),
                     out_idx.data_ptr<int32_t>(), out_val.numel(), counter.data_ptr<int32_t>(), vp, up,
                     ccnt.data_ptr<int32_t>(), fnode.data_ptr<int32_t>(), coff.data_ptr<int32_t>(), cur_stream(),
                     header_bytes(counter));
}

void dgc_compensate(const Tensor& g, const Tensor& u, const Tensor& v, double momentum, bool first) {
  CHECK_F32(g);
  CHECK_F32(u);
  CHECK_F32(v);
  TORCH_CHECK(u.numel() == g.numel() && v.numel() == g.numel(), "u / v size");
  TORCH_CHECK(((reinterpret_cast<uintptr_t>(g.data_ptr()) | reinterpret_cast<uintptr_t>(u.data_ptr()) |
                reinterpret_cast<uintptr_t>(v.data_ptr())) & 15) == 0, "g / u / v must be 16-byte aligned");
  DevGuard guard(g.device());
  grace::dgc_compensate(g.data_ptr<float>(), u.data_ptr<float>(), v.data_ptr<float>(), (float)momentum, g.numel(),
                        first, cur_stream());
}

// ------------------------------------------------------------------------------ PowerSGD
void powersgd_mq(const Tensor& x, const Tensor& small, const Tensor& out, const Tensor& mats, const Tensor& tiles,
                 int64_t mode, const c10::optional<Tensor>& comp_r, double beta, double gamma,
                 const c10::optional<Tensor>& xout, int64_t max_r, const c10::optional<Tensor>& lazy_p,
                 const c10::optional<Tensor>& lazy_q, double lazy_scale, bool zeroed,
                 const c10::optional<Tensor>& bump, const c10::optional<Tensor>& vec,
                 const c10::optional<Tensor>& vec_idx) {
  CHECK_F32(x);
  CHECK_F32(small);
  CHECK_F32(out);
  CHECK_I64(mats);
  CHECK_I32(tiles);
  TORCH_CHECK(mode == 0 || !(comp_r.has_value() || xout.has_value()), "compensation is fused into mode 0 only");
  if (comp_r.has_value()) TORCH_CHECK(xout.has_value(), "comp_r needs xout");
  if (xout.has_value()) TORCH_CHECK(xout->numel() == x.numel(), "xout size");
  if (comp_r.has_value()) TORCH_CHECK(comp_r->numel() == x.numel(), "comp_r size");
  TORCH_CHECK(lazy_p.has_value() == lazy_q.has_value(), "lazy_p and lazy_q go together");
  if (lazy_p.has_value()) {
    TORCH_CHECK(comp_r.has_value(), "the deferred residual needs comp_r (the previous M)");
    CHECK_F32((*lazy_p));
    CHECK_F32((*lazy_q));
    // the previous P / Q share this plan's layout: P [p_total] = out's size, Q [q_total] = small's
    TORCH_CHECK(lazy_p->numel() == out.numel() && lazy_q->numel() == small.numel(), "lazy P / Q sizes");
    TORCH_CHECK(lazy_p->data_ptr() != out.data_ptr(), "lazy P must not alias the P being written");
  }
  int64_t* bp = nullptr;
  if (bump.has_value()) {
    CHECK_I64((*bump));
    TORCH_CHECK(mode == 0 && tiles.numel() >= 3, "the step counter advances in a P = M Q launch with tiles");
    bp = bump->data_ptr<int64_t>();
  }
  TORCH_CHECK(vec.has_value() == vec_idx.has_value(), "vec and vec_idx go together");
  if (vec.has_value()) {
    CHECK_F32((*vec));
    CHECK_I64((*vec_idx));
    TORCH_CHECK(mode == 0 && tiles.numel() >= 3 && vec->numel() == vec_idx->numel(),
                "the 1-D segments are packed by a P = M Q launch with tiles (vec / vec_idx of one size)");
  }
  DevGuard guard(x.device());
  grace::powersgd_mq(x.data_ptr<float>(), small.data_ptr<float>(), out.data_ptr<float>(), out.numel(),
                     mats.data_ptr<int64_t>(), tiles.data_ptr<int32_t>(), (int)(tiles.numel() / 3), (int)mode,
                     opt_f32(comp_r), (float)beta, (float)gamma, opt_f32_mut(xout), (int)max_r, cur_stream(),
                     opt_f32(lazy_p), opt_f32(lazy_q), (float)lazy_scale, zeroed, bp, opt_f32_mut(vec),
                     vec_idx.has_value() ? vec_idx->data_ptr<int64_t>() : nullptr,
                     vec.has_value() ? vec->numel() : 0);
}

void gram_orthonormalize(const Tensor& buf, const Tensor& mats, int64_t which, int64_t n_mat, const Tensor& gtiles,
                         const Tensor& gtile_begin, int64_t passes, int64_t max_r,
                         const c10::optional<Tensor>& zero) {
  CHECK_F32(buf);
  CHECK_I64(mats);
  CHECK_I32(gtiles);
  CHECK_I32(gtile_begin);
  TORCH_CHECK(mats.numel() >= 6 * n_mat && gtile_begin.numel() == n_mat + 1, "gram tables");
  DevGuard guard(buf.device());
  const int64_t nt = gtiles.numel() / 2;
  auto part = at::empty({std::max<int64_t>(nt, 1) * 256}, buf.options().dtype(at::kDouble));
  auto T = at::empty({std::max<int64_t>(n_mat, 1) * 256}, buf.options());
  grace::gram_orthonormalize(buf.data_ptr<float>(), mats.data_ptr<int64_t>(), (int)n_mat, (int)which,
                             gtiles.data_ptr<int32_t>(), (int)nt, gtile_begin.data_ptr<int32_t>(),
                             part.data_ptr<double>(), T.data_ptr<float>(), (int)passes, (int)max_r, opt_f32_mut(zero),
                             zero.has_value() ? zero->numel() : 0, cur_stream());
}

void powersgd_pqt(const Tensor& P, const Tensor& Q, const c10::optional<Tensor>& out, const Tensor& mats,
                  const Tensor& tiles, const c10::optional<Tensor>& resid, int64_t max_r, double scale,
                  const c10::optional<Tensor>& save_p, const c10::optional<Tensor>& save_q,
                  const c10::optional<Tensor>& vec, const c10::optional<Tensor>& vec_idx, double vec_scale,
                  const c10::optional<Tensor>& T) {
  CHECK_F32(P);
  CHECK_F32(Q);
  CHECK_I64(mats);
  CHECK_I32(tiles);
  TORCH_CHECK(out.has_value() || resid.has_value(), "powersgd_pqt: nothing to write");
  if (out.has_value()) CHECK_F32((*out));
  if (resid.has_value()) CHECK_F32((*resid));
  if (resid.has_value() && out.has_value()) TORCH_CHECK(resid->numel() == out->numel(), "resid size");
  TORCH_CHECK(save_p.has_value() == save_q.has_value(), "save_p and save_q go together");
  if (save_p.has_value()) {
    CHECK_F32((*save_p));
    CHECK_F32((*save_q));
    TORCH_CHECK(save_p->numel() == P.numel() && save_q->numel() == Q.numel(), "save_p / save_q sizes");
  }
  TORCH_CHECK(vec.has_value() == vec_idx.has_value(), "vec and vec_idx go together");
  if (vec.has_value()) {
    CHECK_F32((*vec));
    CHECK_I64((*vec_idx));
    TORCH_CHECK(out.has_value() && tiles.numel() >= 3 && vec->numel() == vec_idx->numel(),
                "the 1-D segments are scattered by a P Q^T launch with tiles into out");
  }
  if (T.has_value()) {
    CHECK_F32((*T));
    TORCH_CHECK(max_r <= 4 && T->numel() * 6 >= mats.numel() * 16, "T: fp32 [n_mat][16], r <= 4");
  }
  DevGuard guard(P.device());
  grace::powersgd_pqt(P.data_ptr<float>(), Q.data_ptr<float>(), opt_f32_mut(out), mats.data_ptr<int64_t>(),
                      tiles.data_ptr<int32_t>(), (int)(tiles.numel() / 3), opt_f32_mut(resid), (float)scale,
                      (int)max_r, opt_f32_mut(save_p), opt_f32_mut(save_q), opt_f32(vec),
                      vec_idx.has_value() ? vec_idx->data_ptr<int64_t>() : nullptr,
                      vec.has_value() ? vec->numel() : 0, (float)vec_scale, opt_f32(T), cur_stream());
}

void powersgd_mtp_gram(const Tensor& x, const Tensor& P, const Tensor& Q, const Tensor& mats, const Tensor& tiles,
                       int64_t n_mat, const Tensor& T, int64_t passes, int64_t max_r) {
  CHECK_F32(x);
  CHECK_F32(P);
  CHECK_F32(Q);
  CHECK_F32(T);
  CHECK_I64(mats);
  CHECK_I32(tiles);
  TORCH_CHECK(max_r <= 4, "powersgd_mtp_gram: r <= 4 (larger ranks orthonormalise with the MFMA Gram kernels)");
  TORCH_CHECK(mats.numel() >= 6 * n_mat && T.numel() >= 16 * n_mat, "powersgd_mtp_gram: table sizes");
  TORCH_CHECK(passes >= 1 && passes <= 4, "powersgd_mtp_gram: 1..4 passes");
  DevGuard guard(x.device());
  grace::powersgd_mtp_gram(x.data_ptr<float>(), P.data_ptr<float>(), Q.data_ptr<float>(), mats.data_ptr<int64_t>(),
                           tiles.data_ptr<int32_t>(), (int)(tiles.numel() / 3), (int)n_mat, T.data_ptr<float>(),
                           (int)passes, (int)max_r, cur_stream());
}

void philox_normal(const Tensor& out, int64_t seed, const c10::optional<Tensor>& step,
                   const c10::optional<Tensor>& zero) {
  CHECK_F32(out);
  if (zero.has_value()) CHECK_F32((*zero));
  DevGuard guard(out.device());
  grace::philox_normal(out.data_ptr<float>(), out.numel(), seed_arg(seed, step), cur_stream(), opt_f32_mut(zero),
                       zero.has_value() ? zero->numel() : 0);
}

// ------------------------------------------------------------------------------ 16-bit cast, sketch
void cast16(const Tensor& x, const Tensor& y, bool bf16) {
  CHECK_F32(x);
  CHECK_DEV(y);
  CHECK_CONTIG(y);
  TORCH_CHECK(y.element_size() == 2 && y.numel() >= x.numel(), "y must be a 16-bit tensor of numel >= x");
  DevGuard guard(x.device());
  grace::cast16(x.data_ptr<float>(), reinterpret_cast<uint16_t*>(y.data_ptr()), x.numel(), bf16, cur_stream());
}

void decode16_sum(const Tensor& base, int64_t rank_stride, int64_t n_ranks, bool bf16, double scale,
                  const Tensor& out) {
  CHECK_F32(out);
  check_rows(base, rank_stride, n_ranks, 2 * out.numel());
  DevGuard guard(out.device());
  grace::decode16_sum(base.data_ptr<uint8_t>(), rank_stride, (int)n_ranks, out.numel(), bf16, (float)scale,
                      out.data_ptr<float>(), cur_stream());
}

// sums (int64, fixed point) / counts (int32) [n_seg * q] and arrive (int32 [n_seg]) are a persistent
// workspace that is zero on entry and left zero; seg_chunk_begin [n_seg + 1]; the last block of
// every segment writes its means
void sketch_encode(const Tensor& x, const Tensor& edges, int64_t q, const Tensor& bins, const Tensor& sums,
                   const Tensor& counts, const Tensor& seg, const Tensor& cb, const Tensor& ce, const Tensor& arrive,
                   const Tensor& seg_chunk_begin, const Tensor& means) {
  CHECK_F32(x);
  CHECK_F32(edges);
  CHECK_F32(means);
  CHECK_DEV(bins);
  TORCH_CHECK(q >= 1 && q <= 65535, "quantiles must be in [1, 65535]");
  TORCH_CHECK(q < 256 || bins.element_size() == 2, "q >= 256 needs 16-bit bin codes");
  TORCH_CHECK(bins.numel() >= x.numel(), "bins too small");
  TORCH_CHECK(sums.scalar_type() == at::kLong && counts.scalar_type() == at::kInt && arrive.scalar_type() == at::kInt &&
                  seg_chunk_begin.scalar_type() == at::kInt,
              "sketch_encode: int64 sums, int32 counts / arrive / seg_chunk_begin");
  const int64_t n_seg = seg_chunk_begin.numel() - 1;
  TORCH_CHECK(arrive.numel() >= n_seg && means.numel() >= n_seg * q && sums.numel() >= n_seg * q &&
                  counts.numel() >= n_seg * q && edges.numel() >= n_seg * (q + 1),
              "sketch_encode: tables too small");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  if (q > 1024) {  // global bin accumulators (csrc/kernels/cast_sketch.hip sketch_encode_big)
    grace::sketch_encode_big(ct, (int)n_seg, x.data_ptr<float>(), edges.data_ptr<float>(), (int)q, bins.data_ptr(),
                             (int)bins.element_size(), reinterpret_cast<unsigned long long*>(sums.data_ptr<int64_t>()),
                             reinterpret_cast<uint32_t*>(counts.data_ptr<int32_t>()), arrive.data_ptr<int32_t>(),
                             seg_chunk_begin.data_ptr<int32_t>(), means.data_ptr<float>(), cur_stream());
    return;
  }
  grace::sketch_encode(ct, x.data_ptr<float>(), edges.data_ptr<float>(), (int)q, bins.data_ptr(),
                       (int)bins.element_size(), reinterpret_cast<unsigned long long*>(sums.data_ptr<int64_t>()),
                       reinterpret_cast<uint32_t*>(counts.data_ptr<int32_t>()), arrive.data_ptr<int32_t>(),
                       seg_chunk_begin.data_ptr<int32_t>(), means.data_ptr<float>(), cur_stream());
}

void sketch_decode(const Tensor& base, int64_t rank_stride, int64_t bins_off, int64_t means_off, int64_t q,
                   int64_t bin_bytes, int64_t n_ranks, double scale, const Tensor& out, const Tensor& seg,
                   const Tensor& cb, const Tensor& ce, int64_t n_seg) {
  CHECK_F32(out);
  check_rows(base, rank_stride, n_ranks, std::max(bins_off + bin_bytes * out.numel(), means_off + 4 * q * n_seg));
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(out.device());
  grace::sketch_decode(ct, base.data_ptr<uint8_t>(), rank_stride, bins_off, means_off, (int)q, (int)bin_bytes,
                       (int)n_ranks, (float)scale, out.data_ptr<float>(), cur_stream());
}

// tables (all int32 / fp32, per segment): ranks/slot/st_* [n_seg][max_slots], nrank/nuniq [n_seg],
// lo_idx/hi_idx/w/edges [n_seg][q+1]; h0 [n_seg][2048] and h [n_seg][max_slots][128] zero on entry
// (and left zero on exit)
void quantile_select(const Tensor& x, const Tensor& seg, const Tensor& cb, const Tensor& ce, int64_t n_seg,
                     int64_t max_slots, const Tensor& ranks, const Tensor& nrank, const Tensor& h0, const Tensor& h,
                     const Tensor& st_pfx, const Tensor& st_rank, const Tensor& slot, const Tensor& uniq,
                     const Tensor& nuniq, int64_t q, const Tensor& lo_idx, const Tensor& hi_idx, const Tensor& w,
                     const Tensor& edges) {
  CHECK_F32(x);
  CHECK_F32(w);
  CHECK_F32(edges);
  for (const Tensor* t : {&ranks, &nrank, &h0, &h, &st_pfx, &st_rank, &slot, &uniq, &nuniq, &lo_idx, &hi_idx}) {
    CHECK_I32((*t));
  }
  TORCH_CHECK(max_slots >= 1 && max_slots <= 256, "max_slots must be in [1, 256] (one select thread per rank)");
  const int64_t ms = n_seg * max_slots;
  TORCH_CHECK(ranks.numel() >= ms && st_pfx.numel() >= ms && st_rank.numel() >= ms && slot.numel() >= ms &&
                  uniq.numel() >= ms, "per-rank tables too small");
  TORCH_CHECK(nrank.numel() >= n_seg && nuniq.numel() >= n_seg, "per-segment tables too small");
  TORCH_CHECK(h0.numel() >= n_seg * 2048 && h.numel() >= ms * 128, "histograms too small");
  const int64_t ne = n_seg * (q + 1);
  TORCH_CHECK(lo_idx.numel() >= ne && hi_idx.numel() >= ne && w.numel() >= ne && edges.numel() >= ne,
              "edge tables too small");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::quantile_select(ct, (int)n_seg, x.data_ptr<float>(), (int)max_slots, ranks.data_ptr<int32_t>(),
                         nrank.data_ptr<int32_t>(), h0.data_ptr<int32_t>(), h.data_ptr<int32_t>(),
                         reinterpret_cast<uint32_t*>(st_pfx.data_ptr<int32_t>()), st_rank.data_ptr<int32_t>(),
                         slot.data_ptr<int32_t>(), reinterpret_cast<uint32_t*>(uniq.data_ptr<int32_t>()),
                         nuniq.data_ptr<int32_t>(), (int)q, lo_idx.data_ptr<int32_t>(), hi_idx.data_ptr<int32_t>(),
                         w.data_ptr<float>(), edges.data_ptr<float>(), cur_stream());
}

// ------------------------------------------------------------------------------ fp32 MFMA GEMM
// Operands are raw row-strided views of the given tensors' storage (see gemm_f32.hip):
// kcontig: X(r, k) = x[r*ld + k] over r < rows, k < K; else X(r, k) = x[k*ld + r].
static void check_operand(const Tensor& x, bool kc, int64_t ld, int64_t rows, int64_t K, const char* what) {
  CHECK_DEV(x);
  CHECK_DT(x, at::kFloat);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && ld % 4 == 0, what, ": 16-B alignment");
  TORCH_CHECK(kc ? (K % 4 == 0) : (rows % 4 == 0), what, ": the contiguous extent must be a multiple of 4");
  const int64_t need = kc ? (rows - 1) * ld + K : (K - 1) * ld + rows;
  TORCH_CHECK(x.numel() >= need && ld >= (kc ? K : rows), what, ": view exceeds the tensor");
}

// BN-backward epilogue operands: x [M][N] fp32 dense (the BN input), mask [M*N/8] uint8 (None: no
// ReLU), save [>= 2N] fp32 (mean, invstd)
static bool bn_epi(const c10::optional<Tensor>& bx, const c10::optional<Tensor>& bmask,
                   const c10::optional<Tensor>& bsave, bool relu, int64_t M, int64_t N, grace::BnBwdEpi* e) {
  if (!(bx.has_value() && bx->defined())) return false;
  CHECK_DEV((*bx));
  CHECK_DT((*bx), at::kFloat);
  TORCH_CHECK(bx->numel() == M * N && (bx->is_contiguous() || bx->is_contiguous(at::MemoryFormat::ChannelsLast)) &&
                  reinterpret_cast<uintptr_t>(bx->data_ptr()) % 16 == 0 && N % 8 == 0,
              "bn epilogue: x must be a dense 16-B aligned [M][N] image, N % 8 == 0");
  TORCH_CHECK(bsave.has_value() && bsave->defined() && bsave->is_cuda() && bsave->scalar_type() == at::kFloat &&
                  bsave->numel() >= 4 * N && reinterpret_cast<uintptr_t>(bsave->data_ptr()) % 16 == 0,
              "bn epilogue: save [>= 4N] fp32 (mean, invstd, scale, shift)");
  e->x = bx->data_ptr<float>();
  e->save = bsave->data_ptr<float>();
  e->mask = nullptr;
  e->relu = relu ? 1 : 0;
  if (bmask.has_value() && bmask->defined()) {
    TORCH_CHECK(bmask->is_cuda() && bmask->scalar_type() == at::kByte && bmask->is_contiguous() &&
                    bmask->numel() == M * N / 8, "bn epilogue: mask [M*N/8] uint8");
    e->mask = bmask->data_ptr<uint8_t>();
  }
  return true;
}

// BN-apply prologue operand: save [>= 4C] fp32 (scale at 2C, shift at 3C) of the C-channel BN
static bool bn_pro(const c10::optional<Tensor>& xsave, int64_t C, bool relu, int op, grace::BnApplyPro* f) {
  if (!(xsave.has_value() && xsave->defined())) return false;
  TORCH_CHECK(xsave->is_cuda() && xsave->scalar_type() == at::kFloat && xsave->is_contiguous() &&
                  xsave->numel() >= 4 * C && reinterpret_cast<uintptr_t>(xsave->data_ptr()) % 16 == 0 && C % 4 == 0,
              "bn prologue: save [>= 4C] fp32, 16-B aligned, C % 4 == 0");
  f->save = xsave->data_ptr<float>();
  f->C = (int)C;
  f->relu = relu ? 1 : 0;
  f->op = op;
  return true;
}

int64_t gemm_f32(const Tensor& A, bool a_kc, int64_t lda, const Tensor& B, bool b_kc, int64_t ldb, const Tensor& C,
                 int64_t ldc, int64_t M, int64_t N, int64_t K, int64_t splits, int64_t tile,
                 const c10::optional<Tensor>& stats, const c10::optional<Tensor>& bn_x,
                 const c10::optional<Tensor>& bn_mask, const c10::optional<Tensor>& bn_save, bool bn_relu,
                 const c10::optional<Tensor>& x_save, bool x_relu, int64_t x_op) {
  check_operand(A, a_kc, lda, M, K, "A");
  check_operand(B, b_kc, ldb, N, K, "B");
  CHECK_DEV(C);
  CHECK_DT(C, at::kFloat);
  TORCH_CHECK(C.numel() >= (M - 1) * ldc + N && ldc >= N, "C too small");
  TORCH_CHECK(splits == 0 || splits == 1 || ldc == N, "split-K needs a dense C");
  TORCH_CHECK(tile >= 0 && tile <= 4, "gemm_f32: tile 0 (launcher rule) or 1-4");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "GEMM dims must fit int32");
  float* st = nullptr;
  if (stats.has_value() && stats->defined()) {
    CHECK_DEV((*stats));
    CHECK_DT((*stats), at::kFloat);
    TORCH_CHECK(splits == 1, "GEMM statistics need whole-K tiles (splits = 1)");
    TORCH_CHECK(stats->is_contiguous() && stats->numel() >= ((M + 63) / 64) * 2 * N, "stats: [ceil(M/64)][2][N]");
    st = stats->data_ptr<float>();
  }
  grace::BnBwdEpi epi{};
  const bool has_epi = bn_epi(bn_x, bn_mask, bn_save, bn_relu, M, N, &epi);
  TORCH_CHECK(!has_epi || (st != nullptr && ldc == N), "bn epilogue: needs stats and a dense C");
  grace::BnApplyPro pro{};
  TORCH_CHECK(x_op == 1 || x_op == 2, "bn prologue: x_op 1 (A) or 2 (B)");
  // the transformed operand's channels: A's k (K-contig A) or B's rows (MN-contig B)
  TORCH_CHECK(!(x_save.has_value() && x_save->defined()) || (x_op == 1 ? a_kc : !b_kc),
              "bn prologue: the operand's channels must be its contiguous extent (K-contig A / MN-contig B)");
  const bool has_pro = bn_pro(x_save, x_op == 1 ? K : N, x_relu, (int)x_op, &pro);
  DevGuard guard(C.device());
  return grace::gemm_f32(A.data_ptr<float>(), a_kc, lda, B.data_ptr<float>(), b_kc, ldb, C.data_ptr<float>(), ldc,
                         (int)M, (int)N, (int)K, (int)splits, cur_stream(), (int)tile, st, has_epi ? &epi : nullptr,
                         has_pro ? &pro : nullptr);
}

// 3x3 / pad 1 implicit-GEMM convolution (gemm_f32.hip).  Activations and the weight are NCHW-shaped
// tensors in channels_last memory (NHWC / [Cout][3][3][Cin] images).
static void check_cl(const Tensor& t, std::initializer_list<int64_t> shape, const char* what) {
  CHECK_DEV(t);
  CHECK_DT(t, at::kFloat);
  TORCH_CHECK(t.dim() == 4 && t.sizes() == c10::IntArrayRef(shape), what, ": shape ", t.sizes(), " expected ",
              c10::IntArrayRef(shape));
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), what, ": channels_last memory required");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, what, ": 16-B alignment");
}

int64_t conv3x3_f32(int64_t dir, const Tensor& act, const Tensor& other, const Tensor& C, int64_t stride,
                    int64_t splits, int64_t tile, const c10::optional<Tensor>& stats, int64_t ksize,
                    const c10::optional<Tensor>& bn_x, const c10::optional<Tensor>& bn_mask,
                    const c10::optional<Tensor>& bn_save, bool bn_relu, const c10::optional<Tensor>& x_save,
                    bool x_relu) {
  TORCH_CHECK(dir >= 0 && dir <= 2, "conv3x3_f32: dir 0 (fwd) / 1 (dgrad) / 2 (wgrad)");
  TORCH_CHECK(tile >= 0 && tile <= 4, "conv3x3_f32: tile 0 (launcher rule) or 1-4");
  TORCH_CHECK(stride == 1 || (stride == 2 && dir != 1), "conv3x3_f32: stride 1, or 2 for fwd / wgrad");
  TORCH_CHECK(ksize == 3 || (ksize == 1 && dir != 1), "conv3x3_f32: 3x3 (pad 1), or 1x1 (pad 0) fwd / wgrad");
  const int64_t K = ksize;
  int64_t N, H, W, Cin, Cout;
  if (dir == 1) {  // act = dY [N, Cout, H, W], other = weight, C = dX [N, Cin, H, W]
    N = act.size(0), Cout = act.size(1), H = act.size(2), W = act.size(3), Cin = C.size(1);
    check_cl(act, {N, Cout, H, W}, "dY");
    check_cl(other, {Cout, Cin, K, K}, "weight");
    check_cl(C, {N, Cin, H, W}, "dX");
    TORCH_CHECK(Cout % 32 == 0 && Cin % 4 == 0, "conv3x3_f32 dgrad: Cout % 32, Cin % 4");
  } else {
    N = act.size(0), Cin = act.size(1), H = act.size(2), W = act.size(3);
    const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
    if (dir == 0) {  // other = weight, C = y
      Cout = other.size(0);
      check_cl(other, {Cout, Cin, K, K}, "weight");
      check_cl(C, {N, Cout, Ho, Wo}, "y");
      TORCH_CHECK(Cin % 32 == 0 && Cout % 4 == 0, "conv3x3_f32 fwd: Cin % 32, Cout % 4");
    } else {  // other = dY, C = dW
      Cout = other.size(1);
      check_cl(other, {N, Cout, Ho, Wo}, "dY");
      check_cl(C, {Cout, Cin, K, K}, "dW");
      TORCH_CHECK(Cin % 4 == 0 && Cout % 4 == 0, "conv3x3_f32 wgrad: Cin % 4, Cout % 4");
    }
    check_cl(act, {N, Cin, H, W}, "x");
  }
  TORCH_CHECK(N * H * W < (1 << 24), "conv3x3_f32: N*H*W < 2^24 (float pixel division)");
  TORCH_CHECK(act.numel() < (int64_t(1) << 31) && other.numel() < (int64_t(1) << 31) && C.numel() < (int64_t(1) << 31),
              "conv3x3_f32: operands of < 2^31 elements (32-bit gather indices)");
  float* st = nullptr;
  grace::BnBwdEpi epi{};
  const bool has_epi = dir == 1 && bn_epi(bn_x, bn_mask, bn_save, bn_relu, N * H * W, Cin, &epi);
  grace::BnApplyPro pro{};
  TORCH_CHECK(!(x_save.has_value() && x_save->defined()) || dir != 1, "bn prologue: forward / weight grad only");
  const bool has_pro = dir != 1 && bn_pro(x_save, Cin, x_relu, 0, &pro);
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK((dir == 0 || has_epi) && splits == 1,
                "conv3x3_f32: statistics on the forward / the data grad's BN epilogue, splits = 1");
    CHECK_DEV((*stats));
    CHECK_DT((*stats), at::kFloat);
    const int64_t M = dir == 1 ? N * H * W : N * ((H - 1) / stride + 1) * ((W - 1) / stride + 1);
    const int64_t NC = dir == 1 ? Cin : Cout;
    TORCH_CHECK(stats->is_contiguous() && stats->numel() >= ((M + 63) / 64) * 2 * NC, "stats: [ceil(M/64)][2][N]");
    st = stats->data_ptr<float>();
  }
  TORCH_CHECK(!has_epi || st != nullptr, "bn epilogue: needs stats");
  DevGuard guard(C.device());
  return grace::conv3x3_f32((int)dir, act.data_ptr<float>(), other.data_ptr<float>(), C.data_ptr<float>(), (int)N,
                            (int)H, (int)W, (int)Cin, (int)Cout, (int)stride, (int)splits, (int)tile, st, cur_stream(), (int)ksize,
                            has_epi ? &epi : nullptr, has_pro ? &pro : nullptr);
}

// ------------------------------------------------------------------------------ segment stats
void segment_stats(const Tensor& x, const c10::optional<Tensor>& r, int64_t mode, double beta, double gamma,
                   const c10::optional<Tensor>& xout, const Tensor& seg, const Tensor& cb, const Tensor& ce,
                   const Tensor& seg_chunk_begin, const Tensor& partials, const Tensor& stats) {
  CHECK_F32(x);
  const float* rp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(r.has_value(), "mode 1 needs r");
    CHECK_F32((*r));
    TORCH_CHECK(r->numel() == x.numel(), "r size");
    rp = r->data_ptr<float>();
  }
  float* xp = nullptr;
  if (xout.has_value()) {
    CHECK_F32((*xout));
    TORCH_CHECK(xout->numel() == x.numel(), "xout size");
    xp = xout->data_ptr<float>();
  }
  CHECK_I32(seg_chunk_begin);
  CHECK_DEV(partials);
  CHECK_DT(partials, at::kDouble);
  CHECK_F32(stats);
  const int n_seg = (int)seg_chunk_begin.numel() - 1;
  TORCH_CHECK(stats.numel() >= (int64_t)n_seg * grace::kSegStats, "stats too small");
  TORCH_CHECK(partials.numel() >= seg.numel() * grace::kSegStats, "partials too small");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::segment_stats(ct, n_seg, seg_chunk_begin.data_ptr<int32_t>(), x.data_ptr<float>(), rp, (int)mode,
                       (float)beta, (float)gamma, xp, partials.data_ptr<double>(), stats.data_ptr<float>(),
                       cur_stream());
}

// ------------------------------------------------------------------------------ elementwise
void axpby(const Tensor& x, const Tensor& y, const Tensor& out, double a, double b) {
  CHECK_F32(x);
  CHECK_F32(y);
  CHECK_F32(out);
  TORCH_CHECK(x.numel() == y.numel() && y.numel() == out.numel(), "size mismatch");
  DevGuard guard(out.device());
  grace::axpby(x.data_ptr<float>(), y.data_ptr<float>(), out.data_ptr<float>(), x.numel(), (float)a,
               (float)b, cur_stream());
}

// Copy the memory image of srcs[i] (dense fp32 or bf16 GPU tensors, one dtype per call) to
// dst[dst_off[i] : dst_off[i] + numel] (fp32, bf16 widened).
void gather_segments(const std::vector<Tensor>& srcs, const std::vector<int64_t>& dst_off, const Tensor& dst) {
  CHECK_F32(dst);
  TORCH_CHECK(dst_off.size() == srcs.size(), "one destination offset per source");
  if (srcs.empty()) return;
  const auto dt = srcs[0].scalar_type();
  TORCH_CHECK(dt == at::kFloat || dt == at::kBFloat16, "gather sources must be fp32 or bf16");
  std::vector<const void*> ptrs(srcs.size());
  std::vector<int64_t> len(srcs.size());
  for (size_t i = 0; i < srcs.size(); ++i) {
    const Tensor& t = srcs[i];
    CHECK_DEV(t);
    TORCH_CHECK(t.scalar_type() == dt, "gather sources must share one dtype");
    TORCH_CHECK(t.is_non_overlapping_and_dense(), "gather source must be dense");
    TORCH_CHECK(t.device() == dst.device(), "device mismatch");
    TORCH_CHECK(dst_off[i] >= 0 && dst_off[i] + t.numel() <= dst.numel(), "segment ", i, " exceeds the destination");
    ptrs[i] = t.data_ptr();
    len[i] = t.numel();
  }
  DevGuard guard(dst.device());
  grace::gather_segments(ptrs.data(), dt == at::kBFloat16, dst_off.data(), len.data(), (int)srcs.size(),
                         dst.data_ptr<float>(), cur_stream());
}

// dsts[i] (contiguous) <- srcs[i] (any strides, same shape, <= 4 dims), fp32, one launch per 40 tensors.

// dsts[i] <- bf16(srcs[i]) (round to nearest even), memory images, one launch per 120 tensors.
void cast_segments_bf16(const std::vector<Tensor>& srcs, const std::vector<Tensor>& dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "srcs/dsts length");
  if (srcs.empty()) return;
  std::vector<const float*> sp(srcs.size());
  std::vector<uint16_t*> dp(srcs.size());
  std::vector<int64_t> len(srcs.size());
  for (size_t i = 0; i < srcs.size(); ++i) {
    CHECK_DEV(srcs[i]);
    CHECK_DT(srcs[i], at::kFloat);  // channels_last masters are dense, not contiguous
    CHECK_DEV(dsts[i]);
    CHECK_DT(dsts[i], at::kBFloat16);
    TORCH_CHECK(srcs[i].numel() == dsts[i].numel() && srcs[i].strides() == dsts[i].strides(), "shape/stride mismatch");
    TORCH_CHECK(srcs[i].is_non_overlapping_and_dense(), "cast source must be dense");
    sp[i] = srcs[i].data_ptr<float>();
    dp[i] = reinterpret_cast<uint16_t*>(dsts[i].data_ptr());
    len[i] = srcs[i].numel();
  }
  DevGuard guard(srcs[0].device());
  grace::cast_segments_bf16(sp.data(), dp.data(), len.data(), (int)srcs.size(), cur_stream());
}

void scale_(const Tensor& x, double s) {
  CHECK_F32(x);
  DevGuard guard(x.device());
  grace::scale_inplace(x.data_ptr<float>(), x.numel(), (float)s, cur_stream());
}

std::string build_info() {
  return std::string("grace_amd native: HIP ") + std::to_string(HIP_VERSION_MAJOR) + "." +
         std::to_string(HIP_VERSION_MINOR) + " gfx950";
}

}  // namespace

void grace_bind_comm(py::module& m);  // csrc/comm/rccl_comm.cpp
void grace_bind_nn(py::module& m);    // csrc/nn_bindings.cpp
void grace_bind_xgmi(py::module& m);  // csrc/comm/xgmi_allgather.hip
void grace_bind_health(py::module& m);  // csrc/comm/health.cpp
void grace_bind_runtime(py::module& m);  // csrc/runtime/graph_split.cpp

// ------------------------------------------------------------------------------ Adaq
void adaq_sample(const Tensor& x, const Tensor& seg_off, const Tensor& samp_off, int64_t seed,
                 const c10::optional<Tensor>& step, const Tensor& samples) {
  CHECK_F32(x);
  CHECK_I64(seg_off);
  CHECK_I64(samp_off);
  CHECK_F32(samples);
  TORCH_CHECK(seg_off.numel() == samp_off.numel(), "offset tables");
  DevGuard guard(x.device());
  const int n_seg = (int)seg_off.numel() - 1;
  grace::adaq_sample(x.data_ptr<float>(), n_seg, seg_off.data_ptr<int64_t>(), samp_off.data_ptr<int64_t>(),
                     samples.numel() / 2, seed_arg(seed, step), samples.data_ptr<float>(), cur_stream());
}

void adaq_prepare(const Tensor& x, const Tensor& seg_off, const Tensor& samp_off, const Tensor& stats, double ratio,
                  const Tensor& count, const Tensor& target, const Tensor& kseg, const Tensor& fallback,
                  const Tensor& thr, const Tensor& done, const Tensor& seg, const Tensor& cb, const Tensor& ce) {
  CHECK_F32(x);
  CHECK_F32(stats);
  CHECK_I32(count);
  CHECK_F32(target);
  CHECK_I32(kseg);
  CHECK_F32(fallback);
  CHECK_F32(thr);
  CHECK_I32(done);
  const int n_seg = (int)seg_off.numel() - 1;
  TORCH_CHECK(count.numel() == 2 * n_seg && kseg.numel() == 2 * n_seg && thr.numel() == 2 * n_seg, "group arrays");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::adaq_prepare(ct, n_seg, x.data_ptr<float>(), seg_off.data_ptr<int64_t>(), samp_off.data_ptr<int64_t>(),
                      stats.data_ptr<float>(), (float)ratio, count.data_ptr<int32_t>(), target.data_ptr<float>(),
                      kseg.data_ptr<int32_t>(), fallback.data_ptr<float>(), thr.data_ptr<float>(),
                      done.data_ptr<int32_t>(), cur_stream());
}

void adaq_refine(const Tensor& x, const Tensor& state, const Tensor& fallback, const Tensor& target, int64_t max_iters,
                 const Tensor& thr, const Tensor& count, const Tensor& done, const Tensor& seg, const Tensor& cb,
                 const Tensor& ce) {
  CHECK_F32(x);
  CHECK_I32(state);
  const int n_seg = (int)(thr.numel() / 2);
  TORCH_CHECK(state.numel() >= 2 * 2 * n_seg, "state");
  auto ct = make_ct(seg, cb, ce);
  DevGuard guard(x.device());
  grace::adaq_refine(ct, n_seg, x.data_ptr<float>(), reinterpret_cast<const grace::TopkState*>(state.data_ptr<int32_t>()),
                     fallback.data_ptr<float>(), target.data_ptr<float>(), (int)max_iters, thr.data_ptr<float>(),
                     count.data_ptr<int32_t>(), done.data_ptr<int32_t>(), cur_stream());
}

void adaq_offsets(const Tensor& count, const Tensor& goff, const Tensor& cursor) {
  CHECK_I32(count);
  CHECK_I32(goff);
  CHECK_I32(cursor);
  TORCH_CHECK(goff.numel() == count.numel() + 1 && cursor.numel() == count.numel(), "offset arrays");
  DevGuard guard(count.device());
  grace::adaq_offsets((int)(count.numel() / 2), count.data_ptr<int32_t>(), goff.data_ptr<int32_t>(),
                      cursor.data_ptr<int32_t>(), cur_stream());
}

void adaq_compact(const Tensor& x, const Tensor& thr, const Tensor& goff, const Tensor& cursor, const Tensor& idx,
                  const Tensor& psum, const Tensor& means, const Tensor& counts, const Tensor& seg, const Tensor& cb,
                  const Tensor& ce, const Tensor& seg_chunk_begin) {
  CHECK_F32(x);
  CHECK_F32(thr);
  CHECK_I32(idx);
  CHECK_DT(psum, at::kDouble);
  CHECK_F32(means);
  CHECK_I32(counts);
  CHECK_I32(seg_chunk_begin);
  const int n_seg = (int)(thr.numel() / 2);
  auto ct = make_ct(seg, cb, ce);
  TORCH_CHECK(psum.numel() >= 2 * (int64_t)ct.n_chunks, "psum");
  TORCH_CHECK(means.numel() == 2 * n_seg && counts.numel() == 2 * n_seg, "means/counts");
  DevGuard guard(x.device());
  grace::adaq_compact(ct, n_seg, seg_chunk_begin.data_ptr<int32_t>(), x.data_ptr<float>(), thr.data_ptr<float>(),
                      goff.data_ptr<int32_t>(), cursor.data_ptr<int32_t>(), idx.data_ptr<int32_t>(), idx.numel(),
                      psum.data_ptr<double>(), means.data_ptr<float>(), counts.data_ptr<int32_t>(), cur_stream());
}

// one rank's capacity payload (means, counts, idx[cap]) -> out
void adaq_decode(const Tensor& means, const Tensor& counts, const Tensor& idx, const Tensor& goff_ws,
                 const Tensor& out, double scale) {
  CHECK_F32(means);
  CHECK_I32(counts);
  CHECK_I32(idx);
  CHECK_I32(goff_ws);
  CHECK_F32(out);
  const int ng = (int)counts.numel();
  TORCH_CHECK(means.numel() == ng && goff_ws.numel() >= ng + 1, "means / counts / workspace");
  DevGuard guard(out.device());
  grace::adaq_decode(ng, means.data_ptr<float>(), counts.data_ptr<int32_t>(), idx.data_ptr<int32_t>(), idx.numel(),
                     goff_ws.data_ptr<int32_t>(), out.data_ptr<float>(), (float)scale, cur_stream());
}

// ------------------------------------------------------------------------------ INCEPTIONN
int64_t inceptionn_tiles(int64_t n) { return grace::inceptionn_tiles(n); }

void inceptionn_count(const Tensor& x, int64_t e_b, int64_t mid, const Tensor& cnt, const Tensor& totals) {
  CHECK_F32(x);
  CHECK_I32(cnt);
  CHECK_I32(totals);
  TORCH_CHECK(cnt.numel() >= 4 * grace::inceptionn_tiles(x.numel()) && totals.numel() >= 4, "workspace");
  DevGuard guard(x.device());
  grace::inceptionn_count(x.data_ptr<float>(), x.numel(), (int)e_b, (int)mid, cnt.data_ptr<int32_t>(),
                          totals.data_ptr<int32_t>(), cur_stream());
}

void inceptionn_encode(const Tensor& x, int64_t e_b, int64_t mid, const Tensor& off, const Tensor& totals,
                       const Tensor& stream, const Tensor& codes) {
  CHECK_F32(x);
  CHECK_I32(off);
  CHECK_I32(totals);
  CHECK_DT(stream, at::kByte);
  CHECK_DT(codes, at::kByte);
  TORCH_CHECK(codes.numel() >= (x.numel() + 3) / 4 && totals.numel() >= 4, "codes / totals size");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(stream.data_ptr()) & 3) == 0, "stream must be 4-byte aligned");
  DevGuard guard(x.device());
  grace::inceptionn_encode(x.data_ptr<float>(), x.numel(), (int)e_b, (int)mid, off.data_ptr<int32_t>(),
                           totals.data_ptr<int32_t>(), stream.data_ptr<uint8_t>(), stream.numel(),
                           codes.data_ptr<uint8_t>(), cur_stream());
}

// base: uint8 view of the rank rows (compressor._base.rank_rows)
void inceptionn_decode(const Tensor& base, int64_t rank_stride, int64_t stream_off, int64_t codes_off,
                       int64_t n_ranks, const Tensor& cnt, const Tensor& totals, double scale, const Tensor& out,
                       bool accumulate) {
  CHECK_DEV(base);
  CHECK_DT(base, at::kByte);
  CHECK_I32(cnt);
  CHECK_I32(totals);
  CHECK_F32(out);
  const int64_t n = out.numel();
  TORCH_CHECK(cnt.numel() >= 4 * n_ranks * grace::inceptionn_tiles(n) && totals.numel() >= 4 * n_ranks, "workspace");
  TORCH_CHECK(base.numel() >= (n_ranks - 1) * rank_stride + codes_off + (n + 3) / 4, "rank rows too small");
  DevGuard guard(out.device());
  grace::inceptionn_decode(base.data_ptr<uint8_t>(), rank_stride, stream_off, codes_off, (int)n_ranks, n,
                           cnt.data_ptr<int32_t>(), totals.data_ptr<int32_t>(), (float)scale, out.data_ptr<float>(),
                           accumulate, cur_stream());
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  grace_bind_runtime(m);
  grace_bind_comm(m);
  grace_bind_nn(m);
  grace_bind_xgmi(m);
  grace_bind_health(m);
  m.doc() = "grace_amd native CDNA4 kernels and RCCL runtime";
  m.def("build_info", &build_info);
  m.def("topk_select", &topk_select);
  m.def("topk_compact", &topk_compact);
  m.def("topk_ef", &topk_ef);
  m.def("sparse_scatter_add", &sparse_scatter_add);
  m.def("sparse_scatter_add_dev", &sparse_scatter_add_dev, py::arg("val"), py::arg("idx"), py::arg("count"),
        py::arg("out"), py::arg("scale"), py::arg("accumulate"), py::arg("count_overflow") = false);
  m.def("segment_stats", &segment_stats);
  m.def("randk_gather", &randk_gather);
  m.def("randk_scatter", &randk_scatter);
  m.def("threshold_compact", &threshold_compact);
  m.def("sign_pack", &sign_pack);
  m.def("sign_unpack", &sign_unpack);
  m.def("qsgd_quantize", &qsgd_quantize);
  m.def("qsgd_aggregate", &qsgd_aggregate);
  m.def("qsgd_pack", &qsgd_pack);
  m.attr("QSGD_PACKED2") = grace::kPacked2;
  m.attr("QSGD_PACKED4") = grace::kPacked4;
  m.def("tern_quantize", &tern_quantize);
  m.def("tern_aggregate", &tern_aggregate);
  m.def("natural_encode", &natural_encode);
  m.def("natural_aggregate", &natural_aggregate);
  m.def("u8_encode", &u8_encode);
  m.def("u8_aggregate", &u8_aggregate);
  m.def("dgc_sample", &dgc_sample, py::arg("x"), py::arg("seg_off"), py::arg("samp_off"), py::arg("seed"),
        py::arg("step"), py::arg("samples"), py::arg("u") = py::none(), py::arg("v") = py::none(),
        py::arg("momentum") = 0.0, py::arg("first") = false);
  m.def("dgc_refine", &dgc_refine, py::arg("x"), py::arg("state"), py::arg("target"), py::arg("max_iters"),
        py::arg("thr"), py::arg("count"), py::arg("done"), py::arg("seg"), py::arg("cb"), py::arg("ce"),
        py::arg("ccnt"), py::arg("fnode"), py::arg("u") = py::none(), py::arg("v") = py::none(),
        py::arg("momentum") = 0.0, py::arg("first") = false, py::arg("init") = true);
  m.def("dgc_select_init", &dgc_select_init, py::arg("samples"), py::arg("samp_off"), py::arg("kseg"),
        py::arg("state"), py::arg("thr"), py::arg("count"), py::arg("done"), py::arg("fnode"));
  m.def("dgc_compact", &dgc_compact, py::arg("x"), py::arg("thr"), py::arg("out_val"), py::arg("out_idx"),
        py::arg("counter"), py::arg("seg"), py::arg("cb"), py::arg("ce"), py::arg("ccnt"), py::arg("fnode"),
        py::arg("coff"), py::arg("vmask") = py::none(), py::arg("umask") = py::none());
  m.def("dgc_compensate", &dgc_compensate);
  m.def("powersgd_mq", &powersgd_mq, py::arg("x"), py::arg("small"), py::arg("out"), py::arg("mats"), py::arg("tiles"),
        py::arg("mode"), py::arg("comp_r"), py::arg("beta"), py::arg("gamma"), py::arg("xout"), py::arg("max_r"),
        py::arg("lazy_p") = py::none(), py::arg("lazy_q") = py::none(), py::arg("lazy_scale") = 0.0,
        py::arg("zeroed") = false, py::arg("bump") = py::none(), py::arg("vec") = py::none(),
        py::arg("vec_idx") = py::none());
  m.def("gram_orthonormalize", &gram_orthonormalize, py::arg("buf"), py::arg("mats"), py::arg("which"),
        py::arg("n_mat"), py::arg("gtiles"), py::arg("gtile_begin"), py::arg("passes"), py::arg("max_r"),
        py::arg("zero") = py::none());
  m.def("adaq_sample", &adaq_sample);
  m.def("adaq_prepare", &adaq_prepare);
  m.def("adaq_refine", &adaq_refine);
  m.def("adaq_offsets", &adaq_offsets);
  m.def("adaq_compact", &adaq_compact);
  m.def("adaq_decode", &adaq_decode);
  m.def("inceptionn_tiles", &inceptionn_tiles);
  m.def("inceptionn_count", &inceptionn_count);
  m.def("inceptionn_encode", &inceptionn_encode);
  m.def("inceptionn_decode", &inceptionn_decode);
  m.def("powersgd_pqt", &powersgd_pqt, py::arg("P"), py::arg("Q"), py::arg("out"), py::arg("mats"), py::arg("tiles"),
        py::arg("resid"), py::arg("max_r"), py::arg("scale") = 1.0, py::arg("save_p") = py::none(),
        py::arg("save_q") = py::none(), py::arg("vec") = py::none(), py::arg("vec_idx") = py::none(),
        py::arg("vec_scale") = 1.0, py::arg("T") = py::none());
  m.def("powersgd_mtp_gram", &powersgd_mtp_gram);
  m.def("philox_normal", &philox_normal, py::arg("out"), py::arg("seed"), py::arg("step") = py::none(),
        py::arg("zero") = py::none());
  m.def("cast16", &cast16);
  m.def("decode16_sum", &decode16_sum);
  m.def("sketch_encode", &sketch_encode);
  m.def("sketch_decode", &sketch_decode);
  m.def("quantile_select", &quantile_select);
  m.def("conv3x3_f32", &conv3x3_f32, py::arg("dir"), py::arg("act"), py::arg("other"), py::arg("C"),
        py::arg("stride") = 1, py::arg("splits") = 0, py::arg("tile") = 0, py::arg("stats") = py::none(),
        py::arg("ksize") = 3, py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(),
        py::arg("bn_save") = py::none(), py::arg("bn_relu") = false, py::arg("x_save") = py::none(),
        py::arg("x_relu") = false);
  m.def("gemm_f32", &gemm_f32, py::arg("A"), py::arg("a_kc"), py::arg("lda"), py::arg("B"), py::arg("b_kc"),
        py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("splits"),
        py::arg("tile") = 0, py::arg("stats") = py::none(), py::arg("bn_x") = py::none(),
        py::arg("bn_mask") = py::none(), py::arg("bn_save") = py::none(), py::arg("bn_relu") = false,
        py::arg("x_save") = py::none(), py::arg("x_relu") = false, py::arg("x_op") = 1);
  m.def("axpby", &axpby);
  m.def("scale_", &scale_);
  m.def("gather_segments", &gather_segments);
  m.def("cast_segments_bf16", &cast_segments_bf16);
}
