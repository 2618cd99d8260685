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
void sparse_scatter_add(const float* val, const int32_t* idx, int64_t K, float* out, float scale,
                        bool accumulate, hipStream_t stream);

// ---------------------------------------------------------------- ef.hip (elementwise)
void axpby(const float* x, const float* y, float* out, int64_t n, float a, float b, hipStream_t stream);
void scale_inplace(float* x, int64_t n, float s, hipStream_t stream);

}  // namespace grace
