// One-launch, rank-ordered decode of W sparse payloads into a dense bucket (Top-K / Threshold /
// DGC decompress + aggregate).
//
//   out[t] = ((0 + s*v_0(t)) + s*v_1(t)) + ... + s*v_{W-1}(t)     (terms of ranks that sent t)
//
// The reference decodes each rank's payload into its own dense tensor and sums the W tensors
// (grace_dl/dist/communicator/allgather.py:40-45 + compressor/topk.py:30-36): W dense zero-fills
// and W dense adds.  The per-rank scatter loop it became here still cost a zero-fill launch plus W
// scatter launches on the critical tail of every step.  This kernel does all of it in ONE
// persistent grid:
//   phase 0        zero out[0, n) (16-B stores)
//   phase 1 + r    out[idx_r[j]] += s * val_r[j]   for j < K_r  (indices unique within a payload)
// separated by grid barriers, so every rank's adds land in the same order on every rank: the
// result is bit-identical to the sequential loop (and across ranks, which all gather the same
// payloads).  K_r is either fixed or read from the payload's in-band header (capacity payloads,
// counted into the health words when a payload overflowed).
//
// Barrier: an arrival counter (agent scope) per phase; agent-scope release / acquire fences in
// every wave carry the phase's stores across the 8 XCDs' L2s.  The grid is sized to be co-resident (<= 1 workgroup
// per CU), and every spin is bounded: a barrier that does not complete raises the health fault
// and the workgroup proceeds (the step's optimizer update is then skipped), so no wave can hang.
// The last workgroup to leave resets the counters: the kernel is replayable from a HIP graph.
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kDB = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct DecodeArgs {
  const float* val[kDecodeMaxRanks];
  const int32_t* idx[kDecodeMaxRanks];
  const int32_t* count[kDecodeMaxRanks];  // null: K = cap[r]
  int64_t cap[kDecodeMaxRanks];
};

__device__ __forceinline__ void grid_barrier(int32_t* ctr, int32_t target, uint32_t* health_host, uint32_t* health_dev) {
  // EVERY wave releases at agent scope: a release only waits for the issuing wave's own stores
  // (vmcnt) before the L2 write-back, and the workgroup barrier alone does not drain the other
  // waves' stores to L2 -- with one releasing thread, another wave's phase stores could still be
  // in flight and miss the write-back, and another XCD would read stale lines.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (int64_t(1) << 24)) {  // ~seconds: a workgroup never arrived
        if (health_host != nullptr)
          __hip_atomic_store(health_host + kHealthFault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (health_dev != nullptr)
          __hip_atomic_store(health_dev + kHealthFault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every wave: no stale L1 / L2 line of the phase
}

__global__ __launch_bounds__(kDB) void sparse_decode_kernel(DecodeArgs a, int W, float* __restrict__ out, int64_t n,
                                                           float scale, int32_t* ctr, uint32_t* health_host,
                                                           uint32_t* health_dev, int own) {
  const int G = gridDim.x;
  const int64_t tid = (int64_t)blockIdx.x * kDB + threadIdx.x, stride = (int64_t)G * kDB;
  // phase 0: zero (head to the first 16-B boundary, float4 body, tail).  Every store of `out`
  // is write-through and drops its line from this XCD's L2 (sc1), and the rank phases add with
  // device-coherent atomics (performed past the L2s): the per-XCD L2s are not coherent with each
  // other, and an agent-scope acquire does not evict them, so a line one XCD kept from an
  // earlier phase would otherwise be read stale after another XCD changed it.
  const int64_t head = std::min<int64_t>(n, (int64_t)((16 - (reinterpret_cast<uintptr_t>(out) & 15)) & 15) / 4);
  if (tid < head) __hip_atomic_store(out + tid, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t nv = (n - head) / 4;
  {
    float* body = out + head;
    const int64_t bytes = nv * 16;
    for (int64_t v0 = 0; v0 < nv; v0 += (int64_t(1) << 26)) {  // buffer descriptors address < 2 GB
      const int64_t cnt = std::min<int64_t>(nv - v0, int64_t(1) << 26);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(body + 4 * v0, 0, (int)std::min<int64_t>(bytes - 16 * v0, 0x7fffffff),
                                            0x00020000);
      for (int64_t v = tid; v < cnt; v += stride)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0u, 0u}, rs, (int)(v * 16), 0, 16 /* sc1 */);
    }
  }
  for (int64_t i = head + 4 * nv + tid; i < n; i += stride)
    __hip_atomic_store(out + i, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // phases 1..W: rank r's entries, in rank order
  for (int r = 0; r < W; ++r) {
    grid_barrier(ctr, (r + 1) * G, health_host, health_dev);
    int64_t K = a.cap[r];
    if (a.count[r] != nullptr) {
      const int64_t c = a.count[r][0];
      // counted once per process: for its OWN payload (every rank decodes every payload)
      if (r == own && c > K && blockIdx.x == 0 && threadIdx.x == 0) health_count_overflow(health_host);
      K = c < K ? c : K;
    }
    const float* __restrict__ val = a.val[r];
    const int32_t* __restrict__ idx = a.idx[r];
    // indices are unique within a payload, so no two adds of a phase meet: the device-coherent
    // atomic add is just a coherent read-modify-write, in rank order across the phases;
    // out + round(val * scale), as torch's index_add_(v * scale)
    for (int64_t j = tid; j < K; j += stride) {
      const int32_t t = idx[j];
      if (t >= 0 && t < n)
        __hip_atomic_fetch_add(out + t, __fmul_rn(val[j], scale), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // leave: the last workgroup out resets both counters for the next launch / graph replay
  __syncthreads();
  if (threadIdx.x == 0) {
    const int32_t old = __hip_atomic_fetch_add(ctr + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == G - 1) {
      __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int decode_grid(int64_t n, int64_t kmax) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    GRACE_HIP_CHECK(hipGetDevice(&dev));
    GRACE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  // one workgroup per CU at most (co-resident even beside a concurrent kernel: the barrier never
  // waits on a workgroup that cannot be scheduled); fewer for small buckets
  const int64_t need = std::max<int64_t>((n / 4 + kDB * 8 - 1) / (kDB * 8), (kmax + kDB * 4 - 1) / (kDB * 4));
  return (int)std::max<int64_t>(1, std::min<int64_t>(cus, need));
}

}  // namespace

void sparse_decode_ranks(int W, const float* const* val, const int32_t* const* idx, const int32_t* const* count,
                         const int64_t* cap, float* out, int64_t n, float scale, int32_t* ctr,
                         uint32_t* health_dev, hipStream_t stream, int own) {
  DecodeArgs a{};
  int64_t kmax = 0;
  for (int r = 0; r < W; ++r) {
    a.val[r] = val[r];
    a.idx[r] = idx[r];
    a.count[r] = count[r];
    a.cap[r] = cap[r];
    kmax = std::max<int64_t>(kmax, cap[r]);
  }
  const int G = decode_grid(n, kmax);
  sparse_decode_kernel<<<G, kDB, 0, stream>>>(a, W, out, n, scale, ctr, health_words().host_dev, health_dev, own);
}

}  // namespace grace
