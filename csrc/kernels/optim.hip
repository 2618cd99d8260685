// Fused multi-tensor SGD (torch.optim.SGD semantics) with optional bf16 working-copy refresh.
//
// One launch updates up to kSgdSegs parameters (pointer table in the kernel arguments, so a
// captured HIP graph replays it with no host work).  Work is a flat list of 4096-element tiles:
// tensor i owns blocks [start[i], start[i+1]) and a block finds its tensor by binary search, so
// small tensors cost one block, not a strided grid row.  float4 accesses.  Per element
// (maximize flips g first):
//     g   = g + wd * p
//     buf = first ? g : momentum * buf + (1 - dampening) * g         (momentum != 0)
//     g   = nesterov ? g + momentum * buf : buf
//     p   = p - lr * g ;   w16 = bf16_rne(p)                          (w16 optional)
// which is torch.optim.SGD's update (torch/optim/sgd.py, _single_tensor_sgd) element for
// element in fp32, followed by BF16Weights.refresh()'s cast -- one pass over p/g/buf instead of
// the foreach kernels (two multi_tensor_apply passes) plus the separate cast pass.
// Communication fault guard: while the process-wide fault flag (csrc/comm/health.cpp, set e.g.
// by a timed-out xGMI peer wait in the same step) is raised, every block returns before touching
// p / buf -- a corrupted exchange inside a replayed HIP graph never reaches the weights, and the
// host sees the flag through health_check() without a device sync.
#include "grace_common.h"
#include "grace_kernels.h"

namespace grace {
namespace {

constexpr int kBlock = 256;

struct SgdTable {
  float* p[kSgdSegs];
  const float* g[kSgdSegs];
  float* buf[kSgdSegs];       // nullptr when momentum == 0
  uint16_t* w16[kSgdSegs];    // nullptr: no working copy
  int64_t len[kSgdSegs];
  int32_t start[kSgdSegs + 1];  // first block of each tensor; start[n] = grid size
  int32_t n;
};
constexpr int kTile = kBlock * 4 * 4;  // elements per block (4 float4 per thread)

struct SgdHyper {
  float lr, momentum, dampening, wd;
  int nesterov, maximize, first;
};

__device__ __forceinline__ float sgd_elem(float& p, float g, float* bufp, const SgdHyper& h) {
  if (h.maximize) g = -g;
  if (h.wd != 0.f) g = fmaf(h.wd, p, g);
  if (bufp) {
    const float b = h.first ? g : fmaf(h.momentum, *bufp, (1.f - h.dampening) * g);
    *bufp = b;
    g = h.nesterov ? fmaf(h.momentum, b, g) : b;
  }
  p = fmaf(-h.lr, g, p);
  return p;
}

__global__ __launch_bounds__(kBlock) void sgd_kernel(SgdTable t, SgdHyper h, const uint32_t* __restrict__ fault) {
  if (fault != nullptr && __hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  int lo = 0, hi = t.n - 1;  // last tensor with start <= blockIdx.x
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.start[mid] <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const int s = lo;
  const int64_t e0 = (int64_t)(blockIdx.x - t.start[s]) * kTile;
  const int64_t n = min(t.len[s] - e0, (int64_t)kTile);  // this block's elements
  float* __restrict__ p = t.p[s] + e0;
  const float* __restrict__ g = t.g[s] + e0;
  float* __restrict__ buf = t.buf[s] ? t.buf[s] + e0 : nullptr;
  uint16_t* __restrict__ w = t.w16[s] ? t.w16[s] + e0 : nullptr;
  const int64_t stride = kBlock;
  int64_t tail = 0;
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                     reinterpret_cast<uintptr_t>(buf)) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(w) & 7) == 0;
  if (vec) {
    const int64_t nv = n >> 2;
    const bool m = buf != nullptr;
    // all of a thread's (up to) 4 vectors' loads are issued before the first store: 12 16-B
    // loads in flight per thread instead of 3 (the per-iteration store -> next load ordering
    // otherwise serialises the passes; 3.9 TB/s measured before)
    constexpr int U = kTile / 4 / kBlock;
    float4 pv[U], gv[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = threadIdx.x + (int64_t)u * stride;
      pv[u] = gv[u] = bv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < nv) {
        pv[u] = reinterpret_cast<float4*>(p)[i];
        gv[u] = reinterpret_cast<const float4*>(g)[i];
        if (m) bv[u] = reinterpret_cast<float4*>(buf)[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = threadIdx.x + (int64_t)u * stride;
      if (i >= nv) continue;
      sgd_elem(pv[u].x, gv[u].x, m ? &bv[u].x : nullptr, h);
      sgd_elem(pv[u].y, gv[u].y, m ? &bv[u].y : nullptr, h);
      sgd_elem(pv[u].z, gv[u].z, m ? &bv[u].z : nullptr, h);
      sgd_elem(pv[u].w, gv[u].w, m ? &bv[u].w : nullptr, h);
      reinterpret_cast<float4*>(p)[i] = pv[u];
      if (m) reinterpret_cast<float4*>(buf)[i] = bv[u];
      if (w) {
        uint2 o;
        o.x = (uint32_t)f32_to_bf16_rne(pv[u].x) | ((uint32_t)f32_to_bf16_rne(pv[u].y) << 16);
        o.y = (uint32_t)f32_to_bf16_rne(pv[u].z) | ((uint32_t)f32_to_bf16_rne(pv[u].w) << 16);
        reinterpret_cast<uint2*>(w)[i] = o;
      }
    }
    tail = nv << 2;
  }
  for (int64_t i = tail + threadIdx.x; i < n; i += stride) {
    float pv = p[i];
    sgd_elem(pv, g[i], buf ? buf + i : nullptr, h);
    p[i] = pv;
    if (w) w[i] = f32_to_bf16_rne(pv);
  }
}

}  // namespace

void sgd_step(float* const* p, const float* const* g, float* const* buf, uint16_t* const* w16, const int64_t* len,
              int n_seg, float lr, float momentum, float dampening, float wd, bool nesterov, bool maximize,
              bool first, hipStream_t stream) {
  // the fault word of the device this stream launches on (never another GPU's memory)
  int dev = -1;
  if (hipStreamGetDevice(stream, &dev) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipGetDevice(&dev);
  }
  const uint32_t* dev_fault = health_dev(dev);
  SgdHyper h{lr, momentum, dampening, wd, nesterov ? 1 : 0, maximize ? 1 : 0, first ? 1 : 0};
  for (int s0 = 0; s0 < n_seg; s0 += kSgdSegs) {
    const int m = n_seg - s0 < kSgdSegs ? n_seg - s0 : kSgdSegs;
    SgdTable t{};
    int32_t nb = 0;
    for (int i = 0; i < m; ++i) {
      t.p[i] = p[s0 + i];
      t.g[i] = g[s0 + i];
      t.buf[i] = buf[s0 + i];
      t.w16[i] = w16[s0 + i];
      t.len[i] = len[s0 + i];
      t.start[i] = nb;
      nb += (int32_t)((len[s0 + i] + kTile - 1) / kTile);
    }
    t.start[m] = nb;
    t.n = m;
    const uint32_t* fault = dev_fault ? dev_fault + kHealthFault : nullptr;
    if (nb > 0) hipLaunchKernelGGL(sgd_kernel, dim3((unsigned)nb), dim3(kBlock), 0, stream, t, h, fault);
  }
}

}  // namespace grace
