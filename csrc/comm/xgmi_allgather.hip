// One-shot all-gather over xGMI peer memory (grace_amd's small-payload collective).
//
// Why: an 8 x MI355X node is a fully connected xGMI mesh, 7 point-to-point links per GPU.  A
// ring all-gather (RCCL's default schedule for the compressed payloads of the Allgather
// communicator) moves a rank's payload P through W-1 sequential hops; the Top-K 1 % payload
// of ResNet-50 is only ~2 MB per rank, so that schedule is hop-latency bound.  Here every rank
// PULLS each peer's payload directly over that peer's own link, all W-1 links at once: one
// hop, ~P / link-bandwidth (SURVEY.md §5 "direct one-shot allgather").  The reference has no
// equivalent (Horovod's MPI allgather, /root/reference/grace_dl/dist/communicator/allgather.py:
// 15-38, /root/reference/patch_files/horovod/torch/mpi_ops.py:57-89).
//
// Memory: every rank allocates ONE region, exported to the peers as a HIP IPC handle (the
// handles travel through the torch.distributed Store on the Python side):
//
//     [ Ctrl (256 B): ready gen @0, ready slot @4, consumed gen @128 ][ slot D: cap ][ slot S: cap ]
//
// allocated uncached (hipDeviceMallocUncached: stores bypass the XCD L2s, so a payload written
// by ANY earlier kernel is peer-visible once that kernel is done) when the IPC export accepts
// it, plain hipMalloc otherwise.  Slot D ("direct", uncached regions only): the payload builder
// assembles ONE bucket's payload straight into it (XgmiComm.payload_buffer) -- no staging
// copy; every other payload is staged into slot S.  Which slot a rank's payload sits in is
// decided by THAT rank (its input address, its own uncached allocation) and published next to
// its ready generation ("ready slot" word, stored before the release of `ready`): a puller
// reads the peer's choice instead of assuming its own, so ranks that disagree (one fell back
// to a cached region, or gave slot D to a different bucket) still read the right bytes.
//
// Per all_gather(out, in) call g (every rank issues the same sequence; g = a DEVICE counter,
// so the launches are graph-capturable and replay correctly):
//   1. xg_stage (only when `in` is not the slot): copy `in` into my slot; every block drains its
//      stores and releases at system scope before its arrival; the last block publishes
//      ctrl.ready = g.  Direct mode: xg_pull's first block publishes ready = g instead.
//   2. xg_pull, grid (chunks, W): block (c, q) polls peer q's ready >= g (bounded spin, s_sleep
//      between polls), one system-scope acquire, reads the in-band counts of q's payload (when
//      the caller described its variable-length ranges) and copies only the VALID bytes of
//      each range of its chunk into out[q] (own rank: from `in`).  The launch's last block
//      publishes ctrl.consumed = g, waits until every peer's consumed >= g (nobody reads my
//      slot any more), then bumps the device generation.
// So the slot is free again when xg_pull completes: the next call (or the payload builder, in
// direct mode) may rewrite it in stream order.
//
// Failure: a wait that exceeds the spin limit (a dead or diverged peer; ~10 s by default) does
// NOT copy garbage.  The peer's rows of `out` are ZERO-FILLED (every decoder reads a zero
// payload as "nothing sent": count 0 / zero values), and the process-wide fault flag
// (csrc/comm/health.cpp) is raised in both its device copy (FusedSGD then skips the update:
// nothing corrupted reaches the weights) and its host-mapped copy (health_check() / the engine
// raise on the host without a device sync, also under HIP-graph replay).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "grace_kernels.h"

namespace grace_xgmi {

using at::Tensor;

#define XG_HIP(expr)                                                                                 \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                                                   " at " #expr);                                    \
  } while (0)

constexpr int kThreads = 256;
constexpr int kMaxWorld = 16;
constexpr int64_t kCtrlBytes = 256;
constexpr int kReadyWord = 0;
constexpr int kReadySlotWord = 1;  // 0 = slot D (direct), 1 = slot S (staged); same line as ready
constexpr int kConsumedWord = 32;  // own 128-B line
constexpr int kMaxRanges = 8;

struct Local {        // this rank's bookkeeping (plain device memory, never shared)
  uint32_t gen;       // completed all-gathers
  uint32_t arrive1;   // xg_stage arrival counter (re-armed by the last block)
  uint32_t arrive2;   // xg_pull arrival counter
  uint32_t pad;
};

struct Peers {
  char* base[kMaxWorld];  // every rank's region in THIS process's address space (own = local)
};

// The payload as a cover of disjoint 16-B aligned byte ranges.  A variable range's valid bytes
// are sum_j esz[j] * hdr[j] over up to 4 consecutive int32 words of the payload at byte cnt_off
// (rounded up to 16 B, clamped to nbytes); cnt_off < 0: fixed (all nbytes valid).
struct Ranges {
  int n;
  int64_t off[kMaxRanges];
  int64_t nbytes[kMaxRanges];
  int32_t cnt_off[kMaxRanges];
  int32_t esz[kMaxRanges][4];
};

struct Fault {
  uint32_t* host_dev;  // host-mapped health words (system scope), may be null
  uint32_t* dev;       // device health words, may be null
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ void raise_fault(const Fault& f) {
  if (f.host_dev != nullptr) {
    __hip_atomic_fetch_add(f.host_dev + grace::kHealthXgmiTimeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(f.host_dev + grace::kHealthFault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (f.dev != nullptr) __hip_atomic_store(f.dev + grace::kHealthFault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded wait until (int)(*p - g) >= 0; false on timeout
__device__ bool wait_ge(const uint32_t* p, uint32_t g, uint32_t spin_limit) {
  uint32_t spins = 0;
  while ((int32_t)(ld_sys(p) - g) < 0) {
    __builtin_amdgcn_s_sleep(8);
    if (++spins > spin_limit) return false;
  }
  return true;
}

// every wave drained its stores, workgroup barrier, one lane: system-scope release then the
// arrival add; true in thread 0 of the block whose add completed the count.
__device__ __forceinline__ bool arrive_last(uint32_t* counter, uint32_t total) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return false;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: peers read these bytes
  const uint32_t prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (prev != total - 1) return false;
  __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

__global__ __launch_bounds__(kThreads) void xg_stage(const uint4* __restrict__ in, int64_t nvec, char* my_base,
                                                     int64_t slot_bytes, Local* L) {
  const uint32_t g = __hip_atomic_load(&L->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  uint4* dst = reinterpret_cast<uint4*>(my_base + kCtrlBytes + slot_bytes);  // slot S
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * kThreads)
    dst[i] = in[i];
  if (arrive_last(&L->arrive1, gridDim.x)) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(my_base) + kReadySlotWord, 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(reinterpret_cast<uint32_t*>(my_base) + kReadyWord, g, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// valid 16-B vectors of range i of the payload starting at p (counts read with system loads)
__device__ __forceinline__ int64_t range_vecs(const Ranges& R, int i, const char* p) {
  if (R.cnt_off[i] < 0) return R.nbytes[i] >> 4;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(p + R.cnt_off[i]);
  int64_t b = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (R.esz[i][j] != 0) b += (int64_t)R.esz[i][j] * (int64_t)(int32_t)ld_sys(h + j);
  if (b < 0) b = 0;
  b = (b + 15) >> 4;
  const int64_t mx = R.nbytes[i] >> 4;
  return b < mx ? b : mx;
}

// span: bytes per peer row of `out`; src_shift: byte offset of the pulled part inside every
// payload (0 for the all-gather; rank * chunk for the all-to-all: each rank pulls ITS chunk of
// every peer's payload -- one hop per pair, over that pair's own link)
__global__ __launch_bounds__(kThreads) void xg_pull(const char* __restrict__ in, Ranges R, Peers peers, int rank,
                                                    int world, int direct, uint32_t spin_limit, int64_t span,
                                                    int64_t src_shift, int64_t slot_bytes,
                                                    char* __restrict__ out, Local* L, Fault F, uint32_t fillw) {
  __shared__ int64_t nv[kMaxRanges];
  __shared__ int ok;
  __shared__ int64_t src_off;  // peer q's slot, as q published it
  const int q = blockIdx.y;
  const uint32_t g = __hip_atomic_load(&L->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  char* my_base = peers.base[rank];
  if (direct && blockIdx.x == 0 && q == rank && threadIdx.x == 0) {
    // the payload builder wrote the (uncached) slot in earlier kernels of this stream
    __hip_atomic_store(reinterpret_cast<uint32_t*>(my_base) + kReadySlotWord, 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(reinterpret_cast<uint32_t*>(my_base) + kReadyWord, g, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const char* src = in;
  if (threadIdx.x == 0) {
    ok = 1;
    if (q != rank) {
      if (!wait_ge(reinterpret_cast<const uint32_t*>(peers.base[q]) + kReadyWord, g, spin_limit)) {
        ok = 0;
        raise_fault(F);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale line of q's slot
    }
    src_off = (q != rank && ld_sys(reinterpret_cast<const uint32_t*>(peers.base[q]) + kReadySlotWord) != 0u)
                  ? slot_bytes : 0;
    const char* s = (q == rank ? in : peers.base[q] + kCtrlBytes + src_off) + src_shift;
    for (int i = 0; i < R.n; ++i) nv[i] = ok ? range_vecs(R, i, s) : 0;
  }
  __syncthreads();
  if (q != rank) src = peers.base[q] + kCtrlBytes + src_off;
  src += src_shift;
  char* o = out + (int64_t)q * span;
  const int64_t tid = (int64_t)blockIdx.x * kThreads + threadIdx.x, stride = (int64_t)gridDim.x * kThreads;
  if (ok) {
    for (int i = 0; i < R.n; ++i) {
      const uint4* s4 = reinterpret_cast<const uint4*>(src + R.off[i]);
      uint4* o4 = reinterpret_cast<uint4*>(o + R.off[i]);
      for (int64_t v = tid; v < nv[i]; v += stride) o4[v] = s4[v];
    }
  } else {  // timed-out peer: its rows read as an empty payload (fill 0) or as NaN (an all-reduce's
            // rows: a zero would be a silently wrong sum), never as stale bytes
    uint4* o4 = reinterpret_cast<uint4*>(o);
    for (int64_t v = tid; v < (span >> 4); v += stride) o4[v] = make_uint4(fillw, fillw, fillw, fillw);
  }
  if (arrive_last(&L->arrive2, gridDim.x * gridDim.y)) {
    // every peer block of this launch has read its peer's slot: tell the peers, then wait until
    // no peer reads MY slot any more before the generation (and the slot) moves on
    __hip_atomic_store(reinterpret_cast<uint32_t*>(my_base) + kConsumedWord, g, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      if (!wait_ge(reinterpret_cast<const uint32_t*>(peers.base[p]) + kConsumedWord, g, spin_limit)) raise_fault(F);
    }
    __hip_atomic_store(&L->gen, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

inline hipStream_t current_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

class XgmiPeers {
 public:
  XgmiPeers(int rank, int world, int device, int64_t capacity, int64_t spin_limit)
      : rank_(rank), world_(world), device_(device), cap_((capacity + 255) / 256 * 256),
        spin_((uint32_t)std::max<int64_t>(1, std::min<int64_t>(spin_limit, 0x7fffffff))) {
    if (world < 1 || world > kMaxWorld) throw std::runtime_error("xgmi all-gather: world size must be 1..16");
    if (rank < 0 || rank >= world) throw std::runtime_error("xgmi all-gather: bad rank");
    XG_HIP(hipSetDevice(device));
    grace::health_init(device);
    const size_t bytes = (size_t)(kCtrlBytes + 2 * cap_);
    void* p = nullptr;
    uncached_ = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess;
    if (uncached_ && hipIpcGetMemHandle(&handle_, p) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipFree(p);
      uncached_ = false;
    }
    if (!uncached_) {
      (void)hipGetLastError();
      XG_HIP(hipMalloc(&p, bytes));
      XG_HIP(hipIpcGetMemHandle(&handle_, p));
    }
    mine_ = static_cast<char*>(p);
    XG_HIP(hipMemset(mine_, 0, kCtrlBytes));
    XG_HIP(hipMalloc(&local_, sizeof(Local)));
    XG_HIP(hipMemset(local_, 0, sizeof(Local)));
    XG_HIP(hipDeviceSynchronize());  // zeroed before any peer can poll it
    std::memset(&peers_, 0, sizeof(peers_));
    peers_.base[rank_] = mine_;
  }
  ~XgmiPeers() { close(); }

  py::bytes handle() const { return py::bytes(reinterpret_cast<const char*>(&handle_), sizeof(handle_)); }

  // peers' handles in rank order (own entry ignored)
  void open(const std::vector<std::string>& handles) {
    if ((int)handles.size() != world_) throw std::runtime_error("xgmi all-gather: need one handle per rank");
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    for (int q = 0; q < world_; ++q) {
      if (q == rank_) continue;
      if (handles[q].size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("xgmi all-gather: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[q].data(), sizeof(h));
      void* p = nullptr;
      XG_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      peers_.base[q] = static_cast<char*>(p);
    }
    opened_ = true;
  }

  // Device address of slot D (the payload builder may assemble ONE payload there: direct mode,
  // uncached regions only -- see the header).
  uintptr_t slot_ptr() const { return reinterpret_cast<uintptr_t>(mine_ + kCtrlBytes); }

  // uint8 [nbytes] tensor aliasing slot D (no ownership: valid while this object lives)
  Tensor slot_tensor(int64_t nbytes) const {
    TORCH_CHECK(uncached_, "xgmi all-gather: slot D needs an uncached region");
    TORCH_CHECK(nbytes > 0 && nbytes <= cap_, "slot_tensor: size");
    return torch::from_blob(mine_ + kCtrlBytes, {nbytes},
                            torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, device_));
  }

  // out = [W, n] bytes, in = [n] bytes; n % 16 == 0 and n <= capacity (checked).  `ranges`
  // (int64 [k, 8]: off, nbytes, cnt_off, esz0..esz3, unused) describes the variable-length
  // parts (empty = the whole payload fixed).  Issued on the caller's current stream (capturable).
  // `fill`: the 32-bit word written over a timed-out peer's rows (0: an empty payload for the
  // Allgather decoders; 0xFFFFFFFF: NaN in fp32 / bf16 / fp16, for the gather-reduce all-reduce)
  void all_gather(const Tensor& out, const Tensor& in, const Tensor& ranges, int64_t fill) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi all-gather: open() the peers first");
    TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(), "contiguous GPU tensors");
    TORCH_CHECK(in.get_device() == device_ && out.get_device() == device_, "tensor on the wrong device");
    const int64_t n = in.numel() * in.element_size();
    TORCH_CHECK(out.numel() * out.element_size() == n * world_, "out must be world_size x in");
    TORCH_CHECK(n % 16 == 0 && n <= cap_, "xgmi all-gather: payload must be 16-B granular and <= capacity");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "16-B aligned buffers");
    Ranges R{};
    if (ranges.numel() == 0) {
      R.n = 1;
      R.off[0] = 0;
      R.nbytes[0] = n;
      R.cnt_off[0] = -1;
    } else {
      TORCH_CHECK(!ranges.is_cuda() && ranges.scalar_type() == at::kLong && ranges.dim() == 2 && ranges.size(1) == 8 &&
                      ranges.size(0) <= kMaxRanges, "ranges: CPU int64 [k <= 8, 8]");
      auto a = ranges.accessor<int64_t, 2>();
      R.n = (int)ranges.size(0);
      int64_t end = 0;
      for (int i = 0; i < R.n; ++i) {
        R.off[i] = a[i][0];
        R.nbytes[i] = a[i][1];
        R.cnt_off[i] = (int32_t)a[i][2];
        for (int j = 0; j < 4; ++j) R.esz[i][j] = (int32_t)a[i][3 + j];
        TORCH_CHECK(R.off[i] == end && R.off[i] % 16 == 0 && R.nbytes[i] % 16 == 0 && R.nbytes[i] >= 0,
                    "ranges must tile the payload in order, 16-B aligned");
        TORCH_CHECK(R.cnt_off[i] < 0 || (R.cnt_off[i] % 4 == 0 && R.cnt_off[i] + 16 <= n), "bad count offset");
        end += R.nbytes[i];
      }
      TORCH_CHECK(end == n, "ranges must cover the payload exactly");
    }
    if (n == 0) return;
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    hipStream_t s = current_stream();
    const int64_t nvec = n / 16;
    const int64_t per_blk = (int64_t)kThreads * 8;  // 8 x 16 B per thread per block pass
    const bool direct = reinterpret_cast<uintptr_t>(in.data_ptr()) == slot_ptr();
    TORCH_CHECK(!direct || uncached_, "xgmi all-gather: direct slot writes need an uncached slot");
    if (!direct) {
      int b1 = (int)std::min<int64_t>(std::max<int64_t>((nvec + per_blk - 1) / per_blk, 1), 256);
      hipLaunchKernelGGL(xg_stage, dim3(b1), dim3(kThreads), 0, s, static_cast<const uint4*>(in.data_ptr()), nvec,
                         mine_, cap_, local_);
    }
    int b2 = (int)std::min<int64_t>(std::max<int64_t>((nvec + per_blk - 1) / per_blk, 1), 64);
    const auto& hw = grace::health_words();
    Fault F{hw.host_dev, grace::health_dev(device_)};
    hipLaunchKernelGGL(xg_pull, dim3(b2, world_), dim3(kThreads), 0, s, static_cast<const char*>(in.data_ptr()), R,
                       peers_, rank_, world_, direct ? 1 : 0, spin_, n, (int64_t)0, cap_,
                       static_cast<char*>(out.data_ptr()), local_, F, (uint32_t)fill);
    XG_HIP(hipGetLastError());
  }

  // out[p] = chunk `rank` of rank p's in (chunk = n / W), the all-to-all of the QSGD compressed-
  // domain reduce-scatter: the payload is staged / published exactly like an all-gather's and
  // every rank pulls only its own chunk of each peer's -- (W-1)/W of n over W-1 links at once.
  // out and in: n bytes each, n % (16 W) == 0, n <= capacity.  A timed-out peer's chunk is NaN-
  // filled (0xFF words: the int8 codes then decode as -1 levels, so the fault word is what marks
  // the step; FusedSGD skips it).
  void all_to_all(const Tensor& out, const Tensor& in) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi all-to-all: open() the peers first");
    TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(), "contiguous GPU tensors");
    TORCH_CHECK(in.get_device() == device_ && out.get_device() == device_, "tensor on the wrong device");
    const int64_t n = in.numel() * in.element_size();
    TORCH_CHECK(out.numel() * out.element_size() == n, "all_to_all: out and in must be the same size");
    TORCH_CHECK(n % (16 * world_) == 0 && n <= cap_, "xgmi all-to-all: 16-B granular chunks, <= capacity");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "16-B aligned buffers");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) != slot_ptr(), "all_to_all: stage from a tensor, not slot D");
    if (n == 0) return;
    const int64_t chunk = n / world_;
    Ranges R{};
    R.n = 1;
    R.off[0] = 0;
    R.nbytes[0] = chunk;
    R.cnt_off[0] = -1;
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    hipStream_t s = current_stream();
    const int64_t per_blk = (int64_t)kThreads * 8;
    int b1 = (int)std::min<int64_t>(std::max<int64_t>((n / 16 + per_blk - 1) / per_blk, 1), 256);
    hipLaunchKernelGGL(xg_stage, dim3(b1), dim3(kThreads), 0, s, static_cast<const uint4*>(in.data_ptr()), n / 16,
                       mine_, cap_, local_);
    int b2 = (int)std::min<int64_t>(std::max<int64_t>((chunk / 16 + per_blk - 1) / per_blk, 1), 64);
    const auto& hw = grace::health_words();
    Fault F{hw.host_dev, grace::health_dev(device_)};
    hipLaunchKernelGGL(xg_pull, dim3(b2, world_), dim3(kThreads), 0, s, static_cast<const char*>(in.data_ptr()), R,
                       peers_, rank_, world_, 0, spin_, chunk, (int64_t)rank_ * chunk, cap_,
                       static_cast<char*>(out.data_ptr()), local_, F, 0xFFFFFFFFu);
    XG_HIP(hipGetLastError());
  }

  int64_t capacity() const { return cap_; }
  bool uncached() const { return uncached_; }

  void close() {
    if (mine_ == nullptr) return;
    (void)hipSetDevice(device_);
    (void)hipDeviceSynchronize();
    for (int q = 0; q < world_; ++q)
      if (q != rank_ && peers_.base[q] != nullptr) (void)hipIpcCloseMemHandle(peers_.base[q]);
    (void)hipFree(mine_);
    (void)hipFree(local_);
    mine_ = nullptr;
    local_ = nullptr;
  }

 private:
  int rank_, world_, device_;
  int64_t cap_;
  uint32_t spin_;
  bool uncached_ = false, opened_ = false;
  char* mine_ = nullptr;
  Local* local_ = nullptr;
  hipIpcMemHandle_t handle_{};
  Peers peers_{};
};

void bind(py::module& m) {
  py::class_<XgmiPeers, std::shared_ptr<XgmiPeers>>(m, "XgmiPeers")
      .def(py::init<int, int, int, int64_t, int64_t>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("capacity"), py::arg("spin_limit") = (int64_t)1 << 25)
      .def("handle", &XgmiPeers::handle)
      .def("open", &XgmiPeers::open)
      .def("all_gather", &XgmiPeers::all_gather, py::arg("out"), py::arg("inp"), py::arg("ranges"),
           py::arg("fill") = (int64_t)0)
      .def("all_to_all", &XgmiPeers::all_to_all, py::arg("out"), py::arg("inp"))
      .def("slot_ptr", &XgmiPeers::slot_ptr)
      .def("slot_tensor", &XgmiPeers::slot_tensor)
      .def("close", &XgmiPeers::close)
      .def_property_readonly("capacity", &XgmiPeers::capacity)
      .def_property_readonly("uncached", &XgmiPeers::uncached);
}

}  // namespace grace_xgmi

// called from bindings.cpp's PYBIND11_MODULE
void grace_bind_xgmi(py::module& m) { grace_xgmi::bind(m); }
