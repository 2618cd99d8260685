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
//     [ Ctrl (256 B): ready generation ][ slot 0: cap bytes ][ slot 1: cap bytes ]
//
// allocated uncached (hipDeviceMallocUncached: no L2 copy of a peer-visible line, like RCCL's
// own flag/FIFO buffers) when the IPC export accepts it, plain hipMalloc otherwise; either way
// the hand-off below uses system-scope release/acquire, so it does not rely on the mapping type.
//
// Per all_gather(out, in) call g (every rank issues the same sequence; g = a DEVICE counter,
// so the two launches are graph-capturable and replay correctly):
//   1. xg_stage: copy `in` into my slot[g & 1]; every block drains its stores and releases at
//      system scope before its arrival; the last block publishes ctrl.ready = g (system-scope
//      store).  Never waits on anything.
//   2. xg_pull, grid (chunks, W): block (c, q) polls peer q's ctrl.ready >= g (bounded spin,
//      s_sleep between polls), one system-scope acquire, then copies its chunk of q's slot
//      into out[q] (own rank: straight from `in`); the launch's last block bumps the counter.
//
// Slot reuse without acknowledgements: rank r rewrites slot[g & 1] only in call g + 2, after
// its call g + 1 pull saw every peer's ready >= g + 1 -- which each peer publishes only after its
// call-g pull (stream order), i.e. after it finished reading r's call-g slot.  Peers are never
// more than one call apart for the same reason, so `ready >= g` (wrap-safe) is exact.
//
// A wait that times out (a dead or diverged peer) increments `timeouts` and lets the launch
// finish (garbage result, no hung device); XgmiComm.check() turns that into an exception.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

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
constexpr uint32_t kSpinLimit = 1u << 22;  // polls x s_sleep(8) ~ 1-2 s before giving up

struct Local {        // this rank's bookkeeping (plain device memory, never shared)
  uint32_t gen;       // completed all-gathers
  uint32_t arrive1;   // xg_stage arrival counter (re-armed by the last block)
  uint32_t arrive2;   // xg_pull arrival counter
  uint32_t timeouts;  // waits that gave up
};

struct Peers {
  char* base[kMaxWorld];  // every rank's region in THIS process's address space (own = local)
};

__device__ __forceinline__ uint32_t ld_relaxed(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  const uint32_t g = ld_relaxed(&L->gen) + 1u;
  uint4* dst = reinterpret_cast<uint4*>(my_base + kCtrlBytes + (int64_t)(g & 1u) * slot_bytes);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * kThreads)
    dst[i] = in[i];
  if (arrive_last(&L->arrive1, gridDim.x))
    __hip_atomic_store(reinterpret_cast<uint32_t*>(my_base), g, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kThreads) void xg_pull(const uint4* __restrict__ in, int64_t nvec, Peers peers,
                                                    int rank, int64_t slot_bytes, uint4* __restrict__ out,
                                                    Local* L) {
  const int q = blockIdx.y;
  const uint32_t g = ld_relaxed(&L->gen) + 1u;
  const uint4* src = in;
  if (q != rank) {
    if (threadIdx.x == 0) {
      uint32_t* ready = reinterpret_cast<uint32_t*>(peers.base[q]);
      uint32_t spins = 0;
      while ((int32_t)(__hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - g) < 0) {
        __builtin_amdgcn_s_sleep(8);
        if (++spins > kSpinLimit) {
          __hip_atomic_fetch_add(&L->timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: no stale line of q's slot
    }
    __syncthreads();
    src = reinterpret_cast<const uint4*>(peers.base[q] + kCtrlBytes + (int64_t)(g & 1u) * slot_bytes);
  }
  uint4* o = out + (int64_t)q * nvec;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * kThreads)
    o[i] = src[i];
  if (arrive_last(&L->arrive2, gridDim.x * gridDim.y)) __hip_atomic_store(&L->gen, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

inline hipStream_t current_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

class XgmiPeers {
 public:
  XgmiPeers(int rank, int world, int device, int64_t capacity)
      : rank_(rank), world_(world), device_(device), cap_((capacity + 255) / 256 * 256) {
    if (world < 1 || world > kMaxWorld) throw std::runtime_error("xgmi all-gather: world size must be 1..16");
    if (rank < 0 || rank >= world) throw std::runtime_error("xgmi all-gather: bad rank");
    XG_HIP(hipSetDevice(device));
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

  // out = [W, n] bytes, in = [n] bytes; n % 16 == 0 and n <= capacity (checked).  Issued on the
  // caller's current stream (capturable).
  void all_gather(const Tensor& out, const Tensor& in) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi all-gather: open() the peers first");
    TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(), "contiguous GPU tensors");
    TORCH_CHECK(in.get_device() == device_ && out.get_device() == device_, "tensor on the wrong device");
    const int64_t n = in.numel() * in.element_size();
    TORCH_CHECK(out.numel() * out.element_size() == n * world_, "out must be world_size x in");
    TORCH_CHECK(n % 16 == 0 && n <= cap_, "xgmi all-gather: payload must be 16-B granular and <= capacity");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "16-B aligned buffers");
    if (n == 0) return;
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    hipStream_t s = current_stream();
    const int64_t nvec = n / 16;
    const int64_t per_blk = (int64_t)kThreads * 8;  // 8 x 16 B per thread per block pass
    int b1 = (int)std::min<int64_t>(std::max<int64_t>((nvec + per_blk - 1) / per_blk, 1), 256);
    int b2 = (int)std::min<int64_t>(std::max<int64_t>((nvec + per_blk - 1) / per_blk, 1), 64);
    hipLaunchKernelGGL(xg_stage, dim3(b1), dim3(kThreads), 0, s, static_cast<const uint4*>(in.data_ptr()), nvec,
                       mine_, cap_, local_);
    hipLaunchKernelGGL(xg_pull, dim3(b2, world_), dim3(kThreads), 0, s, static_cast<const uint4*>(in.data_ptr()),
                       nvec, peers_, rank_, cap_, static_cast<uint4*>(out.data_ptr()), local_);
    XG_HIP(hipGetLastError());
  }

  uint32_t timeouts() {
    Local h{};
    XG_HIP(hipMemcpy(&h, local_, sizeof(h), hipMemcpyDeviceToHost));
    return h.timeouts;
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
  bool uncached_ = false, opened_ = false;
  char* mine_ = nullptr;
  Local* local_ = nullptr;
  hipIpcMemHandle_t handle_{};
  Peers peers_{};
};

void bind(py::module& m) {
  py::class_<XgmiPeers, std::shared_ptr<XgmiPeers>>(m, "XgmiPeers")
      .def(py::init<int, int, int, int64_t>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("capacity"))
      .def("handle", &XgmiPeers::handle)
      .def("open", &XgmiPeers::open)
      .def("all_gather", &XgmiPeers::all_gather)
      .def("timeouts", &XgmiPeers::timeouts)
      .def("close", &XgmiPeers::close)
      .def_property_readonly("capacity", &XgmiPeers::capacity)
      .def_property_readonly("uncached", &XgmiPeers::uncached);
}

}  // namespace grace_xgmi

// called from bindings.cpp's PYBIND11_MODULE
void grace_bind_xgmi(py::module& m) { grace_xgmi::bind(m); }
