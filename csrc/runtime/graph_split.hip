// Cross-graph event nodes for the split-stream whole-step capture (grace_amd/parallel/graph.py,
// GraphedStep(split=True)).
//
// A step whose weight gradients run on a side stream, captured as ONE graph, has parallel
// branches; the HIP runtime launches such a graph node by node (~8 ms of host issue per ResNet-50
// step).  Captured instead as TWO graphs -- the critical stream's work (graph A)
// and the side stream's (graph B) -- each graph is a single linear chain, and the fork points
// between them become EXTERNAL event nodes: A records event E_l (hipEventRecordExternal) where
// the side work of layer l may start, B waits on it (hipEventWaitExternal).  PyTorch-ROCm refuses
// external events in torch.cuda.Event, so they live here.
//
// ExtEvent.record / wait act on a raw hipStream_t (torch.cuda.Stream.cuda_stream) and use the
// external flags only while that stream is capturing; eagerly they are ordinary record / wait.
#include <torch/extension.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "grace_kernels.h"

namespace grace_rt {

namespace py = pybind11;

inline void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " at " + what);
}

inline bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hip_ok(hipStreamIsCapturing(s, &st), "hipStreamIsCapturing");
  return st == hipStreamCaptureStatusActive;
}

class ExtEvent {
 public:
  explicit ExtEvent(int device) : device_(device) {
    int prev = 0;
    hip_ok(hipGetDevice(&prev), "hipGetDevice");
    hip_ok(hipSetDevice(device), "hipSetDevice");
    hip_ok(hipEventCreateWithFlags(&ev_, hipEventDisableTiming), "hipEventCreateWithFlags");
    hip_ok(hipSetDevice(prev), "hipSetDevice");
  }
  ~ExtEvent() {
    if (ev_ != nullptr) (void)hipEventDestroy(ev_);
  }
  ExtEvent(const ExtEvent&) = delete;
  ExtEvent& operator=(const ExtEvent&) = delete;

  // While ``stream`` captures, the node is added to the capturing graph directly (after the
  // stream's current capture dependencies, which then become that node): this HIP runtime
  // rejects hipEventRecordWithFlags(hipEventRecordExternal) inside a capture.
  void record(uintptr_t stream) {
    auto s = reinterpret_cast<hipStream_t>(stream);
    if (capturing(s)) {
      add_node(s, true);
    } else {
      hip_ok(hipEventRecord(ev_, s), "hipEventRecord");
    }
  }
  void wait(uintptr_t stream) {
    auto s = reinterpret_cast<hipStream_t>(stream);
    if (capturing(s)) {
      add_node(s, false);
    } else {
      hip_ok(hipStreamWaitEvent(s, ev_, 0), "hipStreamWaitEvent");
    }
  }
  bool query() {
    hipError_t e = hipEventQuery(ev_);
    if (e == hipSuccess) return true;
    if (e == hipErrorNotReady) return false;
    hip_ok(e, "hipEventQuery");
    return false;
  }
  int device() const { return device_; }

 private:
  void add_node(hipStream_t s, bool rec) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t n = 0;
    hip_ok(hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &n), "hipStreamGetCaptureInfo_v2");
    hipGraphNode_t node = nullptr;
    if (rec)
      hip_ok(hipGraphAddEventRecordNode(&node, g, deps, n, ev_), "hipGraphAddEventRecordNode");
    else
      hip_ok(hipGraphAddEventWaitNode(&node, g, deps, n, ev_), "hipGraphAddEventWaitNode");
    hip_ok(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies),
           "hipStreamUpdateCaptureDependencies");
  }

  int device_;
  hipEvent_t ev_ = nullptr;
};

bool stream_capturing(uintptr_t stream) { return capturing(reinterpret_cast<hipStream_t>(stream)); }

// ---------------------------------------------------------------- flag-word cross-stream sync
// The alternative to event nodes: graph A bumps a generation word at its start and, at fork
// point i, a one-thread kernel publishes that generation into flags[i] (agent-scope release
// store); graph B bumps its own generation word at ITS start and, before the side work of fork
// i, a one-thread kernel spins until flags[i] reaches B's generation (agent-scope acquire load,
// s_sleep back-off).  Both graphs stay pure kernel chains.  A never waits on B, and A is
// enqueued before B on every replay, so even two streams sharing one hardware queue cannot
// deadlock (B would just run after A); the spin is bounded: a wait that exceeds ``spin_limit``
// raises the process-wide fault flag (FusedSGD skips the update, the next replay raises) and
// lets B go on, so a wedged replay can never hang the device.
namespace {

__global__ __launch_bounds__(64) void xs_bump_kernel(int64_t* gen) {
  if (threadIdx.x == 0) __hip_atomic_store(gen, gen[0] + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// ``times`` (optional, 2 words per fork point): s_memrealtime (100 MHz) when A signalled fork i /
// when B's wait for it was satisfied -- a profiler-free timeline of the two graphs
__global__ __launch_bounds__(64) void xs_signal_kernel(int64_t* flags, int idx, const int64_t* gen, int64_t* times) {
  if (threadIdx.x == 0) {
    const int64_t g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (times != nullptr) times[2 * idx] = (int64_t)__builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(flags + idx, g, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(64) void xs_wait_kernel(const int64_t* flags, int idx, const int64_t* gen,
                                                     int64_t spin_limit, uint32_t* fault_dev, uint32_t* fault_host,
                                                     int64_t* times) {
  if (threadIdx.x != 0) return;
  const int64_t want = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int64_t n = 0;
  while (__hip_atomic_load(flags + idx, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < want) {
    __builtin_amdgcn_s_sleep(4);
    if (++n > spin_limit) {
      if (fault_dev != nullptr) __hip_atomic_store(fault_dev, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fault_host != nullptr) __hip_atomic_store(fault_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
  if (times != nullptr) times[2 * idx + 1] = (int64_t)__builtin_amdgcn_s_memrealtime();
}

}  // namespace

void xs_bump(const at::Tensor& gen, uintptr_t stream) {
  TORCH_CHECK(gen.is_cuda() && gen.scalar_type() == at::kLong && gen.numel() >= 1, "xs_bump: int64 cuda word");
  hipLaunchKernelGGL(xs_bump_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     gen.data_ptr<int64_t>());
  hip_ok(hipGetLastError(), "xs_bump");
}

int64_t* times_ptr(const c10::optional<at::Tensor>& times, int64_t idx) {
  if (!times.has_value()) return nullptr;
  TORCH_CHECK(times->is_cuda() && times->scalar_type() == at::kLong && 2 * idx + 1 < times->numel(),
              "xs times: int64 cuda tensor of 2 words per fork point");
  return times->data_ptr<int64_t>();
}

void xs_signal(const at::Tensor& flags, int64_t idx, const at::Tensor& gen, uintptr_t stream,
               const c10::optional<at::Tensor>& times) {
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kLong && idx >= 0 && idx < flags.numel(),
              "xs_signal: index outside the int64 flag words");
  TORCH_CHECK(gen.is_cuda() && gen.scalar_type() == at::kLong && gen.numel() >= 1, "xs_signal: int64 cuda word");
  hipLaunchKernelGGL(xs_signal_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     flags.data_ptr<int64_t>(), (int)idx, gen.data_ptr<int64_t>(), times_ptr(times, idx));
  hip_ok(hipGetLastError(), "xs_signal");
}

void xs_wait(const at::Tensor& flags, int64_t idx, const at::Tensor& gen, int64_t spin_limit, uintptr_t stream,
             const c10::optional<at::Tensor>& times) {
  TORCH_CHECK(flags.is_cuda() && flags.scalar_type() == at::kLong && idx >= 0 && idx < flags.numel(),
              "xs_wait: index outside the int64 flag words");
  TORCH_CHECK(gen.is_cuda() && gen.scalar_type() == at::kLong && gen.numel() >= 1, "xs_wait: int64 cuda word");
  TORCH_CHECK(spin_limit > 0, "xs_wait: spin_limit must be > 0 (an unbounded spin could hang the device)");
  // fault words: the device copy (FusedSGD reads it) and the host-mapped one (GraphedStep /
  // health.check read it without a sync); null until parallel/health.py init() ran
  const grace::HealthWords& hw = grace::health_words();
  hipLaunchKernelGGL(xs_wait_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     flags.data_ptr<int64_t>(), (int)idx, gen.data_ptr<int64_t>(), spin_limit,
                     grace::health_dev(flags.get_device()), hw.host_dev, times_ptr(times, idx));
  hip_ok(hipGetLastError(), "xs_wait");
}

// A stream whose kernels may only occupy the CUs set in ``cu_mask`` (bit i of word i / 32 = CU i;
// hipExtStreamCreateWithCUMask) -- e.g. the weight-gradient side stream kept off a quarter of the
// CUs so its MFMA-bound GEMMs cannot starve the latency-bound critical chain of CUs -- or, with an
// empty mask, a plain non-blocking stream of ``priority``.  Never destroyed (process lifetime:
// tensors that crossed it may be freed later with events recorded on it).
uintptr_t create_stream(int device, int priority, const std::vector<uint32_t>& cu_mask) {
  int prev = 0;
  hip_ok(hipGetDevice(&prev), "hipGetDevice");
  hip_ok(hipSetDevice(device), "hipSetDevice");
  hipStream_t s = nullptr;
  if (!cu_mask.empty())
    hip_ok(hipExtStreamCreateWithCUMask(&s, (uint32_t)cu_mask.size(), cu_mask.data()), "hipExtStreamCreateWithCUMask");
  else
    hip_ok(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority), "hipStreamCreateWithPriority");
  hip_ok(hipSetDevice(prev), "hipSetDevice");
  return reinterpret_cast<uintptr_t>(s);
}

std::vector<uint32_t> stream_cu_mask(uintptr_t stream, int words) {
  std::vector<uint32_t> m((size_t)words, 0u);
  hip_ok(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), (uint32_t)words, m.data()),
         "hipExtStreamGetCUMask");
  return m;
}

// Node-type census of a captured graph (torch.cuda.CUDAGraph.raw_cuda_graph()): a graph with
// anything but kernel / memset / memcpy nodes in one chain (host nodes, event nodes, branches)
// leaves the runtime's packet fast path -- the split-capture diagnostics use this.
std::vector<int64_t> graph_node_types(uintptr_t graph) {
  auto g = reinterpret_cast<hipGraph_t>(graph);
  size_t n = 0;
  hip_ok(hipGraphGetNodes(g, nullptr, &n), "hipGraphGetNodes");
  std::vector<hipGraphNode_t> nodes(n);
  if (n) hip_ok(hipGraphGetNodes(g, nodes.data(), &n), "hipGraphGetNodes");
  std::vector<int64_t> counts(16, 0);
  int64_t multi_dep = 0;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    hip_ok(hipGraphNodeGetType(nd, &t), "hipGraphNodeGetType");
    const int ti = (int)t;
    if (ti >= 0 && ti < 15) counts[ti]++;
    size_t nd_deps = 0;
    hip_ok(hipGraphNodeGetDependencies(nd, nullptr, &nd_deps), "hipGraphNodeGetDependencies");
    if (nd_deps > 1) multi_dep++;
  }
  counts[15] = multi_dep;  // nodes joining more than one predecessor (branches)
  return counts;
}

}  // namespace grace_rt

void grace_bind_runtime(py::module& m) {
  using grace_rt::ExtEvent;
  py::class_<ExtEvent, std::shared_ptr<ExtEvent>>(m, "ExtEvent")
      .def(py::init<int>(), py::arg("device"))
      .def("record", &ExtEvent::record, py::arg("stream"))
      .def("wait", &ExtEvent::wait, py::arg("stream"))
      .def("query", &ExtEvent::query)
      .def_property_readonly("device", &ExtEvent::device);
  m.def("stream_capturing", &grace_rt::stream_capturing, py::arg("stream"));
  m.def("create_stream", &grace_rt::create_stream, py::arg("device"), py::arg("priority") = 0,
        py::arg("cu_mask") = std::vector<uint32_t>{});
  m.def("graph_node_types", &grace_rt::graph_node_types, py::arg("graph"),
        "counts by hipGraphNodeType (0 kernel, 1 memcpy, 2 memset, 3 host, 4 graph, 5 empty, 6 wait event, "
        "7 event record, ...); [15] = nodes with more than one dependency");
  m.def("stream_cu_mask", &grace_rt::stream_cu_mask, py::arg("stream"), py::arg("words") = 8);
  m.def("xs_bump", &grace_rt::xs_bump, py::arg("gen"), py::arg("stream"));
  m.def("xs_signal", &grace_rt::xs_signal, py::arg("flags"), py::arg("idx"), py::arg("gen"), py::arg("stream"),
        py::arg("times") = py::none());
  m.def("xs_wait", &grace_rt::xs_wait, py::arg("flags"), py::arg("idx"), py::arg("gen"), py::arg("spin_limit"),
        py::arg("stream"), py::arg("times") = py::none());
}
