// Native RCCL communication runtime for grace_amd (one process per MI355X, RCCL over xGMI).
//
// The reference relies on Horovod's C++ core (background thread, handle table, poll /
// synchronize -- /root/reference/patch_files/horovod/torch/mpi_ops.py:57-60, 407-439) for async
// collectives.  Here the equivalent is small and stream-native:
//
//   * RcclComm owns its own ncclComm_t (bootstrapped from a unique id exchanged through the
//     torch.distributed Store by the Python side) and a dedicated high-priority HIP stream;
//   * every collective first makes the comm stream wait on the caller's current stream (an
//     event, no host sync), is issued on the comm stream, and records a completion event;
//   * Work::wait() makes the caller's current stream wait on that event (the host never
//     blocks); Work::is_completed() polls it; Work::synchronize() blocks the host (debug);
//   * group() batches several collectives into one ncclGroupStart/End (one launch for all
//     payload tensors of many buckets);
//   * a watchdog-friendly check_async_error() surfaces RCCL failures (peer death, timeouts)
//     instead of hanging, and abort() tears the communicator down.
//
// Everything is graph-capturable: no allocation and no host synchronisation on the issue path.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace grace_comm {

using at::Tensor;

#define RCCL_CHECK(expr)                                                                             \
  do {                                                                                               \
    ncclResult_t _r = (expr);                                                                        \
    if (_r != ncclSuccess) throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + \
                                                    " at " #expr);                                   \
  } while (0)
#define HIP_OK(expr)                                                                                 \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                                                   " at " #expr);                                    \
  } while (0)

// Set from Python's atexit: once the interpreter is shutting down the HIP runtime / RCCL may
// already be torn down, so destructors must not call into them (leaking at exit is harmless).
static std::atomic<bool> g_exiting{false};
void mark_exiting() { g_exiting.store(true); }

inline hipStream_t current_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

ncclDataType_t nccl_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kChar: return ncclInt8;
    case at::kByte: return ncclUint8;
    case at::kBool: return ncclUint8;
    case at::kShort:
    default: break;
  }
  throw std::runtime_error("unsupported dtype for RCCL");
}

// bool tensors travel as bytes; only max / min keep them 0/1 (a "sum" would produce 2, 3, ...)
void check_bool_op(const Tensor& t, const std::string& op) {
  if (t.scalar_type() == at::kBool && op != "max" && op != "min")
    throw std::runtime_error("bool all_reduce supports only max / min (logical or / and)");
}

ncclRedOp_t nccl_op(const std::string& op) {
  if (op == "sum") return ncclSum;
  if (op == "max") return ncclMax;
  if (op == "min") return ncclMin;
  if (op == "prod") return ncclProd;
  if (op == "avg") return ncclAvg;
  throw std::runtime_error("unsupported reduce op " + op);
}

class Work {
 public:
  // with_event = false: an inline collective issued while its stream was being captured into a
  // HIP graph; it is ordered by the stream itself, so there is nothing to wait on.
  explicit Work(int device, bool with_event = true) : device_(device) {
    if (with_event) HIP_OK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }
  ~Work() {
    if (done_ != nullptr && !g_exiting.load()) (void)hipEventDestroy(done_);
  }
  hipEvent_t event() const { return done_; }
  void wait() {  // stream-level: the caller's current stream (on the comm's device) waits
    if (done_ == nullptr) return;
    c10::hip::HIPGuardMasqueradingAsCUDA guard(device_);
    HIP_OK(hipStreamWaitEvent(current_stream(), done_, 0));
  }
  bool is_completed() {
    if (done_ == nullptr) return true;
    hipError_t e = hipEventQuery(done_);
    if (e == hipSuccess) return true;
    if (e == hipErrorNotReady) return false;
    HIP_OK(e);
    return false;
  }
  void synchronize() {
    if (done_ != nullptr) HIP_OK(hipEventSynchronize(done_));
  }

 private:
  int device_;
  hipEvent_t done_ = nullptr;
};

py::bytes unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

class RcclComm {
 public:
  // min_ctas / max_ctas > 0: the communicator's workgroup (channel) budget through ncclConfig_t --
  // one ring drives one outbound xGMI link per GPU, so a dense all-reduce over the 7-link mesh
  // needs several channels; the Python side probes candidates on the real bucket size
  // (parallel/native_comm.py RcclComm.tuned).  0 / 0 = RCCL's own choice (ncclCommInitRank).
  RcclComm(int rank, int world, const std::string& id_bytes, int device, bool high_priority, int min_ctas,
           int max_ctas)
      : rank_(rank), world_(world), device_(device), min_ctas_(min_ctas), max_ctas_(max_ctas) {
    if ((int)id_bytes.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad unique id size");
    HIP_OK(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(id.internal, id_bytes.data(), NCCL_UNIQUE_ID_BYTES);
    if (min_ctas > 0 || max_ctas > 0) {
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      if (min_ctas > 0) cfg.minCTAs = min_ctas;
      if (max_ctas > 0) cfg.maxCTAs = max_ctas;
      RCCL_CHECK(ncclCommInitRankConfig(&comm_, world, id, rank, &cfg));
    } else {
      RCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
    }
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, high_priority ? hi : lo));
    HIP_OK(hipEventCreateWithFlags(&fork_, hipEventDisableTiming));
  }
  ~RcclComm() {
    if (g_exiting.load()) return;
    if (comm_ != nullptr) (void)ncclCommDestroy(comm_);
    // The comm stream is deliberately NOT destroyed: tensors that crossed it were
    // record_stream()-ed, and the caching allocator records events on that stream when those
    // tensors are freed -- possibly after this communicator is gone (a destroyed stream there
    // segfaults).  One leaked stream per communicator lifetime is the price.
    (void)hipEventDestroy(fork_);
  }

  int rank() const { return rank_; }
  int min_ctas() const { return min_ctas_; }
  int max_ctas() const { return max_ctas_; }
  int world_size() const { return world_; }
  // what RCCL itself reports for the communicator (ncclCommCount / ncclCommCuDevice): the bench
  // JSON carries it so a driver can check "RCCL saw N ranks" independently of the env
  int nranks() const {
    int n = 0;
    RCCL_CHECK(ncclCommCount(comm_, &n));
    return n;
  }
  int comm_device() const {
    int d = -1;
    RCCL_CHECK(ncclCommCuDevice(comm_, &d));
    return d;
  }
  uintptr_t stream_ptr() const { return reinterpret_cast<uintptr_t>(stream_); }

  std::shared_ptr<Work> all_gather(const Tensor& out, const Tensor& in) {
    Issue is(*this);
    check(out);
    check(in);
    TORCH_CHECK(out.numel() == in.numel() * world_, "all_gather: out must be world_size x in");
    TORCH_CHECK(out.scalar_type() == in.scalar_type(), "dtype mismatch");
    is.begin();
    RCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dtype(in), comm_, is.s));
    return is.end();
  }

  std::shared_ptr<Work> all_reduce(const Tensor& t, const std::string& op) {
    Issue is(*this);
    check(t);
    check_bool_op(t, op);
    is.begin();
    RCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), nccl_op(op), comm_, is.s));
    return is.end();
  }

  std::shared_ptr<Work> broadcast(const Tensor& t, int root) {
    Issue is(*this);
    check(t);
    is.begin();
    RCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), root, comm_, is.s));
    return is.end();
  }

  std::shared_ptr<Work> reduce_scatter(const Tensor& out, const Tensor& in, const std::string& op) {
    Issue is(*this);
    check(out);
    check(in);
    check_bool_op(in, op);
    TORCH_CHECK(in.numel() == out.numel() * world_, "reduce_scatter: in must be world_size x out");
    is.begin();
    RCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dtype(in), nccl_op(op), comm_,
                                 is.s));
    return is.end();
  }

  // out[p] <- chunk `rank` of rank p's in (equal chunks of numel / world): one send and one recv
  // per peer in one group -- on a fully connected xGMI node every pair has its own link
  std::shared_ptr<Work> all_to_all(const Tensor& out, const Tensor& in) {
    Issue is(*this);
    check(out);
    check(in);
    TORCH_CHECK(out.numel() == in.numel() && in.numel() % world_ == 0, "all_to_all: equal sizes, divisible by W");
    TORCH_CHECK(out.scalar_type() == in.scalar_type(), "dtype mismatch");
    const int64_t chunk = in.numel() / world_;
    const size_t esz = in.element_size();
    auto dt = nccl_dtype(in);
    is.begin();
    RCCL_CHECK(ncclGroupStart());
    for (int p = 0; p < world_; ++p) {
      RCCL_CHECK(ncclSend(static_cast<const char*>(in.data_ptr()) + p * chunk * esz, chunk, dt, p, comm_, is.s));
      RCCL_CHECK(ncclRecv(static_cast<char*>(out.data_ptr()) + p * chunk * esz, chunk, dt, p, comm_, is.s));
    }
    RCCL_CHECK(ncclGroupEnd());
    return is.end();
  }

  // Batched: all_gathers of (out_i, in_i) pairs and in-place sum all_reduces in ONE group.
  std::shared_ptr<Work> group(const std::vector<std::pair<Tensor, Tensor>>& gathers,
                              const std::vector<Tensor>& reduces) {
    Issue is(*this);
    for (auto& g : gathers) {
      check(g.first);
      check(g.second);
      TORCH_CHECK(g.first.numel() == g.second.numel() * world_, "group all_gather size");
    }
    for (auto& t : reduces) {
      check(t);
      check_bool_op(t, "sum");
    }
    is.begin();
    RCCL_CHECK(ncclGroupStart());
    for (auto& g : gathers)
      RCCL_CHECK(ncclAllGather(g.second.data_ptr(), g.first.data_ptr(), g.second.numel(), nccl_dtype(g.second),
                               comm_, is.s));
    for (auto& t : reduces)
      RCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), ncclSum, comm_, is.s));
    RCCL_CHECK(ncclGroupEnd());
    return is.end();
  }

  std::string check_async_error() {
    std::shared_lock<std::shared_timed_mutex> lk(mu_);
    if (comm_ == nullptr) return aborted_.load() ? std::string("communicator aborted") : std::string();
    ncclResult_t r = ncclSuccess;
    RCCL_CHECK(ncclCommGetAsyncError(comm_, &r));
    return r == ncclSuccess ? std::string() : std::string(ncclGetErrorString(r));
  }

  // Callable from a watchdog thread while the training thread issues collectives: issue paths
  // hold mu_ shared (enqueue only, never a wait), abort takes it exclusively, so comm_ is never
  // freed under a running ncclXxx call.  If an issuing thread holds the lock for more than 5 s
  // (an enqueue stuck inside RCCL), abort() only marks the communicator aborted and returns
  // false: the issuing thread performs the ncclCommAbort itself when its call returns (Issue's
  // destructor), and every later issue fails on aborted_.  force = true additionally calls
  // ncclCommAbort concurrently -- the documented way to unblock a hung RCCL call, at the price of
  // freeing the communicator under that call (use only when the process is going down anyway).
  bool abort(bool force) {
    aborted_.store(true);
    std::unique_lock<std::shared_timed_mutex> lk(mu_, std::defer_lock);
    if (lk.try_lock_for(std::chrono::seconds(5))) {
      if (comm_ != nullptr) (void)ncclCommAbort(comm_);
      comm_ = nullptr;
      return true;
    }
    if (force) {
      ncclComm_t c = comm_;
      if (c != nullptr && !forced_.exchange(true)) (void)ncclCommAbort(c);
    }
    return false;
  }

 private:
  void check(const Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL tensors must be contiguous GPU tensors");
    TORCH_CHECK(t.get_device() == device_, "tensor on the wrong device");
    TORCH_CHECK(comm_ != nullptr && !aborted_.load(), "communicator aborted");
  }

  // The issue state of ONE collective call, on the calling thread's stack: the shared lock, the
  // device guard and the stream it is issued on (two threads issuing at once -- the DDP hook on
  // the autograd thread and a main-thread all_reduce -- each keep their own).  The fork event
  // is shared, so the record + wait pair runs under fork_mu_.
  //   Forked (default): the comm stream waits on the caller's stream, the collective runs there
  //   and overlaps whatever the caller does next.  Inline: the collective is issued on the
  //   caller's current stream -- inside a whole-step HIP graph that is one more node in a single
  //   chain instead of an event fork + join (a forked capture costs ~0.4 ms/step on MI355X).
  struct Issue {
    RcclComm& c;
    std::shared_lock<std::shared_timed_mutex> lk;
    c10::optional<c10::hip::HIPGuardMasqueradingAsCUDA> guard;
    hipStream_t s = nullptr;
    explicit Issue(RcclComm& comm) : c(comm), lk(comm.mu_) {}
    ~Issue() {
      const bool deferred_abort = c.aborted_.load() && c.comm_ != nullptr && !g_exiting.load();
      guard.reset();
      lk.unlock();
      if (deferred_abort) c.abort(false);  // an abort() that could not take the lock (see abort)
    }
    void begin() {
      // the caller's current stream is looked up on the COMM's device (a different current
      // device would record the fork / run an inline collective on another device's stream)
      guard.emplace(c.device_);
      if (c.inline_) {
        s = current_stream();
        return;
      }
      s = c.stream_;
      std::lock_guard<std::mutex> f(c.fork_mu_);
      HIP_OK(hipEventRecord(c.fork_, current_stream()));
      HIP_OK(hipStreamWaitEvent(c.stream_, c.fork_, 0));
    }
    std::shared_ptr<Work> end() {
      std::shared_ptr<Work> w;
      if (c.inline_) {
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        HIP_OK(hipStreamIsCapturing(s, &st));
        w = std::make_shared<Work>(c.device_, st == hipStreamCaptureStatusNone);
        if (w->event() != nullptr) HIP_OK(hipEventRecord(w->event(), s));
      } else {
        w = std::make_shared<Work>(c.device_);
        HIP_OK(hipEventRecord(w->event(), s));
      }
      return w;
    }
  };

 public:
  void set_inline(bool on) { inline_ = on; }
  bool is_inline() const { return inline_; }

 private:
  int rank_, world_, device_;
  int min_ctas_ = 0, max_ctas_ = 0;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::atomic<bool> inline_{false};
  hipEvent_t fork_;
  std::mutex fork_mu_;
  std::shared_timed_mutex mu_;
  std::atomic<bool> aborted_{false};
  std::atomic<bool> forced_{false};
};

void bind(py::module& m) {
  py::class_<Work, std::shared_ptr<Work>>(m, "RcclWork")
      .def("wait", &Work::wait)
      .def("is_completed", &Work::is_completed)
      .def("synchronize", &Work::synchronize);
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<int, int, const std::string&, int, bool, int, int>(), py::arg("rank"), py::arg("world"),
           py::arg("unique_id"), py::arg("device"), py::arg("high_priority") = true, py::arg("min_ctas") = 0,
           py::arg("max_ctas") = 0)
      .def_property_readonly("min_ctas", &RcclComm::min_ctas)
      .def_property_readonly("max_ctas", &RcclComm::max_ctas)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world_size", &RcclComm::world_size)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("comm_device", &RcclComm::comm_device)
      .def_property_readonly("stream_ptr", &RcclComm::stream_ptr)
      .def("all_gather", &RcclComm::all_gather)
      .def("all_reduce", &RcclComm::all_reduce, py::arg("t"), py::arg("op") = "sum")
      .def("broadcast", &RcclComm::broadcast)
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::arg("out"), py::arg("inp"), py::arg("op") = "sum")
      .def("group", &RcclComm::group)
      .def("all_to_all", &RcclComm::all_to_all)
      .def("check_async_error", &RcclComm::check_async_error)
      .def_property("inline", &RcclComm::is_inline, &RcclComm::set_inline)
      .def("abort", &RcclComm::abort, py::arg("force") = false);
  m.def("rccl_unique_id", &unique_id);
  m.def("rccl_mark_exiting", &mark_exiting);
}

}  // namespace grace_comm

// called from bindings.cpp's PYBIND11_MODULE
void grace_bind_comm(py::module& m) { grace_comm::bind(m); }
