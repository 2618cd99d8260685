// Process-wide communication health words: how a device-side communication fault surfaces
// on the host without a device synchronisation, and stops the optimizer from applying a
// corrupted gradient inside a replayed HIP graph.
//
//   host      pinned, host-mapped, coherent (fine-grained) words: device kernels write them
//             with system-scope atomics, the host reads them with a plain load -- health_check()
//             costs nothing and is safe while a stream is being captured or a graph replays;
//   dev       the same fault flag in device memory (cheap to read from every optimizer block).
//
//   word 0  fault flag: any communication fault (set by the xGMI one-shot all-gather when a peer
//           wait times out).  grace::sgd_kernel (FusedSGD) skips its update while it is set.
//   word 1  xGMI peer-wait timeouts (count)
//
// The reference has no equivalent: Horovod's background thread reports MPI errors through its
// handle table (/root/reference/patch_files/horovod/torch/mpi_ops.py:407-439).
#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdexcept>
#include <string>

#include "grace_kernels.h"

namespace grace {

namespace {
HealthWords g_health{nullptr, nullptr, nullptr};
std::mutex g_health_mu;

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " at " + what);
}
}  // namespace

const HealthWords& health_words() { return g_health; }

void health_init() {
  std::lock_guard<std::mutex> lk(g_health_mu);
  if (g_health.host != nullptr) return;
  void* h = nullptr;
  hip_ok(hipHostMalloc(&h, kHealthWords * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent),
         "hipHostMalloc(health)");
  std::memset(h, 0, kHealthWords * sizeof(uint32_t));
  void* hd = nullptr;
  hip_ok(hipHostGetDevicePointer(&hd, h, 0), "hipHostGetDevicePointer(health)");
  void* d = nullptr;
  hip_ok(hipMalloc(&d, kHealthWords * sizeof(uint32_t)), "hipMalloc(health)");
  hip_ok(hipMemset(d, 0, kHealthWords * sizeof(uint32_t)), "hipMemset(health)");
  hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize(health)");
  g_health.host = static_cast<uint32_t*>(h);
  g_health.host_dev = static_cast<uint32_t*>(hd);
  g_health.dev = static_cast<uint32_t*>(d);
}

namespace {

py::tuple health_check() {
  if (g_health.host == nullptr) return py::make_tuple(0u, 0u);
  const volatile uint32_t* w = g_health.host;
  return py::make_tuple((uint32_t)w[kHealthFault], (uint32_t)w[kHealthXgmiTimeouts]);
}

// Clears both copies (synchronous: not for use inside a capture).
void health_reset() {
  if (g_health.host == nullptr) return;
  hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize(health_reset)");
  volatile uint32_t* w = g_health.host;
  for (int i = 0; i < kHealthWords; ++i) w[i] = 0;
  hip_ok(hipMemset(g_health.dev, 0, kHealthWords * sizeof(uint32_t)), "hipMemset(health_reset)");
  hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize(health_reset)");
}

// Test hook: raise the fault as a device kernel would (both copies).
void health_inject() {
  health_init();
  volatile uint32_t* w = g_health.host;
  w[kHealthFault] = 1;
  uint32_t one = 1;
  hip_ok(hipMemcpy(g_health.dev + kHealthFault, &one, sizeof(one), hipMemcpyHostToDevice), "hipMemcpy(health)");
}

}  // namespace
}  // namespace grace

void grace_bind_health(py::module& m) {
  m.def("health_init", &grace::health_init, "allocate the process-wide communication health words (before capture)");
  m.def("health_check", &grace::health_check, "(fault flag, xGMI peer-wait timeouts) read from host-mapped memory");
  m.def("health_reset", &grace::health_reset);
  m.def("health_inject", &grace::health_inject);
}
