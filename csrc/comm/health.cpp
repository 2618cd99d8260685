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
//   word 2  capacity-payload overflows (count; informational, not a fault: Threshold / DGC spill
//           into the residual, INCEPTIONN drops classes -- grace_amd.parallel.health.overflows())
//
// The reference has no equivalent: Horovod's background thread reports MPI errors through its
// handle table (/root/reference/patch_files/horovod/torch/mpi_ops.py:407-439).
#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "grace_kernels.h"

namespace grace {

namespace {
HealthWords g_health{};
std::mutex g_health_mu;

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " at " + what);
}
}  // namespace

const HealthWords& health_words() { return g_health; }

uint32_t* health_dev(int device) {
  if (device < 0 || device >= kHealthMaxDevices) return nullptr;
  return __atomic_load_n(&g_health.dev[device], __ATOMIC_ACQUIRE);
}

// Host words: pinned, mapped, coherent and PORTABLE (one allocation, valid on every device of the
// process).  Device words: one small allocation per device ordinal, made on that device -- an
// optimizer or comm on device d only ever reads / writes dev[d] (no cross-device pointer, no
// stray context on device 0).
void health_init(int device) {
  std::lock_guard<std::mutex> lk(g_health_mu);
  if (device < 0) hip_ok(hipGetDevice(&device), "hipGetDevice(health)");
  if (device >= kHealthMaxDevices) throw std::runtime_error("health_init: device ordinal out of range");
  if (g_health.host == nullptr) {
    void* h = nullptr;
    hip_ok(hipHostMalloc(&h, kHealthWords * sizeof(uint32_t),
                         hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable),
           "hipHostMalloc(health)");
    std::memset(h, 0, kHealthWords * sizeof(uint32_t));
    void* hd = nullptr;
    hip_ok(hipHostGetDevicePointer(&hd, h, 0), "hipHostGetDevicePointer(health)");
    g_health.host = static_cast<uint32_t*>(h);
    g_health.host_dev = static_cast<uint32_t*>(hd);
  }
  if (g_health.dev[device] == nullptr) {
    int prev = 0;
    hip_ok(hipGetDevice(&prev), "hipGetDevice(health)");
    hip_ok(hipSetDevice(device), "hipSetDevice(health)");
    void* d = nullptr;
    hip_ok(hipMalloc(&d, kHealthWords * sizeof(uint32_t)), "hipMalloc(health)");
    hip_ok(hipMemset(d, 0, kHealthWords * sizeof(uint32_t)), "hipMemset(health)");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize(health)");
    hip_ok(hipSetDevice(prev), "hipSetDevice(health)");
    __atomic_store_n(&g_health.dev[device], static_cast<uint32_t*>(d), __ATOMIC_RELEASE);
  }
}

namespace {

py::tuple health_check() {
  if (g_health.host == nullptr) return py::make_tuple(0u, 0u, 0u);
  const volatile uint32_t* w = g_health.host;
  return py::make_tuple((uint32_t)w[kHealthFault], (uint32_t)w[kHealthXgmiTimeouts], (uint32_t)w[kHealthCapOverflow]);
}

// Clears every copy (synchronous: not for use inside a capture).
void health_reset() {
  if (g_health.host == nullptr) return;
  int prev = 0;
  hip_ok(hipGetDevice(&prev), "hipGetDevice(health_reset)");
  for (int d = 0; d < kHealthMaxDevices; ++d) {
    if (g_health.dev[d] == nullptr) continue;
    hip_ok(hipSetDevice(d), "hipSetDevice(health_reset)");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize(health_reset)");
  }
  volatile uint32_t* w = g_health.host;
  for (int i = 0; i < kHealthWords; ++i) w[i] = 0;
  for (int d = 0; d < kHealthMaxDevices; ++d) {
    if (g_health.dev[d] == nullptr) continue;
    hip_ok(hipSetDevice(d), "hipSetDevice(health_reset)");
    hip_ok(hipMemset(g_health.dev[d], 0, kHealthWords * sizeof(uint32_t)), "hipMemset(health_reset)");
    hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize(health_reset)");
  }
  hip_ok(hipSetDevice(prev), "hipSetDevice(health_reset)");
}

// Test hook: raise the fault as a device kernel would (host words + every device copy).
void health_inject() {
  health_init(-1);
  volatile uint32_t* w = g_health.host;
  w[kHealthFault] = 1;
  uint32_t one = 1;
  for (int d = 0; d < kHealthMaxDevices; ++d)
    if (g_health.dev[d] != nullptr)
      hip_ok(hipMemcpy(g_health.dev[d] + kHealthFault, &one, sizeof(one), hipMemcpyHostToDevice), "hipMemcpy(health)");
}

// device ordinals whose words exist (tests)
std::vector<int> health_devices() {
  std::vector<int> v;
  for (int d = 0; d < kHealthMaxDevices; ++d)
    if (g_health.dev[d] != nullptr) v.push_back(d);
  return v;
}

}  // namespace
}  // namespace grace

void grace_bind_health(py::module& m) {
  m.def("health_init", &grace::health_init, py::arg("device") = -1,
        "allocate the communication health words: host words once, device words of `device` (before capture)");
  m.def("health_devices", &grace::health_devices);
  m.def("health_check", &grace::health_check, "(fault flag, xGMI peer-wait timeouts) read from host-mapped memory");
  m.def("health_reset", &grace::health_reset);
  m.def("health_inject", &grace::health_inject);
}
