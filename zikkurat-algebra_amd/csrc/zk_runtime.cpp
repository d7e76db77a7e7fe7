// zk_runtime.cpp -- per-device context: stream, grow-only arena, pinned staging.
#include "zk_runtime.hpp"

namespace zk {

[[noreturn]] void fatal(const char *what, const char *file, int line) {
  fprintf(stderr, "[zkalgebra_gpu] fatal: %s (%s:%d)\n", what, file, line);
  fflush(stderr);
  abort();
}

void Arena::reserve(size_t bytes) {
  if (bytes <= cap_) return;
  if (base_) ZK_CHECK(hipFree(base_));
  base_ = nullptr;
  cap_ = 0;
  // grow geometrically to avoid re-allocation churn across sizes
  size_t cap = bytes + bytes / 4;
  ZK_CHECK(hipMalloc(&base_, cap));
  cap_ = cap;
}

Arena::~Arena() {
  // process teardown: the runtime may already be gone; leak deliberately
}

void *Device::host_staging(size_t bytes) {
  if (bytes > pinned_cap) {
    if (pinned) ZK_CHECK(hipHostFree(pinned));
    ZK_CHECK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
    pinned_cap = bytes;
  }
  return pinned;
}

static std::mutex g_devices_mu;
static std::vector<Device *> g_devices;

Device &current_device() {
  int id = 0;
  ZK_CHECK(hipGetDevice(&id));
  std::lock_guard<std::mutex> lock(g_devices_mu);
  if ((int)g_devices.size() <= id) g_devices.resize(id + 1, nullptr);
  if (!g_devices[id]) {
    Device *d = new Device();
    d->id = id;
    ZK_CHECK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
    g_devices[id] = d;
  }
  return *g_devices[id];
}

KernelTimer &dominant_timer() {
  static KernelTimer t;
  return t;
}

}  // namespace zk
