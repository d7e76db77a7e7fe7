// zk_runtime.cpp -- per-device context: stream, grow-only arena, pinned staging.
#include "zk_runtime.hpp"
#include <atomic>

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

void stream_wait(Device &dev, hipStream_t st) {
  if (!dev.sync_ev) ZK_CHECK(hipEventCreateWithFlags(&dev.sync_ev, hipEventDisableTiming));
  ZK_CHECK(hipEventRecord(dev.sync_ev, st));
  for (;;) {
    const hipError_t e = hipEventQuery(dev.sync_ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) ZK_CHECK(e);
  }
}

// ---------------------------------------------------------------------------- kernel timer
static std::atomic<bool> g_timer_on{false};

void timer_set_enabled(bool on) { g_timer_on.store(on); }

void timer_begin(Device &dev, int slot, hipStream_t st) {
  if (slot < 0 || slot > 1) return;
  if (!g_timer_on.load()) {
    dev.timer.armed[slot] = false;
    return;
  }
  if (!dev.timer.ev0[slot]) {  // created on the device whose streams record them (the caller's)
    ZK_CHECK(hipEventCreate(&dev.timer.ev0[slot]));
    ZK_CHECK(hipEventCreate(&dev.timer.ev1[slot]));
  }
  dev.timer.armed[slot] = true;
  dev.timer.counted = true;
  ZK_CHECK(hipEventRecord(dev.timer.ev0[slot], st ? st : dev.stream));
}

void timer_end(Device &dev, int slot, hipStream_t st) {
  if (slot < 0 || slot > 1) return;
  if (dev.timer.armed[slot]) ZK_CHECK(hipEventRecord(dev.timer.ev1[slot], st ? st : dev.stream));
}

void timer_collect(Device &dev) {
  for (int k = 0; k < 2; k++) {
    if (!dev.timer.armed[k]) continue;
    float ms = 0;
    ZK_CHECK(hipEventSynchronize(dev.timer.ev1[k]));
    ZK_CHECK(hipEventElapsedTime(&ms, dev.timer.ev0[k], dev.timer.ev1[k]));
    dev.timer.total_ms += ms;
    dev.timer.armed[k] = false;
  }
  if (dev.timer.counted) dev.timer.launches++;
  dev.timer.counted = false;
}

void timer_reset_all() {
  std::vector<Device *> devs;
  {
    std::lock_guard<std::mutex> lock(g_devices_mu);
    devs = g_devices;
  }
  for (Device *d : devs)
    if (d) {
      std::lock_guard<std::mutex> lock(d->mu);
      d->timer.total_ms = 0;
      d->timer.launches = 0;
    }
}

void timer_read_all(double *total_ms, long *launches) {
  std::vector<Device *> devs;
  {
    std::lock_guard<std::mutex> lock(g_devices_mu);
    devs = g_devices;
  }
  double t = 0;
  long n = 0;
  for (Device *d : devs)
    if (d) {
      std::lock_guard<std::mutex> lock(d->mu);
      t += d->timer.total_ms;
      n += d->timer.launches;
    }
  if (total_ms) *total_ms = t;
  if (launches) *launches = n;
}

}  // namespace zk
