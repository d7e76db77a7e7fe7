// zk_runtime.cpp -- per-device context: stream, grow-only arena, pinned staging.
#include "zk_runtime.hpp"
#include <string.h>
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

// ---------------------------------------------------------------------------- staged copies
static constexpr size_t RING_CHUNK = (size_t)32 << 20;

static void ring_init(Device &dev) {
  if (dev.ring[0]) return;
  for (int i = 0; i < 2; i++) {
    ZK_CHECK(hipHostMalloc(&dev.ring[i], RING_CHUNK, hipHostMallocDefault));
    ZK_CHECK(hipEventCreateWithFlags(&dev.ring_ev[i], hipEventDisableTiming));
  }
}

// memcpy on the host pool: 4 MiB pieces
static void par_memcpy(void *dst, const void *src, size_t bytes) {
  constexpr size_t PIECE = (size_t)4 << 20;
  const int np = (int)((bytes + PIECE - 1) / PIECE);
  host_parallel_for(np, [&](int i) {
    const size_t off = (size_t)i * PIECE;
    const size_t len = bytes - off < PIECE ? bytes - off : PIECE;
    memcpy((char *)dst + off, (const char *)src + off, len);
  });
}

void copy_h2d_staged(Device &dev, void *dst_dev, const void *src_host, size_t bytes) {
  if (bytes == 0) return;
  ring_init(dev);
  size_t off = 0;
  for (int k = 0; off < bytes; k++, off += RING_CHUNK) {
    const size_t len = bytes - off < RING_CHUNK ? bytes - off : RING_CHUNK;
    const int r = k & 1;
    ZK_CHECK(hipEventSynchronize(dev.ring_ev[r]));  // the DMA that last read this chunk is done
    par_memcpy(dev.ring[r], (const char *)src_host + off, len);
    ZK_CHECK(hipMemcpyAsync((char *)dst_dev + off, dev.ring[r], len, hipMemcpyHostToDevice, dev.stream));
    ZK_CHECK(hipEventRecord(dev.ring_ev[r], dev.stream));
  }
}

void copy_d2h_staged(Device &dev, void *dst_host, const void *src_dev, size_t bytes) {
  if (bytes == 0) return;
  ring_init(dev);
  const int nk = (int)((bytes + RING_CHUNK - 1) / RING_CHUNK);
  auto len_of = [&](int k) {
    const size_t off = (size_t)k * RING_CHUNK;
    return bytes - off < RING_CHUNK ? bytes - off : RING_CHUNK;
  };
  for (int k = 0; k <= nk; k++) {
    if (k < nk) {  // DMA chunk k into ring[k & 1] (its previous contents were copied out in step k-1)
      ZK_CHECK(hipMemcpyAsync(dev.ring[k & 1], (const char *)src_dev + (size_t)k * RING_CHUNK, len_of(k),
                              hipMemcpyDeviceToHost, dev.stream));
      ZK_CHECK(hipEventRecord(dev.ring_ev[k & 1], dev.stream));
    }
    if (k >= 1) {  // meanwhile copy chunk k-1 out to the caller
      const int j = k - 1;
      ZK_CHECK(hipEventSynchronize(dev.ring_ev[j & 1]));
      par_memcpy((char *)dst_host + (size_t)j * RING_CHUNK, dev.ring[j & 1], len_of(j));
    }
  }
}

// ---------------------------------------------------------------------------- kernel timer
static std::atomic<bool> g_timer_on{false};

void timer_set_enabled(bool on) { g_timer_on.store(on); }

void timer_begin(Device &dev) {
  if (!g_timer_on.load()) {
    dev.timer.armed = false;
    return;
  }
  if (!dev.timer.ev0) {  // created on the device whose stream records them (the caller's)
    ZK_CHECK(hipEventCreate(&dev.timer.ev0));
    ZK_CHECK(hipEventCreate(&dev.timer.ev1));
  }
  dev.timer.armed = true;
  ZK_CHECK(hipEventRecord(dev.timer.ev0, dev.stream));
}

void timer_end(Device &dev) {
  if (dev.timer.armed) ZK_CHECK(hipEventRecord(dev.timer.ev1, dev.stream));
}

void timer_collect(Device &dev) {
  if (!dev.timer.armed) return;
  float ms = 0;
  ZK_CHECK(hipEventSynchronize(dev.timer.ev1));
  ZK_CHECK(hipEventElapsedTime(&ms, dev.timer.ev0, dev.timer.ev1));
  dev.timer.total_ms += ms;
  dev.timer.launches++;
  dev.timer.armed = false;
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
