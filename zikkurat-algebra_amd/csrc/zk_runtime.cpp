// zk_runtime.cpp -- per-device context: stream, grow-only arena, pinned staging.
#include "zk_runtime.hpp"
#include <atomic>
#include <chrono>
#include <map>
#include <algorithm>
#include <cstring>
#include <thread>

namespace zk {

static std::atomic<int> g_error_mode{0};
void set_error_mode(int mode) { g_error_mode.store(mode == 1 ? 1 : 0); }

[[noreturn]] void fatal(const char *what, const char *file, int line) {
  char msg[512];
  snprintf(msg, sizeof msg, "%s (%s:%d)", what, file, line);
  fprintf(stderr, "[zkalgebra_gpu] %s: %s\n", g_error_mode.load() ? "error" : "fatal", msg);
  fflush(stderr);
  if (g_error_mode.load()) throw Error(msg);
  abort();
}

static thread_local std::string t_last_error;
void record_error(const char *msg) { t_last_error = msg; }
int take_last_error(char *msg, size_t cap) {
  if (t_last_error.empty()) return 0;
  if (msg && cap) {
    strncpy(msg, t_last_error.c_str(), cap - 1);
    msg[cap - 1] = 0;
  }
  t_last_error.clear();
  return 1;
}

static std::atomic<size_t> g_arena_limit{0};
void arena_set_limit(size_t bytes) { g_arena_limit.store(bytes); }

bool Arena::try_reserve(size_t bytes) {
  if (bytes <= cap_) return true;
  const size_t limit = g_arena_limit.load();
  if (limit && bytes > limit) return false;
  if (base_) ZK_CHECK(hipFree(base_));
  base_ = nullptr;
  cap_ = 0;
  // grow geometrically to avoid re-allocation churn across sizes; exactly `bytes` if the
  // headroom does not fit
  size_t cap = bytes + bytes / 4;
  if (limit && cap > limit) cap = limit;
  if (hipMalloc(&base_, cap) != hipSuccess) {
    (void)hipGetLastError();  // out-of-memory is not sticky: clear it
    base_ = nullptr;
    cap = bytes;
    if (hipMalloc(&base_, cap) != hipSuccess) {
      (void)hipGetLastError();
      base_ = nullptr;
      return false;
    }
  }
  cap_ = cap;
  return true;
}

void Arena::reserve(size_t bytes) {
  if (!try_reserve(bytes)) fatal("out of device memory for the call's working set", __FILE__, __LINE__);
}

void Arena::release() {
  if (base_) ZK_CHECK(hipFree(base_));
  base_ = nullptr;
  cap_ = 0;
  off_ = 0;
}

Arena::~Arena() {
  // process teardown: the runtime may already be gone; leak deliberately
}

void *Device::host_staging(size_t bytes) {
  if (bytes > pinned_cap) {
    if (pinned) ZK_CHECK(hipHostFree(pinned));
    ZK_CHECK(hipHostMalloc(&pinned, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    pinned_cap = bytes;
    void *dp = nullptr;
    ZK_CHECK(hipHostGetDevicePointer(&dp, pinned, 0));
    ZK_REQUIRE(dp == pinned, "pinned staging: the device address differs from the host address");
  }
  return pinned;
}

hipStream_t Device::aux_stream() {
  if (!aux) {
    ZK_CHECK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    ZK_CHECK(hipEventCreateWithFlags(&aux_ev, hipEventDisableTiming));
  }
  return aux;
}

hipStream_t Device::aux2_stream() {
  if (!aux2) ZK_CHECK(hipStreamCreateWithFlags(&aux2, hipStreamNonBlocking));
  return aux2;
}

hipEvent_t Device::split_event(int h) {
  while ((int)split_ev.size() <= h) {
    hipEvent_t e;
    ZK_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    split_ev.push_back(e);
  }
  return split_ev[h];
}

void Device::release_memory() {
  arena.release();
  if (pinned) ZK_CHECK(hipHostFree(pinned));
  pinned = nullptr;
  pinned_cap = 0;
  if (xfer) ZK_CHECK(hipHostFree(xfer));
  xfer = nullptr;
  xfer_cap = 0;
}

static std::mutex g_devices_mu;
static std::map<std::pair<int, int>, Device *> g_devices;  // (id, slot) -> context (never freed)

Device &device_context(int id, int slot) {
  std::lock_guard<std::mutex> lock(g_devices_mu);
  auto it = g_devices.find({id, slot});
  if (it != g_devices.end()) return *it->second;
  DeviceGuard on(id);
  hipStream_t stream = nullptr;
  ZK_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  Device *d = new Device();
  d->id = id;
  d->slot = slot;
  d->uid = (int)g_devices.size();
  d->stream = stream;
  g_devices[{id, slot}] = d;
  return *d;
}

Device &current_device() {
  int id = 0;
  ZK_CHECK(hipGetDevice(&id));
  return device_context(id, 0);
}

std::vector<Device *> all_devices() {
  std::lock_guard<std::mutex> lock(g_devices_mu);
  std::vector<Device *> v;
  for (auto &kv : g_devices) v.push_back(kv.second);
  return v;
}

static std::mutex g_set_mu;
static std::vector<int> g_set;
static bool g_set_init = false;

static int device_count_or_zero() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

std::vector<int> device_set() {
  std::lock_guard<std::mutex> lock(g_set_mu);
  if (!g_set_init) {
    g_set_init = true;
    const char *env = getenv("ZKG_DEVICES");
    if (env && *env) {
      const int count = device_count_or_zero();
      std::vector<int> v;
      if (std::string(env) == "all") {
        for (int i = 0; i < count; i++) v.push_back(i);
      } else {
        const char *p = env;
        while (*p) {
          char *end = nullptr;
          const long id = strtol(p, &end, 10);
          if (end == p || id < 0 || id >= count) {
            fprintf(stderr, "[zkalgebra_gpu] ZKG_DEVICES=%s: invalid device list, ignored\n", env);
            v.clear();
            break;
          }
          v.push_back((int)id);
          p = *end == ',' ? end + 1 : end;
        }
      }
      g_set = v;
    }
  }
  return g_set;
}

int set_device_set(const int *ids, int n) {
  const int count = device_count_or_zero();
  for (int i = 0; i < n; i++)
    if (ids[i] < 0 || ids[i] >= count) return -1;
  std::lock_guard<std::mutex> lock(g_set_mu);
  g_set.assign(ids, ids + (n > 0 ? n : 0));
  g_set_init = true;
  return 0;
}

void stream_wait(Device &dev, hipStream_t st) {
  if (!dev.sync_ev) ZK_CHECK(hipEventCreateWithFlags(&dev.sync_ev, hipEventDisableTiming));
  ZK_CHECK(hipEventRecord(dev.sync_ev, st));
  // spin for the first 0.2 ms (the wake-up latency of a blocking wait is ~0.1 ms, which the
  // short calls would pay in full), then yield, and beyond 20 ms sleep 20 us between polls so
  // long calls (config-5 MSMs, 2^26 transforms) do not pin a host core.  (Round 3 slept from
  // 2 ms on: a 20 us sleep returns after ~50-100 us on the host, which every 2-20 ms call -- the
  // 2^20 MSM, the 2^24 NTT -- paid at its end: BLS12-381 2^20 export phase 0.07 vs 0.02 ms at 2^16.)
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(dev.sync_ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) ZK_CHECK(e);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (us > 20000) std::this_thread::sleep_for(std::chrono::microseconds(20));
    else if (us > 200) std::this_thread::yield();
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
  const std::vector<Device *> devs = all_devices();
  for (Device *d : devs)
    if (d) {
      std::lock_guard<std::mutex> lock(d->mu);
      d->timer.total_ms = 0;
      d->timer.launches = 0;
    }
}

void timer_read_all(double *total_ms, long *launches) {
  const std::vector<Device *> devs = all_devices();
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

// ---------------------------------------------------------------------------
// copy_to_host

void copy_to_host(Device &dev, hipStream_t st, void *dst, const void *src, size_t bytes) {
  constexpr size_t PIECE = (size_t)32 << 20;
  constexpr int THREADS = 8;
  if (bytes < 2 * PIECE) {
    ZK_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    stream_wait(dev, st);
    return;
  }
  if (dev.xfer_cap < 2 * PIECE) {
    if (dev.xfer) ZK_CHECK(hipHostFree(dev.xfer));
    dev.xfer = nullptr;
    ZK_CHECK(hipHostMalloc(&dev.xfer, 2 * PIECE, hipHostMallocDefault));
    dev.xfer_cap = 2 * PIECE;
  }
  for (int j = 0; j < 2; j++)
    if (!dev.xfer_ev[j]) ZK_CHECK(hipEventCreateWithFlags(&dev.xfer_ev[j], hipEventDisableTiming));
  char *stage = static_cast<char *>(dev.xfer);
  const size_t np = (bytes + PIECE - 1) / PIECE;
  auto enqueue = [&](size_t k) {
    const size_t off = k * PIECE, len = std::min(PIECE, bytes - off);
    ZK_CHECK(hipMemcpyAsync(stage + (k & 1) * PIECE, static_cast<const char *>(src) + off, len,
                            hipMemcpyDeviceToHost, st));
    ZK_CHECK(hipEventRecord(dev.xfer_ev[k & 1], st));
  };
  auto drain = [&](size_t k) {  // piece k: staged -> caller memory on THREADS host threads
    const size_t off = k * PIECE, len = std::min(PIECE, bytes - off);
    for (;;) {  // spin (a blocking wait adds ~0.1 ms of wake-up latency per piece)
      const hipError_t e = hipEventQuery(dev.xfer_ev[k & 1]);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) ZK_CHECK(e);
      std::this_thread::yield();
    }
    const char *from = stage + (k & 1) * PIECE;
    char *to = static_cast<char *>(dst) + off;
    const size_t part = (len / THREADS + 63) & ~(size_t)63;
    host_parallel_for(THREADS, [&](int i) {
      const size_t lo = std::min(len, (size_t)i * part), hi = std::min(len, lo + part);
      if (hi > lo) memcpy(to + lo, from + lo, hi - lo);
    });
  };
  enqueue(0);
  for (size_t k = 1; k < np; k++) {
    enqueue(k);     // the DMA of piece k overlaps the host copy of piece k - 1 (the other half)
    drain(k - 1);
  }
  drain(np - 1);
}

}  // namespace zk
