// zk_runtime.cpp -- per-device context: stream, grow-only arena, pinned staging.
#include "zk_runtime.hpp"
#include <sys/mman.h>
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
// HostPrefault

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23  // Linux 5.14
#endif

static void prefault_range(char *lo, char *hi) {
  const uintptr_t pg = 4096;
  char *a = (char *)((uintptr_t)lo & ~(pg - 1));
  if (madvise(a, (size_t)(hi - a), MADV_POPULATE_WRITE) == 0) return;
  // no MADV_POPULATE_WRITE: touch every page of the range, writing back the value read
  for (char *p = lo; p < hi; p = (char *)(((uintptr_t)p + pg) & ~(pg - 1))) {
    volatile char *v = p;
    *v = *v;
  }
}

bool HostPrefault::enabled() {
  static const bool on = [] {
    const char *e = getenv("ZK_PREFAULT");
    return !(e && e[0] == '0');
  }();
  return on;
}

void HostPrefault::start(void *ptr, size_t bytes, int threads) {
  join();
  if (!ptr || !bytes || threads < 1 || !enabled()) return;
  char *base = static_cast<char *>(ptr);
  // transparent huge pages for the 2 MiB-aligned interior (a hint: fewer, larger page faults)
  const uintptr_t huge = (uintptr_t)2 << 20;
  const uintptr_t h0 = ((uintptr_t)base + huge - 1) & ~(huge - 1), h1 = ((uintptr_t)base + bytes) & ~(huge - 1);
  if (h1 > h0) (void)madvise((void *)h0, h1 - h0, MADV_HUGEPAGE);
  const size_t piece = ((bytes + threads - 1) / threads + huge - 1) & ~(size_t)(huge - 1);
  for (size_t off = 0; off < bytes; off += piece) {
    char *lo = base + off, *hi = base + std::min(bytes, off + piece);
    th_.emplace_back([lo, hi] { prefault_range(lo, hi); });
  }
}

void HostPrefault::join() {
  for (auto &t : th_)
    if (t.joinable()) t.join();
  th_.clear();
}

}  // namespace zk
