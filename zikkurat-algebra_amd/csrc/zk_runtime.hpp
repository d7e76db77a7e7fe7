// zk_runtime.hpp -- device context shared by the MSM and NTT paths.
//
// The reference is single-threaded and allocates scratch with malloc per call
// (bls12_381_G1_proj.c:517, poly.c:459).  Here each device keeps one grow-only
// workspace arena and one stream; a per-device mutex makes every C-ABI entry
// point reentrant and thread-safe (SURVEY.md 8b "Threading": Haskell `unsafe`
// ccalls may arrive concurrently from several capabilities).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include "zk_hostpool.hpp"

namespace zk {

// error handling: no error codes cross the reference ABI (void functions), so by default a
// failure on the device path is fatal and loud (the reference asserts) -- never a silent CPU
// fallback.  zkg_set_error_mode(1) makes it recoverable instead: fatal() throws zk::Error, every
// C-ABI entry point catches it (guard / guard_ret below), records the message for the calling
// thread (zkg_last_error) and returns with its outputs unspecified.
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};
[[noreturn]] void fatal(const char *what, const char *file, int line);
void set_error_mode(int mode);  // 0: print and abort (default), 1: throw zk::Error
void record_error(const char *msg);
int take_last_error(char *msg, size_t cap);  // 1 and the message if the thread has one (cleared)
template <class Fn>
inline void guard(Fn &&fn) {
  try {
    fn();
  } catch (const Error &e) {
    record_error(e.what());
  }
}
template <class R, class Fn>
inline R guard_ret(R on_error, Fn &&fn) {
  try {
    return fn();
  } catch (const Error &e) {
    record_error(e.what());
    return on_error;
  }
}
// runs fn on a worker thread's behalf: an Error is kept in *err (first one wins, under *mu)
// instead of escaping the thread; the spawning thread rethrows it after join (rethrow_first)
template <class Fn>
inline void catch_into(std::string *err, std::mutex *mu, Fn &&fn) {
  try {
    fn();
  } catch (const Error &e) {
    std::lock_guard<std::mutex> lock(*mu);
    if (err->empty()) *err = e.what();
  }
}
inline void rethrow_first(const std::string &err) {
  if (!err.empty()) throw Error(err);
}
// joins every thread of `th` when the scope ends (also while an Error unwinds it)
struct JoinAll {
  std::vector<std::thread> &th;
  ~JoinAll() {
    for (auto &t : th)
      if (t.joinable()) t.join();
  }
};
#define ZK_CHECK(x)                                                       \
  do {                                                                    \
    hipError_t e__ = (x);                                                 \
    if (e__ != hipSuccess) {                                              \
      (void)hipGetLastError(); /* not sticky: later hipGetLastError checks stay clean */ \
      ::zk::fatal(hipGetErrorString(e__), __FILE__, __LINE__);            \
    }                                                                     \
  } while (0)
#define ZK_REQUIRE(cond, msg)                                             \
  do {                                                                    \
    if (!(cond)) ::zk::fatal(msg, __FILE__, __LINE__);                    \
  } while (0)

// The calling thread on device `dev` while the guard lives.  The previous device is restored on
// every exit -- also while a zk::Error unwinds the scope (recoverable error mode) -- and the
// destructor never throws: a failed restore is cleared from HIP's last-error state instead.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    ZK_CHECK(hipGetDevice(&prev));
    if (prev != dev) ZK_CHECK(hipSetDevice(dev));
  }
  DeviceGuard(const DeviceGuard &) = delete;
  DeviceGuard &operator=(const DeviceGuard &) = delete;
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != prev)
      if (hipSetDevice(prev) != hipSuccess) (void)hipGetLastError();
  }
};

// Bump allocator over a grow-only device buffer. reset() at the start of every call.
// try_reserve() reports an allocation failure (hipMalloc out of memory, or the test hook's
// cap, arena_set_limit) instead of aborting, so callers can degrade (smaller MSM window
// groups, dropping cached NTT twiddles) before giving up; release() returns the memory.
class Arena {
 public:
  void reserve(size_t bytes);      // try_reserve or fatal
  bool try_reserve(size_t bytes);  // grows (re-allocates) only when larger than current
  void release();                  // frees the buffer (the next reserve re-allocates)
  size_t capacity() const { return cap_; }
  void reset() { off_ = 0; }
  void rewind(size_t off) { off_ = off; }  // release everything taken after used() == off
  template <class T>
  T *take(size_t count) {
    size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
    ZK_REQUIRE(off_ + bytes <= cap_, "zk arena overflow (internal sizing bug)");
    T *p = reinterpret_cast<T *>(base_ + off_);
    off_ += bytes;
    return p;
  }
  size_t used() const { return off_; }
  ~Arena();

 private:
  char *base_ = nullptr;
  size_t cap_ = 0;
  size_t off_ = 0;
};

// Timing probe of the dominant kernel (MSM bucket accumulation / NTT pass chain), used by
// bench.py.  Per device: its events belong to that device and are only touched while the
// device's mutex is held (every MSM / NTT call holds it).
// Two slots (durations added), so a call may time two kernels on different streams.
struct KernelTimer {
  hipEvent_t ev0[2] = {nullptr, nullptr}, ev1[2] = {nullptr, nullptr};
  bool armed[2] = {false, false};  // this call recorded ev0[slot]
  bool counted = false;            // this call contributes one launch
  double total_ms = 0;
  long launches = 0;
};

// test hook: device bytes one arena may hold (0: unlimited), to exercise the degrade paths
void arena_set_limit(size_t bytes);

// One device context: a stream, an arena and pinned staging, guarded by `mu`.  Context
// (id, 0) is the one the C-ABI entry points use on the calling thread's device; contexts
// (id, k > 0) exist when the device set (below) lists device id more than once, so that
// logical shards on one physical device run on streams and arenas of their own.
struct Device {
  int id = 0;    // physical HIP device
  int slot = 0;  // context index on that device
  int uid = 0;   // unique per context (keys per-context caches)
  hipStream_t stream = nullptr;
  Arena arena;
  std::mutex mu;
  // pinned host staging for small D2H results; fine-grained and mapped at the same address on
  // the device, so kernels write their exports into it directly (the MSM's job sums)
  void *pinned = nullptr;
  size_t pinned_cap = 0;
  void *host_staging(size_t bytes);
  // pinned double buffer of the large device-to-host copies into caller memory (copy_to_host)
  void *xfer = nullptr;
  size_t xfer_cap = 0;
  hipEvent_t xfer_ev[2] = {nullptr, nullptr};
  KernelTimer timer;
  hipEvent_t sync_ev = nullptr;  // stream_wait's marker
  // second stream of this context (host-input copies overlapping the first stream's work) and
  // an event to join it; created on first use (aux_stream)
  hipStream_t aux = nullptr;
  hipEvent_t aux_ev = nullptr;
  hipStream_t aux_stream();
  // third stream: the bucket sorts of a split host-input MSM run on it beside the previous
  // split's accumulation (created on first use)
  hipStream_t aux2 = nullptr;
  hipStream_t aux2_stream();
  std::vector<hipEvent_t> split_ev;  // per point split of a host-input MSM (split_event)
  hipEvent_t split_event(int h);
  void release_memory();         // arena + pinned staging (caller holds mu, stream idle)
};

// Copy `bytes` from device memory `src` (ordered after the work on `st`) into CALLER host memory
// `dst` and wait (caller holds dev.mu).  Large copies go through the context's pinned double
// buffer in 32 MiB pieces: the DMA engine fills one half while the host pool copies the other
// into `dst` on 8 threads.  A caller's output array is often FRESH (the Haskell binding allocates
// one per call, Poly.hs:405): through the runtime's pageable path the first touch of its pages
// cost a 2^24 NTT 35-43 ms against 22 ms into resident pages -- the runtime pins the destination
// in place (fault + pin inside the call) and unpins it later -- while 8 host threads fault the
// pages in as they copy (profiles/r05g_*..r05n_*).  Small copies take the plain pageable path.
void copy_to_host(Device &dev, hipStream_t st, void *dst, const void *src, size_t bytes);

// Wait for everything enqueued on st by spinning on an event (caller holds dev.mu): the
// synchronous entry points return as soon as the GPU is done, without the wake-up latency of
// a blocking stream synchronisation (up to ~0.1 ms measured in the MSM's export phase).
void stream_wait(Device &dev, hipStream_t st);

// The device of the calling thread (hipGetDevice), lazily initialised: context (id, 0).
Device &current_device();
// Context (id, slot), created on first use (its stream lives on device id).
Device &device_context(int id, int slot);
// Every context created so far (for zkg_release).
std::vector<Device *> all_devices();

// Device set of the host-buffer MSM entry points: the pairs are split into contiguous
// chunks, one per listed device (a device may be listed more than once: one context per
// occurrence), computed concurrently, and the partial sums added in list order.  Empty or
// one entry: the calling thread's device only.  Initialised from the environment variable
// ZKG_DEVICES ("all", or a comma-separated list of device ids) on first use.
std::vector<int> device_set();
int set_device_set(const int *ids, int n);  // 0 on success, -1 for an invalid id

// kernel timer (caller holds dev.mu for begin/end/collect)
void timer_set_enabled(bool on);
void timer_begin(Device &dev, int slot = 0, hipStream_t st = nullptr);  // records ev0 (slot < 0: no-op)
void timer_end(Device &dev, int slot = 0, hipStream_t st = nullptr);    // records ev1
void timer_collect(Device &dev);  // after the streams are synchronised: accumulate the armed slots
void timer_reset_all();
void timer_read_all(double *total_ms, long *launches);

inline unsigned div_up(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

}  // namespace zk
