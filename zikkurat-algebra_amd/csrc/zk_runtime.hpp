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
#include <functional>
#include <mutex>
#include <string>
#include <vector>

namespace zk {

// error handling: no error codes cross the reference ABI (void functions), so a
// failure on the device path is fatal and loud -- never a silent CPU fallback.
[[noreturn]] void fatal(const char *what, const char *file, int line);
#define ZK_CHECK(x)                                                       \
  do {                                                                    \
    hipError_t e__ = (x);                                                 \
    if (e__ != hipSuccess) ::zk::fatal(hipGetErrorString(e__), __FILE__, __LINE__); \
  } while (0)
#define ZK_REQUIRE(cond, msg)                                             \
  do {                                                                    \
    if (!(cond)) ::zk::fatal(msg, __FILE__, __LINE__);                    \
  } while (0)

// Bump allocator over a grow-only device buffer. reset() at the start of every call.
class Arena {
 public:
  void reserve(size_t bytes);  // grows (re-allocates) only when larger than current
  void reset() { off_ = 0; }
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

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  Arena arena;
  std::mutex mu;
  // pinned host staging for small D2H results
  void *pinned = nullptr;
  size_t pinned_cap = 0;
  void *host_staging(size_t bytes);
};

// The device of the calling thread (hipGetDevice), lazily initialised.
Device &current_device();

// simple kernel timing probe used by bench.py: the last launch of the named
// "dominant" kernel family records its duration here (ms) when enabled.
struct KernelTimer {
  bool enabled = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double total_ms = 0;
  long launches = 0;
};
KernelTimer &dominant_timer();

// Small persistent host thread pool for the serial-on-GPU tails that split into
// independent pieces (e.g. the MSM's per-window Horner segments).  run() is
// synchronous; the calling thread works too.  Calls from several threads serialise.
void host_parallel_for(int n, const std::function<void(int)> &fn);

inline unsigned div_up(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

}  // namespace zk
