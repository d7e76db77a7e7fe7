// zk_runtime.cpp -- per-device context: stream, grow-only arena, pinned staging.
#include "zk_runtime.hpp"
#include <atomic>
#include <condition_variable>
#include <thread>

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

namespace {
struct HostPool {
  std::mutex run_mu;  // one job at a time
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  const std::function<void(int)> *fn = nullptr;
  int n = 0;
  std::atomic<int> next{0}, done{0};
  int workers = 0;
  HostPool() {
    unsigned hw = std::thread::hardware_concurrency();
    workers = hw > 2 ? (int)(hw - 1 < 7 ? hw - 1 : 7) : 0;
    for (int i = 0; i < workers; i++) std::thread([this] { loop(); }).detach();
  }
  void drain() {
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= n) break;
      (*fn)(i);
      done.fetch_add(1);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return gen != seen; });
        seen = gen;
      }
      drain();
    }
  }
  void run(int count, const std::function<void(int)> &f) {
    std::lock_guard<std::mutex> g(run_mu);
    {
      std::lock_guard<std::mutex> lk(mu);
      fn = &f;
      n = count;
      next = 0;
      done = 0;
      gen++;
    }
    cv.notify_all();
    drain();
    while (done.load() < count) std::this_thread::yield();
    std::lock_guard<std::mutex> lk(mu);
    n = 0;  // late-waking workers find nothing to do
  }
};
}  // namespace

void host_parallel_for(int n, const std::function<void(int)> &fn) {
  if (n <= 0) return;
  static HostPool *pool = new HostPool();  // leaked on purpose: detached workers outlive static teardown
  if (n == 1 || pool->workers == 0) {
    for (int i = 0; i < n; i++) fn(i);
    return;
  }
  pool->run(n, fn);
}

KernelTimer &dominant_timer() {
  static KernelTimer t;
  return t;
}

}  // namespace zk
