// zk_hostpool.cpp -- persistent host worker pool for the serial-on-GPU tails that split
// into independent pieces (the MSM's per-window Horner segments, zk_msm_impl.hpp).
// Plain C++ (no HIP): tests/native/test_hostpool.cpp builds it with ThreadSanitizer.
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>
#include "zk_hostpool.hpp"

namespace zk {

namespace {
// Persistent host worker pool.  Every run() publishes its own Job (count, function,
// counters) in the active list; workers pick any job with unclaimed indices, so calls
// from several threads (several devices) share the workers instead of queueing behind
// each other.  A job's fields are immutable after publication and the Job object is
// reference-counted, so a worker that wakes late only ever touches a live, complete job
// (its index counter is exhausted, so it never calls a function whose caller returned).
struct Job {
  const std::function<void(int)> *fn;
  int n;
  std::atomic<int> next{0}, done{0};
  Job(const std::function<void(int)> *f, int count) : fn(f), n(count) {}
  bool has_work() const { return next.load(std::memory_order_relaxed) < n; }
  void drain() {
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= n) break;
      (*fn)(i);
      done.fetch_add(1, std::memory_order_release);
    }
  }
};

struct HostPool {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::shared_ptr<Job>> active;  // guarded by mu
  int workers = 0;
  HostPool() {
    unsigned hw = std::thread::hardware_concurrency();
    workers = hw > 2 ? (int)(hw - 1 < 7 ? hw - 1 : 7) : 0;
    for (int i = 0; i < workers; i++) std::thread([this] { loop(); }).detach();
  }
  std::shared_ptr<Job> pick() {  // caller holds mu
    for (auto &j : active)
      if (j->has_work()) return j;
    return nullptr;
  }
  void loop() {
    for (;;) {
      std::shared_ptr<Job> job;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return (job = pick()) != nullptr; });
      }
      job->drain();
    }
  }
  void run(int count, const std::function<void(int)> &f, const std::function<void()> *main_fn = nullptr) {
    auto job = std::make_shared<Job>(&f, count);
    {
      std::lock_guard<std::mutex> lk(mu);
      active.push_back(job);
    }
    cv.notify_all();
    if (main_fn) (*main_fn)();
    job->drain();
    while (job->done.load(std::memory_order_acquire) < count) std::this_thread::yield();
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = 0; i < active.size(); i++)
      if (active[i] == job) {
        active.erase(active.begin() + i);
        break;
      }
  }
};
}  // namespace

static HostPool *shared_pool() {
  static HostPool *pool = new HostPool();  // leaked on purpose: detached workers outlive static teardown
  return pool;
}

void host_parallel_for(int n, const std::function<void(int)> &fn) {
  if (n <= 0) return;
  HostPool *pool = shared_pool();
  if (n == 1 || pool->workers == 0) {
    for (int i = 0; i < n; i++) fn(i);
    return;
  }
  pool->run(n, fn);
}

void host_parallel_for_main(int n, const std::function<void(int)> &fn, const std::function<void()> &main_fn) {
  HostPool *pool = shared_pool();
  if (n <= 0 || pool->workers == 0) {
    for (int i = 0; i < n; i++) fn(i);
    main_fn();
    return;
  }
  pool->run(n, fn, &main_fn);
}

}  // namespace zk
