// Stress test of the host worker pool (zikkurat-algebra_amd/csrc/zk_hostpool.cpp), built
// with -fsanitize=thread by tests/test_native.py: several caller threads (as several
// devices / Haskell capabilities would) run jobs of different sizes concurrently and
// back to back; every index must run exactly once per job and every job must see its
// own function; host_parallel_for_main's caller-side consumer must see every result.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>
#include "zk_hostpool.hpp"

int main() {
  const int callers = 4, rounds = 300;
  std::atomic<int> failures{0};
  std::vector<std::thread> th;
  for (int t = 0; t < callers; t++) {
    th.emplace_back([t, &failures] {
      for (int r = 0; r < rounds; r++) {
        const int n = 1 + (r * 7 + t * 13) % 37;  // sizes change call to call
        std::vector<std::atomic<int>> hit(n);
        for (auto &h : hit) h.store(0);
        const int tag = t * 100000 + r;
        std::atomic<int> wrong{0};
        zk::host_parallel_for(n, [&, tag](int i) {
          if (tag != t * 100000 + r) wrong++;
          hit[i].fetch_add(1);
        });
        for (int i = 0; i < n; i++)
          if (hit[i].load() != 1) failures++;
        if (wrong.load()) failures++;
        // the pipelined form: the caller's main function consumes results while the workers
        // produce them (the MSM's host Horner chain)
        std::vector<std::atomic<int>> ready(n);
        std::vector<int> val(n, 0);
        for (auto &x : ready) x.store(0);
        long sum = 0;
        zk::host_parallel_for_main(
            n,
            [&](int i) {
              val[i] = i + tag;
              ready[i].store(1, std::memory_order_release);
            },
            [&] {
              for (int i = n - 1; i >= 0; i--) {
                while (!ready[i].load(std::memory_order_acquire)) std::this_thread::yield();
                sum += val[i];
              }
            });
        if (sum != (long)n * tag + (long)n * (n - 1) / 2) failures++;
      }
    });
  }
  for (auto &x : th) x.join();
  if (failures.load()) {
    std::printf("FAIL %d\n", failures.load());
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
