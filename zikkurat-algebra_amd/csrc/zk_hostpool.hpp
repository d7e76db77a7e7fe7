// zk_hostpool.hpp -- host thread pool (zk_hostpool.cpp)
#pragma once
#include <functional>

namespace zk {

// Runs fn(0..n-1) on a small persistent host thread pool and returns when all are done.
// The calling thread works too.  Thread-safe: concurrent calls (several devices, several
// caller threads) share the workers.
void host_parallel_for(int n, const std::function<void(int)> &fn);

// Runs fn(0..n-1) on the workers (indices claimed in increasing order) WHILE the calling
// thread runs main_fn, then helps with what is left and returns when all are done.
// main_fn may wait for results of fn (every claimed index runs to completion on a worker,
// workers never block).  Without workers fn(0..n-1) run first, then main_fn.
void host_parallel_for_main(int n, const std::function<void(int)> &fn, const std::function<void()> &main_fn);

}  // namespace zk
