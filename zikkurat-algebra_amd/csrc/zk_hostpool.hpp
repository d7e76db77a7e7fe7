// zk_hostpool.hpp -- host thread pool (zk_hostpool.cpp)
#pragma once
#include <functional>

namespace zk {

// Runs fn(0..n-1) on a small persistent host thread pool and returns when all are done.
// The calling thread works too.  Thread-safe: concurrent calls (several devices, several
// caller threads) share the workers.
void host_parallel_for(int n, const std::function<void(int)> &fn);

}  // namespace zk
