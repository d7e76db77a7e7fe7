// zk_comm.cpp -- the library's own multi-GPU exchange: one RCCL communicator per process (one
// process per GPU), and the device-resident sharded MSM built on it.
//
// The reference computes an MSM with one synchronous call on one CPU
// (bls12_381_G1_proj.c:630-644).  An MSM is a group sum, so it partitions exactly: rank r owns a
// contiguous chunk of the pairs in its own HBM, computes the partial sum S_r on its GPU, and the
// partials (3 NP u64 each: 96 / 144 B) are all-gathered with ncclAllGather on the library's own
// stream -- over xGMI between the GPUs of a node -- and added on every rank in (rank, shard)
// order.  RCCL has no elliptic-curve reduction operator, so "reduce" = all-gather + local adds;
// the payload is a few hundred bytes, so the exchange is latency-bound (one collective per MSM).
//
// Everything runs on the HIP runtime this library links (/opt/rocm): no torch, no second
// runtime in the process.  The rendezvous (sharing the 128-byte unique id) is the caller's: rank
// 0 calls zkg_comm_unique_id, every rank passes the id to zkg_comm_init.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>
#include <unistd.h>
#include <mutex>
#include <string>
#include <vector>
#include "../../include/zkalgebra_gpu.h"
#include "zk_host.hpp"
#include "zk_msm.hpp"
#include "zk_runtime.hpp"

using namespace zk;

static_assert(ZKG_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

namespace {

struct Comm {
  std::mutex mu;
  ncclComm_t comm = nullptr;
  int rank = 0, world = 0, device = -1;
  // device staging of the exchanged payloads (grown on demand, freed by zkg_comm_destroy)
  void *d_send = nullptr, *d_recv = nullptr;
  size_t cap_send = 0, cap_recv = 0;
};
Comm g_comm;

int report(const char *what, ncclResult_t r) {
  fprintf(stderr, "[zkalgebra_gpu] %s: %s\n", what, ncclGetErrorString(r));
  fflush(stderr);
  return (int)r;
}
#define ZK_NCCL(what, x)                         \
  do {                                           \
    ncclResult_t r__ = (x);                      \
    if (r__ != ncclSuccess) return report(what, r__); \
  } while (0)

void grow(void *&p, size_t &cap, size_t bytes) {
  if (bytes <= cap) return;
  if (p) ZK_CHECK(hipFree(p));
  ZK_CHECK(hipMalloc(&p, bytes));
  cap = bytes;
}

// RCCL prints a version banner on stdout when it initialises; the caller's stdout is not ours
// (bench.py's contract is one JSON line there), so stdout points at stderr while RCCL sets up
struct StdoutToStderr {
  int saved = -1;
  StdoutToStderr() {
    fflush(stdout);
    saved = dup(1);
    if (saved >= 0) dup2(2, 1);
  }
  ~StdoutToStderr() {
    fflush(stdout);
    if (saved >= 0) {
      dup2(saved, 1);
      close(saved);
    }
  }
};

// ncclAllGather of `bytes` per rank from host `send` into host `recv` (world * bytes), through
// device staging on the communicator device's library stream.  Caller holds g_comm.mu.
int allgather_host(const void *send, void *recv, size_t bytes) {
  DeviceGuard on(g_comm.device);
  Device &dev = current_device();
  std::lock_guard<std::mutex> lock(dev.mu);
  grow(g_comm.d_send, g_comm.cap_send, bytes);
  grow(g_comm.d_recv, g_comm.cap_recv, bytes * (size_t)g_comm.world);
  ZK_CHECK(hipMemcpyAsync(g_comm.d_send, send, bytes, hipMemcpyHostToDevice, dev.stream));
  ZK_NCCL("ncclAllGather", ncclAllGather(g_comm.d_send, g_comm.d_recv, bytes, ncclUint8, g_comm.comm, dev.stream));
  ZK_CHECK(hipMemcpyAsync(recv, g_comm.d_recv, bytes * (size_t)g_comm.world, hipMemcpyDeviceToHost, dev.stream));
  stream_wait(dev, dev.stream);
  return 0;
}

// rank-ordered sum of `count` projective partials (3 NP u64 each, reference Montgomery form),
// normalised
template <class C>
void sum_partials(const uint64_t *parts, int count, uint64_t *out) {
  using HF = typename HostOf<C>::Fp;
  constexpr int NP = C::NP64;
  zkh::Fe<HF> b3;
  HostOf<C>::b3(b3);
  zkh::Proj<HF> acc, p, r;
  memcpy(acc.X.v, parts, NP * 8);
  memcpy(acc.Y.v, parts + NP, NP * 8);
  memcpy(acc.Z.v, parts + 2 * NP, NP * 8);
  for (int k = 1; k < count; k++) {
    const uint64_t *q = parts + (size_t)k * 3 * NP;
    memcpy(p.X.v, q, NP * 8);
    memcpy(p.Y.v, q + NP, NP * 8);
    memcpy(p.Z.v, q + 2 * NP, NP * 8);
    zkh::proj_add(r, acc, p, b3);
    acc = r;
  }
  zkh::proj_normalize(r, acc);
  memcpy(out, r.X.v, NP * 8);
  memcpy(out + NP, r.Y.v, NP * 8);
  memcpy(out + 2 * NP, r.Z.v, NP * 8);
}

template <class C>
int sharded_msm(int n, const uint64_t *d_expos, int nl, bool mont, const uint64_t *d_grps, int window, int shards,
                uint64_t *tgt) {
  constexpr int NP = C::NP64;
  // payload per rank: the `shards` partials and one status word (non-zero: this rank's chunk
  // failed).  A rank whose chunk MSM throws (recoverable error mode, e.g. out of device memory)
  // still takes part in the all-gather, so its peers are not left waiting in the collective; then
  // every rank returns an error.
  const size_t per = (size_t)shards * 3 * NP + 1;
  std::vector<uint64_t> mine(per, 0), all(per * (size_t)g_comm.world);
  std::string local_err;
  try {
    DeviceGuard on(g_comm.device);
    for (int k = 0; k < shards; k++) {  // the rank's chunk as `shards` contiguous sub-chunks
      const size_t lo = (size_t)n * k / shards, hi = (size_t)n * (k + 1) / shards;
      msm_g1<C>((int)(hi - lo), d_expos + lo * nl, nl, d_grps + lo * 2 * NP, /*host_inputs=*/false, mont, window,
                mine.data() + (size_t)k * 3 * NP);
    }
  } catch (const std::exception &e) {  // zk::Error, and std::bad_alloc etc. from the host side: every
    local_err = e.what();               // rank still joins the all-gather
    mine[per - 1] = 1;
  } catch (...) {
    local_err = "zkg_g1_msm_device_sharded: unknown exception in the chunk MSM";
    mine[per - 1] = 1;
  }
  if (int e = allgather_host(mine.data(), all.data(), per * 8)) return e;
  for (int r = 0; r < g_comm.world; r++)
    if (all[(size_t)r * per + per - 1]) {
      if (!local_err.empty()) throw Error(local_err);
      throw Error("zkg_g1_msm_device_sharded: rank " + std::to_string(r) + " failed its chunk MSM");
    }
  std::vector<uint64_t> parts((size_t)shards * g_comm.world * 3 * NP);
  for (int r = 0; r < g_comm.world; r++)
    memcpy(parts.data() + (size_t)r * shards * 3 * NP, all.data() + (size_t)r * per, (size_t)shards * 3 * NP * 8);
  sum_partials<C>(parts.data(), shards * g_comm.world, tgt);
  return 0;
}

}  // namespace

extern "C" {

ZKG_API int zkg_comm_unique_id(void *out) {
  return guard_ret(-3, [&]() -> int {
  ncclUniqueId id;
  StdoutToStderr quiet;
  ZK_NCCL("ncclGetUniqueId", ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof id);
  return 0;
  });
}

ZKG_API int zkg_comm_init(int rank, int world, const void *unique_id) {
  return guard_ret(-3, [&]() -> int {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  if (g_comm.comm) {
    fprintf(stderr, "[zkalgebra_gpu] zkg_comm_init: a communicator already exists (zkg_comm_destroy first)\n");
    return -1;
  }
  if (world < 1 || rank < 0 || rank >= world || !unique_id) {
    fprintf(stderr, "[zkalgebra_gpu] zkg_comm_init: invalid rank %d / world %d\n", rank, world);
    return -1;
  }
  int dev = 0;
  ZK_CHECK(hipGetDevice(&dev));
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof id);
  ncclComm_t c = nullptr;
  {
    StdoutToStderr quiet;
    ZK_NCCL("ncclCommInitRank", ncclCommInitRank(&c, world, id, rank));
  }
  g_comm.comm = c;
  g_comm.rank = rank;
  g_comm.world = world;
  g_comm.device = dev;
  // first collective: RCCL connects its channels lazily, so one tiny all-gather here keeps that
  // setup out of the first timed exchange
  uint64_t one = (uint64_t)rank;
  std::vector<uint64_t> every((size_t)world);
  if (int e = allgather_host(&one, every.data(), 8)) return e;
  for (int r = 0; r < world; r++)
    if (every[r] != (uint64_t)r) {
      fprintf(stderr, "[zkalgebra_gpu] zkg_comm_init: all-gather check failed at rank %d\n", r);
      return -2;
    }
  return 0;
  });
}

ZKG_API int zkg_comm_destroy(void) {
  return guard_ret(-3, [&]() -> int {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  if (!g_comm.comm) return 0;
  DeviceGuard on(g_comm.device);
  {
    Device &dev = current_device();
    std::lock_guard<std::mutex> dlock(dev.mu);
    ZK_CHECK(hipStreamSynchronize(dev.stream));
  }
  const ncclResult_t r = ncclCommDestroy(g_comm.comm);
  g_comm.comm = nullptr;
  if (g_comm.d_send) ZK_CHECK(hipFree(g_comm.d_send));
  if (g_comm.d_recv) ZK_CHECK(hipFree(g_comm.d_recv));
  g_comm.d_send = g_comm.d_recv = nullptr;
  g_comm.cap_send = g_comm.cap_recv = 0;
  g_comm.world = 0;
  g_comm.device = -1;
  if (r != ncclSuccess) return report("ncclCommDestroy", r);
  return 0;
  });
}

ZKG_API int zkg_comm_rank(void) {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  return g_comm.comm ? g_comm.rank : -1;
}

ZKG_API int zkg_comm_world(void) {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  return g_comm.comm ? g_comm.world : 0;
}

ZKG_API int zkg_comm_allgather(const void *send, void *recv, size_t bytes) {
  return guard_ret(-3, [&]() -> int {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  if (!g_comm.comm) return -1;
  return allgather_host(send, recv, bytes);
  });
}

ZKG_API int zkg_comm_barrier(void) {
  return guard_ret(-3, [&]() -> int {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  if (!g_comm.comm) return -1;
  std::vector<uint8_t> all((size_t)g_comm.world);
  uint8_t one = 1;
  return allgather_host(&one, all.data(), 1);
  });
}

ZKG_API int zkg_comm_max_f64(double *x) {
  return guard_ret(-3, [&]() -> int {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  if (!g_comm.comm) return -1;
  std::vector<double> all((size_t)g_comm.world);
  if (int e = allgather_host(x, all.data(), sizeof(double))) return e;
  for (double v : all)
    if (v > *x) *x = v;
  return 0;
  });
}

ZKG_API int zkg_g1_comm_sum_partials(int curve, const uint64_t *partials, int count, uint64_t *tgt_proj) {
  return guard_ret(-3, [&]() -> int {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  if (!g_comm.comm || count < 1) return -1;
  const int NP = curve == ZKG_BN128 ? BN254::NP64 : BLS381::NP64;
  const size_t bytes = (size_t)count * 3 * NP * 8;
  std::vector<uint64_t> all((size_t)count * g_comm.world * 3 * NP);
  if (int e = allgather_host(partials, all.data(), bytes)) return e;
  if (curve == ZKG_BN128) sum_partials<BN254>(all.data(), count * g_comm.world, tgt_proj);
  else sum_partials<BLS381>(all.data(), count * g_comm.world, tgt_proj);
  return 0;
  });
}

ZKG_API int zkg_g1_msm_device_sharded(int curve, int npoints_local, const uint64_t *d_expos, int expo_nlimbs,
                                      int expos_mont, const uint64_t *d_grps, int window_size, int local_shards,
                                      uint64_t *tgt_proj) {
  return guard_ret(-3, [&]() -> int {
  std::lock_guard<std::mutex> lock(g_comm.mu);
  if (!g_comm.comm || local_shards < 1 || npoints_local < 0 || expo_nlimbs < 1) return -1;
  const int c = window_size <= 0 ? 0 : (window_size < 4 ? 4 : (window_size > 24 ? 24 : window_size));
  if (curve == ZKG_BN128)
    return sharded_msm<BN254>(npoints_local, d_expos, expo_nlimbs, expos_mont != 0, d_grps, c, local_shards, tgt_proj);
  return sharded_msm<BLS381>(npoints_local, d_expos, expo_nlimbs, expos_mont != 0, d_grps, c, local_shards, tgt_proj);
  });
}

}  // extern "C"
