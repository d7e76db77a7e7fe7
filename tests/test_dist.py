"""Multi-rank MSM path on CPU: world_size 2 (and 4) over gloo, through bench.py's own
config-5 code path (bench.Dist + bench.sharded_msm_step + sharded.shard_range).

Each rank computes the partial MSM of its contiguous shard (here the oracle is injected in
place of the per-GPU kernel, the only GPU-bound piece -- the kernel itself is covered by the
-m gpu tests, including tests/test_gpu_dist.py which runs this path on the GPU), the
partials are exchanged with the same all-gather bench.py uses over RCCL, and every rank
combines them in rank order with the library's host-side point addition.  The result must
equal the unsharded MSM bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, curve, n_total, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
    from types import SimpleNamespace

    import bench
    import zkalgebra as zk
    from oracle.oracle import Oracle
    from sharded import allgather_partials, combine_partials, shard_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist = bench.Dist(SimpleNamespace(backend="gloo"), device=0)
    assert (dist.rank, dist.world) == (rank, world)
    lo, hi = shard_range(n_total, rank, world)
    sc = zk.gen_fr(curve, 0x5A4B0005, hi - lo, start=lo)
    pts = zk.gen_points(curve, 0x5A4B0005, hi - lo, start=lo)
    partial = Oracle().msm(curve, sc, pts, mont=True, out="proj")
    aff = bench.sharded_msm_step(zk, curve, hi - lo, None, None, 0, dist, msm_fn=lambda: partial)
    proj, aff2 = combine_partials(curve, allgather_partials(partial))
    assert (aff == aff2).all()
    q.put((rank, aff.tolist(), proj.tolist()))
    dist.close()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_sharded_msm_gloo(oracle, zk, curve, world):
    import multiprocessing as mp  # plain spawn: the parent (pytest) process never loads torch
    n_total = 3000 + world  # uneven split exercises shard_range
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, curve, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sc = zk.gen_fr(curve, 0x5A4B0005, n_total)
    pts = zk.gen_points(curve, 0x5A4B0005, n_total)
    want_aff = oracle.msm(curve, sc, pts, mont=True)
    want_proj = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=True, out="proj"))
    for rank, aff, proj in res:
        assert np.array_equal(np.array(aff, dtype=np.uint64), want_aff), rank
        assert np.array_equal(np.array(proj, dtype=np.uint64), want_proj), rank


def test_shard_range_partition():
    sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
    from sharded import shard_range
    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
@pytest.mark.parametrize("G,n", [(2, 1000), (3, 1001), (8, 1003), (8, 5)])
def test_library_shard_combine_order(oracle, zk, curve, G, n):
    """the split the library's device set uses behind the reference symbols (zk_msm_impl.hpp
    msm_g1: chunk k = [n k / G, n (k+1) / G), partial sums added in list order, empty chunks
    skipped) reproduces the unsplit MSM bit for bit -- checked with the oracle on the CPU"""
    sc = zk.gen_fr(curve, 0x77 + n, n)
    pts = zk.gen_points(curve, 0x78 + n, n)
    acc = None
    for k in range(G):
        lo, hi = n * k // G, n * (k + 1) // G
        if hi == lo:
            continue
        part = oracle.msm(curve, sc[lo:hi].copy(), pts[lo:hi].copy(), mont=True, out="proj")
        acc = part if acc is None else oracle.proj_add(curve, acc, part)
    assert np.array_equal(oracle.to_affine(curve, acc), oracle.msm(curve, sc, pts, mont=True))
