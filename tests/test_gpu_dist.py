"""The multi-GPU MSM path of bench.py (config 5 shape: contiguous shards, all-gather of the
partial sums, rank-ordered adds) with the PRODUCT kernel on every rank: 2 ranks share the
one GPU of the test box and exchange over gloo (the 8-GPU RCCL run is the driver's).  The
sharded affine result must equal the single-call MSM of the whole input bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
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
    from sharded import shard_range

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist = bench.Dist(SimpleNamespace(backend="gloo"), device=0)
    zk.load().zkg_set_device(0)
    lo, hi = shard_range(n_total, rank, world)
    sc = zk.gen_fr(curve, 0x5A4B0005, hi - lo, start=lo)
    pts = zk.gen_points(curve, 0x5A4B0005, hi - lo, start=lo)
    d_s, d_p = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
    aff = bench.sharded_msm_step(zk, curve, hi - lo, d_s, d_p, 0, dist)
    d_s.free()
    d_p.free()
    q.put((rank, aff.tolist()))
    dist.close()


@pytest.mark.parametrize("curve", ["bn128", "bls12_381"])
def test_sharded_msm_two_ranks_one_gpu(gpu, curve):
    import multiprocessing as mp  # plain spawn: the parent (pytest) process never loads torch
    world, n_total = 2, (1 << 16) + 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, curve, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = gpu.msm_affine(curve, gpu.gen_fr(curve, 0x5A4B0005, n_total), gpu.gen_points(curve, 0x5A4B0005, n_total))
    for rank, aff in res:
        assert np.array_equal(np.array(aff, dtype=np.uint64), want), rank
