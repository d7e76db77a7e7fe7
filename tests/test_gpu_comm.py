"""The library's own multi-GPU exchange (zk_comm.cpp: RCCL from /opt/rocm, linked by the
library) on the one-GPU box: a world-1 communicator, so every collective runs through RCCL for
real (RCCL refuses two ranks on one device).  The config-5 test sends the 8 shard partials of
BASELINE configs[4] through ncclAllGather (zkg_g1_msm_device_sharded with 8 local shards) and
checks the affine sum against the reference's own output for that config.  Reference entry being
sharded: bls12_381_G1_proj.c:630-644."""
import numpy as np
import pytest

from golden_io import baseline_configs

pytestmark = pytest.mark.gpu
CURVES = ["bn128", "bls12_381"]


def test_comm_world1_collectives(gpu, comm):
    lib = gpu.load()
    assert lib.zkg_comm_world() == 1 and lib.zkg_comm_rank() == 0
    comm.barrier()
    assert comm.max(3.25) == 3.25
    x = np.arange(37, dtype=np.uint8)
    got = comm.allgather(x)
    assert got.shape == (1, 37) and np.array_equal(got[0], x)


@pytest.mark.parametrize("curve", CURVES)
def test_comm_sum_partials_rank_order(gpu, comm, oracle, curve):
    """the exchange + rank-ordered sum of the library (zkg_g1_comm_sum_partials) equals the host
    sum of the same partials"""
    n = 3000
    sc = gpu.gen_fr(curve, 0x61, n)
    pts = gpu.gen_points(curve, 0x62, n)
    parts = [gpu.msm(curve, sc[k * 500:(k + 1) * 500].copy(), pts[k * 500:(k + 1) * 500].copy()) for k in range(6)]
    got = comm.sum_partials(curve, np.stack(parts))
    want = oracle.normalize(curve, oracle.msm(curve, sc, pts, mont=True, out="proj"))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("shards", [1, 3, 8])
def test_msm_device_sharded_vs_oracle(gpu, comm, oracle, curve, shards):
    n = (1 << 14) + 5  # uneven sub-chunks
    sc = gpu.gen_fr(curve, 0x63 + shards, n)
    pts = gpu.gen_points(curve, 0x64 + shards, n)
    d_s, d_p = gpu.DeviceBuffer(sc), gpu.DeviceBuffer(pts)
    try:
        got = comm.msm_device_sharded(curve, n, d_s, d_p, local_shards=shards)
    finally:
        d_s.free()
        d_p.free()
    assert np.array_equal(gpu.g1_to_affine(curve, got), oracle.msm(curve, sc, pts, mont=True))


def test_msm_device_sharded_empty_and_misuse(gpu, comm):
    curve = "bls12_381"
    d = gpu.DeviceBuffer.empty(64)
    try:
        got = comm.msm_device_sharded(curve, 0, d, d, local_shards=4)
        assert np.all(gpu.g1_to_affine(curve, got) == np.uint64(0xFFFFFFFFFFFFFFFF))  # infinity
        with pytest.raises(RuntimeError):
            comm.msm_device_sharded(curve, 1, d, d, local_shards=0)
    finally:
        d.free()


def test_config5_eight_partials_through_rccl_vs_reference(gpu, comm):
    """BASELINE config 5 (2^26 pairs): the 8 shard partials of the 8-GPU split all-gathered by
    ncclAllGather on a world-1 communicator and summed in shard order == the reference's output"""
    cfg = baseline_configs()["config5_bls12_381_msm_2^26"]
    curve = "bls12_381"
    n = 1 << cfg["log_n"]
    d_s = gpu.DeviceBuffer(gpu.gen_fr(curve, cfg["seed"], n))
    d_p = gpu.DeviceBuffer(gpu.gen_points(curve, cfg["seed"], n))
    try:
        got = comm.msm_device_sharded(curve, n, d_s, d_p, local_shards=8)
        assert [int(x) for x in gpu.g1_to_affine(curve, got)] == cfg["affine"]
        got1 = comm.msm_device_sharded(curve, n, d_s, d_p, local_shards=1)
        assert np.array_equal(got1, got)
    finally:
        d_s.free()
        d_p.free()
