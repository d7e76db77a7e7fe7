"""The multi-GPU bench's rendezvous on the CPU: sharded.LibComm hands the RCCL unique id from
rank 0 to the other ranks through a file (no torch, no TCP store), then every rank calls
zkg_comm_init with it.  Here the library's zkg_comm_* entry points are replaced by a recording
stand-in (the real ones need a GPU; tests/test_gpu_comm.py runs them on the GPU box), so the test
checks exactly the Python protocol bench.py --gpus N uses: one id per launch, seen by every rank,
the file removed afterwards, and launches with different keys kept apart."""
import ctypes
import multiprocessing as mp
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakeLib:
    """stand-in for the library's zkg_comm_*: init is collective like ncclCommInitRank (it returns
    only once every rank of the launch has called it), so rank 0 may then remove the id file"""

    def __init__(self, key, rdir):
        self.key, self.rdir = key, rdir
        self.got = None

    def zkg_comm_unique_id(self, buf):
        ctypes.memmove(buf, os.urandom(128), 128)
        return 0

    def zkg_comm_init(self, rank, world, buf):
        self.got = (rank, world, bytes(buf.raw[:128]))
        open(os.path.join(self.rdir, f"joined_{self.key}_{rank}"), "w").close()
        t0 = time.time()
        while sum(os.path.exists(os.path.join(self.rdir, f"joined_{self.key}_{r}")) for r in range(world)) < world:
            if time.time() - t0 > 60:
                return -1
            time.sleep(0.01)
        return 0

    def zkg_comm_destroy(self):
        return 0


def _rank(rank, world, key, rdir, q, nonce=None, env=None):
    sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
    os.environ["ZKG_RDZV_KEY"] = key
    os.environ["ZKG_RDZV_DIR"] = rdir
    os.environ.update(env or {})
    if nonce:
        os.environ["ZKG_RDZV_NONCE"] = nonce
    import sharded
    fake = _FakeLib(key, rdir)
    sharded.zk.load = lambda: fake
    c = sharded.LibComm(rank, world, timeout=60)
    c.close()
    q.put((key, fake.got))


@pytest.mark.parametrize("world", [2, 4])
def test_file_rendezvous_one_id_per_launch(tmp_path, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    keys = ["launchA", "launchB"]  # two concurrent launches must not mix their ids
    procs = [ctx.Process(target=_rank, args=(r, world, k, str(tmp_path), q)) for k in keys for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in keys:
        got = [g for kk, g in res if kk == k]
        assert sorted(g[0] for g in got) == list(range(world))
        assert all(g[1] == world for g in got)
        assert len({g[2] for g in got}) == 1  # every rank of the launch holds rank 0's id
    ids = {g[2] for _, g in res}
    assert len(ids) == 2
    time.sleep(0.2)
    assert not [f for f in os.listdir(tmp_path) if f.startswith("zkg_rdzv_")]  # removed by rank 0


def test_rendezvous_path_default_key(monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
    import sharded
    monkeypatch.delenv("ZKG_RDZV_KEY", raising=False)
    monkeypatch.delenv("ZKG_RDZV_DIR", raising=False)
    monkeypatch.setenv("MASTER_PORT", "29517")
    p = sharded.rendezvous_path()
    assert p.endswith(f"zkg_rdzv_{os.getppid()}_29517.id")


def test_stale_id_of_an_earlier_launch_is_ignored(tmp_path):
    """an id file left by an earlier launch with the same key (e.g. its rank 0 died) carries that
    launch's nonce: a rank of the new launch that starts before the new rank 0 must wait for the
    new id instead of joining the dead launch's communicator"""
    key, stale = "launchS", os.urandom(128)
    (tmp_path / f"zkg_rdzv_{key}.id").write_bytes(stale + b"old-launch")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    r1 = ctx.Process(target=_rank, args=(1, 2, key, str(tmp_path), q, "new-launch"))
    r1.start()
    time.sleep(1.0)  # rank 1 polls the stale file first
    r0 = ctx.Process(target=_rank, args=(0, 2, key, str(tmp_path), q, "new-launch"))
    r0.start()
    got = [q.get(timeout=120)[1] for _ in range(2)]
    for p in (r0, r1):
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][2] == got[1][2] != stale
    assert not (tmp_path / f"zkg_rdzv_{key}.id").exists()


def test_rank0_failed_init_removes_its_id(tmp_path, monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
    import sharded
    monkeypatch.setenv("ZKG_RDZV_KEY", "launchF")
    monkeypatch.setenv("ZKG_RDZV_DIR", str(tmp_path))
    fake = _FakeLib("launchF", str(tmp_path))
    fake.zkg_comm_init = lambda rank, world, buf: -1
    monkeypatch.setattr(sharded.zk, "load", lambda: fake)
    with pytest.raises(RuntimeError, match="zkg_comm_init"):
        sharded.LibComm(0, 2, timeout=5)
    assert not (tmp_path / "zkg_rdzv_launchF.id").exists()


def test_multi_rank_without_torchrun_or_key_fails_fast(monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
    import sharded
    for k in ("ZKG_RDZV_KEY", "TORCHELASTIC_RUN_ID"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(RuntimeError, match="ZKG_RDZV_KEY"):
        sharded.rendezvous_path()


def _agent(rank, world, key, rdir, q, env):
    """one node's elastic agent: its rank is its child, so every rank has a different parent pid"""
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_rank, args=(rank, world, key, rdir, q, None, env))
    p.start()
    p.join(timeout=120)
    sys.exit(p.exitcode or 0)


def test_torchrun_nonce_is_the_same_on_every_node(tmp_path):
    """multi-node torchrun: ZKG_RDZV_KEY + a shared ZKG_RDZV_DIR, no ZKG_RDZV_NONCE, each rank the
    child of its own agent (different parent pids): the torchrun nonce (run id, restart count) must
    match on every rank, or the ranks on other nodes never accept rank 0's id"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    env = {"TORCHELASTIC_RUN_ID": "job-42", "TORCHELASTIC_RESTART_COUNT": "0"}
    agents = [ctx.Process(target=_agent, args=(r, 3, "multinode", str(tmp_path), q, env)) for r in range(3)]
    for a in agents:
        a.start()
    got = [q.get(timeout=120)[1] for _ in agents]
    for a in agents:
        a.join(timeout=60)
        assert a.exitcode == 0
    assert len({g[2] for g in got}) == 1
    assert sorted(g[0] for g in got) == [0, 1, 2]


def test_torchrun_nonce_has_no_process_ids(monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))
    import sharded
    monkeypatch.delenv("ZKG_RDZV_NONCE", raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "abc")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "2")
    assert sharded.rendezvous_nonce() == b"abc:2"
