"""bench.py --gpus N without torchrun: the parent process starts the N rank processes itself
(bench.launch_ranks) before any GPU call, forwards rank 0's one JSON line, and propagates a failing
rank's exit code after stopping the others; under an external launcher a world that differs from
--gpus is refused.  (VERDICT r04 "next round" item 1: `python3 bench.py --gpus 8` used to time one
rank silently.)  The ranks here are a stub worker script, so the test needs no GPU; the GPU box
runs the real bench through the same launcher (profiles/r05*_bench2_*)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = textwrap.dedent("""
    import json, os, sys, time
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    mode = sys.argv[1]
    info = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                                           "ZKG_RDZV_KEY", "ZKG_RDZV_NONCE")}
    open(os.path.join(sys.argv[2], f"rank{rank}.json"), "w").write(json.dumps(info))
    if mode == "fail1" and rank == 1:
        sys.exit(3)
    if mode == "fail1":
        time.sleep(600)  # rank 0 "blocked in a collective": the launcher must stop it
    if mode == "silent":
        sys.exit(0)
    if rank == 0:
        if mode == "chatty":  # a library printing to stdout (gloo's peer-connection line)
            print("[Gloo] Rank 0 is connected to 1 peer ranks.", flush=True)
        print(json.dumps({"metric": "stub", "n_gpus": world, "value": 1.0}), flush=True)
""")


def _launch(tmp_path, n, mode, timeout=120):
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
            f"sys.exit(bench.launch_ranks({n}, [{mode!r}, {str(tmp_path)!r}], script={str(stub)!r}, grace_s=2))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=timeout)
    return p, time.time() - t0


@pytest.mark.parametrize("n", [2, 3, 8])
def test_launcher_starts_n_ranks_and_forwards_one_line(tmp_path, n):
    p, _ = _launch(tmp_path, n, "ok")
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    assert json.loads(lines[0])["n_gpus"] == n
    infos = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(n)]
    assert [int(i["RANK"]) for i in infos] == list(range(n))
    assert [int(i["LOCAL_RANK"]) for i in infos] == list(range(n))
    assert all(int(i["WORLD_SIZE"]) == n for i in infos)
    assert all(i["MASTER_ADDR"] == "127.0.0.1" for i in infos)
    for k in ("MASTER_PORT", "ZKG_RDZV_KEY", "ZKG_RDZV_NONCE"):  # one launch: one value on every rank
        assert len({i[k] for i in infos}) == 1 and infos[0][k]


def test_launcher_propagates_failure_and_stops_other_ranks(tmp_path):
    p, dt = _launch(tmp_path, 2, "fail1")
    assert p.returncode == 3, (p.returncode, p.stderr)
    assert "rank 1 exited with 3" in p.stderr
    assert dt < 60  # rank 0 (sleeping 600 s) was stopped, not waited for


def test_launcher_fails_without_result_line(tmp_path):
    p, _ = _launch(tmp_path, 2, "silent")
    assert p.returncode != 0
    assert "no result line" in p.stderr


def _bench(args, env_extra, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def test_external_world_mismatch_is_refused():
    p = _bench(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "--gpus 4" in p.stderr and "WORLD_SIZE=2" in p.stderr
    assert not p.stdout.strip()


def test_real_bench_ranks_fail_loudly_without_gpu():
    """the real bench through its own launcher on a host without a GPU: every rank fails in
    zk.require_gpu, the launcher returns non-zero and prints no result line (no world-1 line)"""
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {})
    assert p.returncode != 0
    assert not p.stdout.strip()


def test_launcher_stdout_is_the_json_line_only(tmp_path):
    """rank 0's non-JSON stdout (gloo prints its peer-connection line there) goes to stderr, so
    the launcher's stdout is exactly the one result line"""
    p, _ = _launch(tmp_path, 2, "chatty")
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2
    assert "[Gloo]" in p.stderr
