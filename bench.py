#!/usr/bin/env python3
"""Benchmark of the MSM / NTT hot path (BASELINE.json metric: "BLS12-381 G1 MSM pairs/sec at
2^20; Fr NTT 2^24 elems/sec (1/2/4/8 GPU)").

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workloads (synthetic, deterministic generator zk_gen.cpp: uniform Fr scalars in Montgomery
form -- the Haskell `msm` path -- and an arithmetic progression of random order-r subgroup
points in affine Montgomery form; inputs resident in HBM when the timed region starts):
  * headline, every N: the BLS12-381 G1 MSM with 2^20 pairs PER GPU (BASELINE configs[1] at
    N = 1).  At N > 1 rank r holds pairs [r 2^20, (r+1) 2^20) of one N * 2^20-pair MSM; a step
    is every rank's chunk MSM plus the library's own exchange of the partial sums
    (zkg_g1_msm_device_sharded: ncclAllGather over xGMI on the library's stream, rank-ordered
    adds) -- per-GPU work fixed as N grows ("weak").  A step is one complete MSM (digits, bucket
    sort, accumulation, bucket reduction, host finish, affine output).
  * config5 key, every N (BASELINE configs[4]): the 2^26-pair BLS12-381 MSM split into N
    contiguous shards (2^26 on one GPU at N = 1): total work fixed ("strong"), parity against
    the reference's own output for that config (tests/golden/baseline_configs.json).
  * NTT (configs[2]): BLS12-381 Fr NTT and iNTT of 2^24 elements on every rank (replicas:
    a single 2^24 transform is a few ms on one GPU); aggregate elems/s over ranks.
  * config4 (configs[3], N = 1 only): the BN128 G1 MSM of 2^24 pairs (KZG-commit shaped), a
    secondary line with its own parity check against the reference's output.
Multi-GPU processes hold ONE HIP runtime (the library's, /opt/rocm) and never import torch: the
rendezvous is a file (sharded.rendezvous_path), barrier / max-over-ranks / the exchange are the
library's RCCL calls.  (--backend gloo: the torch.distributed CPU rehearsal used by the tests.)
Rank 0 at N = 1 also reports the rate through the reference-named entry points with host
buffers (what the Haskell binding pays: PCIe included) and the reference's own C
(oracle/_ref, lib/cbits compiled in place) timed on host cores at the bench sizes.
"""
import argparse
import glob
import hashlib
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MSM_BYTES_PER_PAIR = {"bls12_381": 128, "bn128": 96}  # scalar 32 B + affine point
NTT_BYTES_PER_ELEM = 64  # read + write 32 B per transform
SEED = {"bls12_381": 0x5A4B0002, "bn128": 0x5A4B0004}
SEED_CONFIG5 = 0x5A4B0005
METRIC = "BLS12-381 G1 MSM pairs/sec at 2^20; Fr NTT 2^24 elems/sec (1/2/4/8 GPU)"
FR_LIMBS = 9  # device Fr: 9 x 29-bit limbs (zk_field.hpp) -> 2 * 9 * 9 = 162 v_mad_u64_u32 per product


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--curve", default="bls12_381", choices=["bls12_381", "bn128"])
    ap.add_argument("--log-n", type=int, default=20, help="log2 pairs PER GPU of the headline MSM")
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--ntt-log", type=int, default=24)
    ap.add_argument("--ntt-steps", type=int, default=5)
    ap.add_argument("--no-ntt", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) rates")
    ap.add_argument("--no-extras", action="store_true", help="skip the small-MSM sizes and the group FFT")
    ap.add_argument("--no-config4", action="store_true", help="skip the secondary BN128 2^24 (config 4) MSM line")
    ap.add_argument("--no-config5", action="store_true", help="skip the 2^26 (config 5) strong-scaling line")
    ap.add_argument("--config5-steps", type=int, default=3)
    ap.add_argument("--cpu-msm-log", type=int, default=20, help="log2 pairs of the CPU baseline MSM")
    ap.add_argument("--cpu-ntt-log", type=int, default=24, help="log2 size of the CPU baseline NTT")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--force-comm", action="store_true",
                    help="create the library's RCCL communicator even at world size 1 (one-GPU rehearsal of the "
                         "multi-GPU code path: rendezvous, zkg_g1_msm_device_sharded, barrier, max)")
    ap.add_argument("--backend", default="rccl", choices=["rccl", "gloo"],
                    help="exchange between ranks: rccl = the library's own RCCL communicator over xGMI; "
                         "gloo = torch.distributed on the CPU (rehearsals without GPUs)")
    return ap.parse_args()


def baseline():
    """expected outputs of the BASELINE configs, produced by the reference (tools/make_golden.py)"""
    p = os.path.join(ROOT, "tests", "golden", "baseline_configs.json")
    return json.load(open(p)) if os.path.exists(p) else {}


def profile_order(path):
    """sort key of a profile file name rNN<tag>_...: round, then the tag in the order tags are
    issued (a..z, then aa..az, ...), so r02e < r02au (plain string order would put r02e last)"""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    if not m:
        return (-1, 0, "", path)
    return (int(m.group(1)), len(m.group(2)), m.group(2), path)


def latest_profile(pattern):
    """newest committed profile file matching profiles/<pattern> (file names carry the round)"""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=profile_order)
    if not files:
        return None, None
    try:
        return os.path.relpath(files[-1], ROOT), json.load(open(files[-1]))
    except (OSError, ValueError):
        return None, None


def load_pmc(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/*pmc*.json)"""
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), key=profile_order):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        for k, v in d.items():
            if isinstance(v, dict) and k.split("::")[-1].startswith(kernel) and "hbm_bytes_per_launch" in v:
                best = dict(v, source=os.path.relpath(f, ROOT))
    return best


def load_rocprof_ms(kernel_prefix):
    """average duration (ms) of the kernel whose name starts with kernel_prefix in the newest
    committed rocprofv3 --stats summary (profiles/*kernel_stats.csv)"""
    import csv
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*kernel_stats.csv")), key=profile_order)
    for path in reversed(files):  # newest summary that timed this kernel (others profile other legs)
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Name"].replace("void ", "").replace("zk::", "")
                if name.startswith(kernel_prefix):
                    return {"ms": float(row["AverageNs"]) / 1e6, "calls": int(row["Calls"]),
                            "source": os.path.relpath(path, ROOT)}
    return None


def valu_ceiling():
    src, d = latest_profile("*valu_ceiling*.json")
    if not d:
        return None
    return {"source": src, "mad_rate": d["rates"]["v_mad_u64_u32"]["lane_ops_per_s"],
            "mad_clock_mhz": d["rates"]["v_mad_u64_u32"]["clock_mhz"]}


class Dist:
    """rank plumbing: init, barrier, max over ranks, exchange.  backend "rccl": the library's own
    communicator (sharded.LibComm; no torch in the process); "gloo": torch.distributed on the CPU
    (rehearsals and the CPU tests)."""

    def __init__(self, args, device):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.dist = None
        self.comm = None
        if self.world > 1 or (args.backend == "rccl" and getattr(args, "force_comm", False)):
            if args.backend == "gloo":
                import torch.distributed as dist
                dist.init_process_group("gloo")
                self.dist = dist
            else:
                from sharded import LibComm
                self.comm = LibComm(self.rank, self.world)

    def world_seen(self):
        """ranks the exchange actually connects (the library's communicator / the gloo group)"""
        if self.comm:
            import zkalgebra as zk
            return int(zk.load().zkg_comm_world())
        if self.dist:
            return int(self.dist.get_world_size())
        return 1

    def barrier(self):
        if self.comm:
            self.comm.barrier()
        elif self.dist:
            self.dist.barrier()

    def max(self, x):
        if self.comm:
            return self.comm.max(x)
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def allgather_partials(self, partial):
        if self.comm:
            return list(self.comm.allgather(partial))
        from sharded import allgather_partials
        return allgather_partials(partial)

    def close(self):
        if self.comm:
            self.comm.close()
        elif self.dist:
            self.dist.destroy_process_group()


def sharded_msm_step(zk, curve, n_local, d_s, d_p, window, dist, msm_fn=None):
    """One step of the multi-GPU MSM: this rank's shard on its GPU, the exchange of the partial
    projective sums and their rank-ordered sum, on every rank.  On GPUs with the library's
    communicator the whole step is one call (zkg_g1_msm_device_sharded).  msm_fn lets the CPU
    (gloo) test stand in for the GPU kernel; the shard / exchange / combine logic is the same."""
    from sharded import combine_partials
    if msm_fn is None and dist.comm is not None:
        return zk.g1_to_affine(curve, dist.comm.msm_device_sharded(curve, n_local, d_s, d_p, mont=True,
                                                                    window=window))
    partial = msm_fn() if msm_fn else zk.msm_device(curve, n_local, d_s, d_p, mont=True, window=window)
    if dist.world > 1:
        _, aff = combine_partials(curve, dist.allgather_partials(partial))
    else:
        aff = zk.g1_to_affine(curve, partial)
    return aff


def timed(dist, step, steps, warmup, sync, zk=None):
    """warmup, then exactly `steps` steps between barrier + device sync on both sides; seconds
    per step, max over ranks, and the last step's result.  With zk: the library's kernel timer
    covers exactly the timed steps (read it with zk.timer(enable=False) afterwards)."""
    out = None
    for _ in range(warmup):
        out = step()
    sync()
    if zk is not None:
        zk.timer(enable=True, reset=True)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    sync()
    return dist.max(time.perf_counter() - t0) / steps, out


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, script=None, grace_s=10.0):
    """Launcher of `bench.py --gpus N` run without torchrun (no WORLD_SIZE in the environment):
    start N fresh rank processes of `script` (this file) with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT and one rendezvous key + nonce for the launch, forward rank 0's
    stdout (the JSON line) and return a non-zero code if any rank fails -- the other ranks are then
    terminated (by their own pids), so a rank blocked in a collective cannot hang the launch.
    The launcher itself never imports the library or torch and makes no GPU call: every HIP
    runtime lives in a rank process."""
    import signal
    import subprocess
    import threading
    import uuid
    script = script or os.path.abspath(__file__)
    port = _free_port()
    nonce = uuid.uuid4().hex
    procs = []

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    def on_signal(signum, _frame):
        stop_all()
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    lines = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       ZKG_RDZV_KEY=f"bench_{os.getpid()}_{port}", ZKG_RDZV_NONCE=nonce)
            procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=env,
                                          stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                          text=True))

        def pump():  # rank 0's stdout, line by line: the JSON line to ours, anything else (a
            # library's own chatter, e.g. gloo's "connected to 1 peer ranks") to stderr
            for line in procs[0].stdout:
                lines.append(line)
                out = sys.stdout if line.lstrip().startswith("{") else sys.stderr
                out.write(line)
                out.flush()

        t = threading.Thread(target=pump, daemon=True)
        t.start()
        rc = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                rc = bad[0][1]
                r = bad[0][0]
                print(f"[bench launcher] rank {r} exited with {rc}; stopping the other ranks", file=sys.stderr, flush=True)
                stop_all()
                t_end = time.time() + grace_s
                while time.time() < t_end and any(p.poll() is None for p in procs):
                    time.sleep(0.05)
                stop_all(signal.SIGKILL)
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.05)
        for p in procs:
            p.wait()
        t.join(timeout=5)
        if rc == 0 and not any(line.lstrip().startswith("{") for line in lines):
            print("[bench launcher] rank 0 printed no result line", file=sys.stderr, flush=True)
            rc = 1
        return rc if rc >= 0 else 128 - rc  # a rank killed by signal k -> 128 + k
    finally:
        stop_all(signal.SIGKILL)
        for s, h in old.items():
            signal.signal(s, h)


def check_world(args):
    """--gpus N is the world the caller asked for: under an external launcher (WORLD_SIZE set) it
    must match WORLD_SIZE, or the run would report a world it was not asked for.  Returns the
    error message, or None."""
    env = os.environ.get("WORLD_SIZE")
    if env is not None and int(env) != args.gpus:
        return f"--gpus {args.gpus} but the launcher started WORLD_SIZE={env} ranks"
    return None


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no external launcher: this process only starts the N ranks (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    err = check_world(args)
    if err:
        print(f"[bench] {err}", file=sys.stderr, flush=True)
        sys.exit(2)
    import numpy as np
    import zkalgebra as zk
    from sharded import shard_range

    local = int(os.environ.get("LOCAL_RANK", "0"))
    zk.require_gpu()
    device = local % zk.device_count()  # (several ranks share a GPU only in single-GPU rehearsals)
    zk.load().zkg_set_device(device)
    dist = Dist(args, device)
    world, rank = dist.world, dist.rank
    if dist.world_seen() != args.gpus:
        print(f"[bench] rank {rank}: the communicator holds {dist.world_seen()} ranks, --gpus asked for {args.gpus}",
              file=sys.stderr, flush=True)
        sys.exit(2)

    curve = args.curve
    log_n = args.log_n
    n_local = 1 << log_n
    n_total = n_local * world
    seed = SEED[curve]
    workload = f"{curve}_g1_msm_2^{log_n}" + (f"_per_gpu_x{world}" if world > 1 else "")
    lo = rank * n_local
    t = time.time()
    scalars = zk.gen_fr(curve, seed, n_local, start=lo)
    points = zk.gen_points(curve, seed, n_local, start=lo)
    gen_s = time.time() - t
    d_s, d_p = zk.DeviceBuffer(scalars), zk.DeviceBuffer(points)

    def sync():
        zk.load().zkg_device_synchronize()
        dist.barrier()

    step_s, aff = timed(dist, lambda: sharded_msm_step(zk, curve, n_local, d_s, d_p, args.window, dist),
                        args.steps, args.warmup, sync, zk)
    kt_ms, kt_n = zk.timer(enable=False)

    ms_per_step = step_s * 1e3
    value = n_total / step_s
    c = args.window if args.window else zk.load().zkg_msm_window(zk.CURVE_ID[curve], n_local, 4, 1)
    accum_s = dist.max((kt_ms / kt_n) / 1e3 if kt_n else float("nan"))

    # parity of the timed result against the reference's own output (tests/golden)
    parity = None
    key = "config2_bls12_381_msm_2^20" if curve == "bls12_381" else "config4_bn128_msm_2^24"
    cfg = baseline().get(key)
    if world == 1 and cfg and cfg["log_n"] == log_n and cfg["seed"] == seed:
        parity = [int(x) for x in aff] == cfg["affine"]

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32-limb Montgomery Fp (381-bit)" if curve == "bls12_381" else "u32-limb Montgomery Fp (254-bit)",
        "data": "synthetic (deterministic generator zk_gen.cpp: uniform Fr scalars in Montgomery form, "
                "random order-r subgroup points P0+i*H in affine Montgomery form)",
        "config": {"workload": workload, "curve": curve, "pairs_total": n_total, "pairs_per_gpu": n_local,
                   "scalars": "Fr Montgomery (Haskell msm path)", "window_c": c,
                   "parallelism": (f"shard{world} (contiguous chunks; partial sums exchanged by the library's "
                                   f"RCCL all-gather over xGMI)" if dist.comm else
                                   f"shard{world} (contiguous chunks; CPU gloo exchange, rehearsal)")
                   if dist.comm or world > 1 else "single"},
        "parity_vs_reference": parity,
        "parity_key": key if parity is not None else None,
        "input_gen_s": gen_s,
    }
    if world > 1:
        result["parity_note"] = ("the reference has no output for a %d-pair input; config5 carries the multi-GPU "
                                 "parity check" % n_total)
    result.update(msm_rooflines(curve, n_local, c, accum_s))
    d_s.free()
    d_p.free()

    if not args.no_config5 and curve == "bls12_381":
        result["config5"] = bench_config5(zk, args, dist)
    if not args.no_ntt:
        result["ntt"] = bench_ntt(zk, args, dist)
    if rank == 0 and world == 1 and curve == "bls12_381" and not args.no_config4:
        result["config4"] = bench_config4(zk)
    if rank == 0 and world == 1 and not args.no_e2e:
        result["end_to_end"] = end_to_end(zk, curve, scalars, points, ms_per_step, result.get("ntt"), args, aff)
    if rank == 0 and world == 1 and not args.no_extras:
        result["msm_sizes"] = bench_msm_sizes(zk)
        result["group_fft"] = bench_group_fft(zk)
        result["group_fft_kzg"] = bench_group_fft(zk, m=12, reps=5)  # KZG SRS size (examples/KZG.hs:55)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(zk, curve, seed, args.cpu_msm_log, args.cpu_ntt_log)
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()


def _median_ms(fn, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def bench_msm_sizes(zk, reps=20):
    """Small device-resident MSMs (KZG-commit sizes, examples/KZG.hs:81,88): BLS12-381 at 2^10 /
    2^12 / 2^16 (median of `reps` calls, each a complete MSM incl. the host finish), and the
    reference's own outputs for its golden random_n1000 / random_n4096 cases (tests/golden) as the
    parity check of the small-input (bit-job) path."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_io import msm_cases
    curve = "bls12_381"
    out = {"curve": curve, "reps": reps, "timing": "device-resident inputs, median wall time per call"}
    gold = {name: (sc, pts, aff) for name, sc, pts, mont, aff, _ in msm_cases(curve) if name in
            ("random_n1000", "random_n4096")}
    for name, (sc, pts, aff) in gold.items():
        n = sc.shape[0]
        ds, dp = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
        got = zk.msm_device(curve, n, ds, dp)
        ms = _median_ms(lambda: zk.msm_device(curve, n, ds, dp), reps)
        ds.free()
        dp.free()
        aff_got = zk.msm_affine(curve, sc, pts)
        dev_aff = zk.batch_to_affine(curve, got.reshape(1, -1))[0]
        out[f"golden_{name}"] = {"n": n, "ms": ms, "parity_vs_reference": bool(np.array_equal(dev_aff, aff)),
                                 "host_buffer_entry_parity": bool(np.array_equal(aff_got, aff))}
    for lg in (10, 12, 16):
        n = 1 << lg
        sc, pts = zk.gen_fr(curve, 0x5A4B0002, n), zk.gen_points(curve, 0x5A4B0002, n)
        ds, dp = zk.DeviceBuffer(sc), zk.DeviceBuffer(pts)
        zk.msm_device(curve, n, ds, dp)
        out[f"2^{lg}_ms"] = _median_ms(lambda: zk.msm_device(curve, n, ds, dp), reps)
        ds.free()
        dp.free()
    out["bits_path_max_n"] = 4096
    return out


def bench_group_fft(zk, m=16, reps=3):
    """The group (curve) FFT, <C>_G1_proj_fft_forward / _inverse (bls12_381_G1_proj.c:679-790), on
    2^m subgroup points, device-resident: ms per transform, whether the GLV stages ran, and the
    round trip inverse(forward(P)) == P (exact, normalised projective)."""
    import ctypes
    import numpy as np
    lib = zk.load()
    lib.zkg_g1_fft_device.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.c_void_p, ctypes.c_void_p]
    out = {"log_n": m, "reps": reps}
    for curve in ("bls12_381", "bn128"):
        out[f"{curve}_plan_bits_per_stage"] = zk.g1_fft_plan(curve, m) or [1] * m
        n = 1 << m
        pts = zk.batch_from_affine(curve, zk.gen_points(curve, 0x5A4B0007, n))
        sg = zk.get_fft_subgroup(curve, m)
        g = sg.gen_array()
        d_in, d_out = zk.DeviceBuffer(pts), zk.DeviceBuffer.empty(pts.nbytes)
        r = {}
        for name, inv in (("forward", 0), ("inverse", 1)):
            call = lambda: lib.zkg_g1_fft_device(zk.CURVE_ID[curve], inv, m, zk._p(g), d_in.ptr, d_out.ptr)  # noqa
            call()
            lib.zkg_device_synchronize()

            def once():
                call()
                lib.zkg_device_synchronize()
            r[f"{name}_ms"] = _median_ms(once, reps)
            r[f"{name}_glv"] = bool(zk.g1_fft_last_glv())
        d_in.free()
        d_out.free()
        r["round_trip_exact"] = bool(np.array_equal(zk.inverse_fft(sg, zk.forward_fft(sg, pts)), pts))
        out[curve] = r
    return out


def bench_config5(zk, args, dist):
    """BASELINE configs[4]: the 2^26-pair BLS12-381 MSM split into `world` contiguous shards (the
    whole input on one GPU at N = 1; 2^23 pairs per GPU at N = 8), through the same library call
    as the headline.  Total work fixed ("strong"); parity against the reference's own output."""
    from sharded import shard_range
    curve, log_n, seed = "bls12_381", 26, SEED_CONFIG5
    n_total = 1 << log_n
    world, rank = dist.world, dist.rank
    lo, hi = shard_range(n_total, rank, world)
    t = time.time()
    d_s = zk.DeviceBuffer(zk.gen_fr(curve, seed, hi - lo, start=lo))
    d_p = zk.DeviceBuffer(zk.gen_points(curve, seed, hi - lo, start=lo))
    gen_s = time.time() - t

    def sync():
        zk.load().zkg_device_synchronize()
        dist.barrier()

    step_s, aff = timed(dist, lambda: sharded_msm_step(zk, curve, hi - lo, d_s, d_p, 0, dist),
                        args.config5_steps, 1, sync, zk)
    kt_ms, kt_n = zk.timer(enable=False)
    accum_s = dist.max((kt_ms / kt_n) / 1e3 if kt_n else float("nan"))
    d_s.free()
    d_p.free()
    cfg = baseline().get("config5_bls12_381_msm_2^26")
    parity = ([int(x) for x in aff] == cfg["affine"]) if cfg and cfg["seed"] == seed and cfg["log_n"] == log_n else None
    c = zk.load().zkg_msm_window(zk.CURVE_ID["bls12_381"], hi - lo, 4, 1)
    out = {"workload": f"bls12_381_g1_msm_2^26_sharded{world}", "unit": "pairs/s", "value": n_total / step_s,
           "ms": step_s * 1e3, "n_gpus": world, "scaling": "strong (2^26 pairs in total at every N)",
           "pairs_per_gpu_max": hi - lo, "steps": args.config5_steps, "warmup": 1, "window_c": c,
           "kernel_ms_max_over_ranks": accum_s * 1e3, "parity_vs_reference": parity,
           "parity_key": "config5_bls12_381_msm_2^26", "input_gen_s": gen_s,
           "exchange": "zkg_g1_msm_device_sharded (ncclAllGather of the partial sums on the library's stream)"
           if dist.comm else ("torch.distributed gloo all-gather on the CPU (rehearsal)" if world > 1 else "none (one GPU)")}
    roof = msm_rooflines(curve, hi - lo, c, accum_s, rocprof=False)
    out["roofline"] = roof["roofline"]
    if "valu_roofline" in roof:
        out["valu_roofline"] = roof["valu_roofline"]
    return out


def msm_rooflines(curve, n, c, accum_s, rocprof=True):
    """HBM roofline (the contract's) and VALU-issue roofline of the dominant kernel, k_accum.
    Work per launch: one XYZZ mixed add per nonzero signed digit, ~n * ceil(255/c) madds
    (BLS12-381 / BN128 scalars are < 2^255 after REDC).  Both fractions are given for the
    in-run HIP-event time AND for the newest committed rocprofv3 --stats average of the same
    kernel (profiles/*kernel_stats.csv), so they can be recomputed from profiles/."""
    windows = -(-255 // c)
    madds = windows * n
    algo_bytes = MSM_BYTES_PER_PAIR[curve] * n
    pmc = load_pmc("k_accum")
    rp = load_rocprof_ms("k_accum<" + ("BLS381" if curve == "bls12_381" else "BN254") + ">") if rocprof else None
    out = {"roofline": {"bound": "hbm", "achieved": algo_bytes / accum_s / 1e9, "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": algo_bytes / accum_s / 1e9 / HBM_PEAK_GBPS,
                        "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
                        "traffic_source": (pmc or {}).get("source"),
                        "kernel": "k_accum (bucket accumulation)", "kernel_ms": accum_s * 1e3,
                        "kernel_ms_source": "HIP events recorded around every k_accum launch on the library's "
                                            "own stream (zkg_timer_*), averaged over the timed steps",
                        "algorithmic_bytes_per_launch": algo_bytes,
                        "note": "MSM is VALU-issue bound (integer multiply-add), see valu_roofline"}}
    if rp:
        out["roofline"].update({"kernel_ms_rocprof": rp["ms"], "kernel_ms_rocprof_source": rp["source"],
                                "frac_rocprof": algo_bytes / (rp["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS})
    ceil = valu_ceiling()
    isa_src, isa = latest_profile(f"*isa_k_accum_{curve}.json")
    if ceil and isa and "hot_loop" in isa:
        per = isa["hot_loop"]["per_iteration"]
        slots = isa["hot_loop"]["issue_slots_per_iteration"]
        mads = per.get("v_mad_u64_u32", 0)
        out["valu_roofline"] = {
            "bound": "VALU issue (v_mad_u64_u32 and the other half-rate ops)",
            "unit": "half-rate issue slots/s",
            "madds_per_launch": madds,
            "issue_slots_per_madd": slots,
            "v_mad_u64_u32_per_madd": mads,
            "achieved": madds * slots / accum_s,
            "peak": ceil["mad_rate"],
            "frac": madds * slots / accum_s / ceil["mad_rate"],
            "mad_only_frac": madds * mads / accum_s / ceil["mad_rate"],
            "peak_source": f"{ceil['source']}: measured v_mad_u64_u32 issue rate (inline-asm chains, "
                           f"8 waves/SIMD, {ceil['mad_clock_mhz']:.0f} MHz held under that load)",
            "count_source": f"{isa_src}: static instruction counts of k_accum's hot loop (one madd per "
                            "iteration); half-rate ops = 1 slot, full-rate 32-bit ops = 1/2 slot",
        }
        if rp:
            out["valu_roofline"]["frac_rocprof"] = madds * slots / (rp["ms"] * 1e-3) / ceil["mad_rate"]
    return out


def bench_config4(zk, steps=3, warmup=1):
    """Secondary line at N = 1: BASELINE configs[3], the BN128 G1 MSM of 2^24 pairs (KZG-commit
    shaped, examples/KZG.hs:77-81), device-resident, with parity against the reference's own
    output for that config (tests/golden/baseline_configs.json)."""
    curve, log_n = "bn128", 24
    n, seed = 1 << log_n, SEED["bn128"]
    t = time.time()
    d_s, d_p = zk.DeviceBuffer(zk.gen_fr(curve, seed, n)), zk.DeviceBuffer(zk.gen_points(curve, seed, n))
    gen_s = time.time() - t
    for _ in range(warmup):
        zk.msm_device(curve, n, d_s, d_p)
    zk.load().zkg_device_synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        proj = zk.msm_device(curve, n, d_s, d_p)
    zk.load().zkg_device_synchronize()
    dt = (time.perf_counter() - t0) / steps
    aff = zk.g1_to_affine(curve, proj)
    cfg = baseline().get("config4_bn128_msm_2^24")
    parity = ([int(x) for x in aff] == cfg["affine"]) if cfg and cfg["seed"] == seed and cfg["log_n"] == log_n else None
    d_s.free()
    d_p.free()
    return {"workload": "bn128_g1_msm_2^24", "unit": "pairs/s", "value": n / dt, "ms": dt * 1e3, "steps": steps,
            "warmup": warmup, "window_c": zk.load().zkg_msm_window(zk.CURVE_ID[curve], n, 4, 1), "parity_vs_reference": parity,
            "input_gen_s": gen_s}


def bench_ntt(zk, args, dist):
    import numpy as np
    curve = "bls12_381"
    m = args.ntt_log
    n = 1 << m
    x = zk.gen_fr(curve, 0x5A4B0003, n)
    sg = zk.get_fft_subgroup(curve, m)
    g = sg.gen_array()
    d_x = zk.DeviceBuffer(x)
    d_f = zk.DeviceBuffer.empty(x.nbytes)
    d_i = zk.DeviceBuffer.empty(x.nbytes)
    zk.ntt_device(curve, m, g, d_x, d_f)
    zk.ntt_device(curve, m, g, d_f, d_i, inverse=True)
    zk.load().zkg_device_synchronize()
    res = {"workload": f"bls12_381_fr_ntt_2^{m}" + (f"_replicas{dist.world}" if dist.world > 1 else ""),
           "unit": "elems/s", "n_gpus": dist.world,
           "scaling": "weak (one independent 2^24 transform per GPU)" if dist.world > 1 else "single"}
    ceil = valu_ceiling()
    isa_src, isa = latest_profile("*isa_k_ntt_pass.json")
    for name, src, dst, inv in (("forward", d_x, d_f, False), ("inverse", d_f, d_i, True)):
        dist.barrier()
        zk.timer(enable=True, reset=True)
        t0 = time.perf_counter()
        for _ in range(args.ntt_steps):
            zk.ntt_device(curve, m, g, src, dst, inverse=inv)
        zk.load().zkg_device_synchronize()
        dt = dist.max(time.perf_counter() - t0) / args.ntt_steps
        kms, kn = zk.timer(enable=False)
        kt = kms / kn / 1e3
        products = n // 2 * m + 2 * n  # butterfly products + the inter-pass / closing products
        r = {"elems_per_s": dist.world * n / dt, "ms": dt * 1e3, "kernel_ms": kt * 1e3,
             "roofline": {"bound": "hbm", "achieved": NTT_BYTES_PER_ELEM * n / kt / 1e9,
                          "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                          "frac": NTT_BYTES_PER_ELEM * n / kt / 1e9 / HBM_PEAK_GBPS}}
        if ceil:
            mads = products * 2 * FR_LIMBS * FR_LIMBS
            r["valu_roofline"] = {"fr_products": products, "v_mad_u64_u32": mads,
                                  "unit": "v_mad_u64_u32/s", "mad_only_achieved": mads / kt, "peak": ceil["mad_rate"],
                                  "mad_only_frac": mads / kt / ceil["mad_rate"], "peak_source": ceil["source"]}
            model = (isa or {}).get("curves", {}).get(curve, {}).get("transforms", {}).get(f"m{m}_{name}")
            if model:
                slots = model["issue_slots"]
                r["valu_roofline"].update({
                    "bound": "VALU issue", "issue_slots_per_transform": slots, "unit": "half-rate issue slots/s",
                    "achieved": slots / kt, "frac": slots / kt / ceil["mad_rate"],
                    "count_source": f"{isa_src}: static issue slots of every k_ntt_pass loop x its trip count "
                                    "per launch shape, summed over the passes (tools/ntt_isa_model.py)"})
        rp = load_rocprof_ms("k_ntt_pass<BLS_Fr, 256>") if m == 24 else None
        if rp:  # 2^24 = three 256-point passes of this kernel (forward and inverse alike)
            r["kernel_ms_rocprof"] = 3 * rp["ms"]
            r["kernel_ms_rocprof_source"] = rp["source"] + " (3 x the average k_ntt_pass<BLS_Fr, 256> launch)"
            r["roofline"]["frac_rocprof"] = NTT_BYTES_PER_ELEM * n / (3 * rp["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS
        res[name] = r
    res["value"] = res["forward"]["elems_per_s"]
    # cold call: the first transform after zkg_release (working-set arena allocated and the
    # per-(m, generator, direction) twiddle tables built inside the call), beside the warm one
    zk.load().zkg_device_synchronize()
    zk.release()
    dist.barrier()
    t0 = time.perf_counter()
    zk.ntt_device(curve, m, g, d_x, d_f)
    zk.load().zkg_device_synchronize()
    res["forward"]["cold_ms"] = (time.perf_counter() - t0) * 1e3
    res["forward"]["cold_note"] = ("first call after zkg_release: arena hipMalloc + twiddle-table build "
                                   "(k_tw_tables / k_tw_inner / k_tw_pass, 512 MiB pass-0 table) + the transform")
    f = d_f.to_host(x)
    back = d_i.to_host(x)
    zk.ntt_device(curve, m, g, d_x, d_i, inverse=True)  # the inverse of the config input itself
    ix = d_i.to_host(x)
    cfg = baseline().get("config3_bls12_381_ntt_2^24")
    ok = cfg and cfg["log_n"] == m
    res["parity_vs_reference"] = {
        "forward_sha256_match": (hashlib.sha256(f.tobytes()).hexdigest() == cfg["forward_sha256"]) if ok else None,
        "inverse_sha256_match": (hashlib.sha256(ix.tobytes()).hexdigest() == cfg.get("inverse_sha256"))
        if ok and "inverse_sha256" in cfg else None,
        "roundtrip_exact": bool(np.array_equal(back, x)),
    }
    for b in (d_x, d_f, d_i):
        b.free()
    return res


def end_to_end(zk, curve, scalars, points, device_ms, ntt, args, device_aff, reps=5):
    """The reference-named entry points with HOST buffers, as the Haskell binding calls them
    (inputs cross PCIe every call; caller memory is ordinary pageable memory)."""
    import numpy as np
    n = scalars.shape[0]
    out = {}
    zk.msm_affine(curve, scalars, points)  # warm (arena, staging)
    t0 = time.perf_counter()
    for _ in range(reps):
        aff = zk.msm_affine(curve, scalars, points)
    dt = (time.perf_counter() - t0) / reps
    h2d = scalars.nbytes + points.nbytes
    out["msm"] = {"symbol": f"{curve}_G1_proj_MSM_mont_coeff_affine_out", "pairs_per_s": n / dt, "ms": dt * 1e3,
                  "device_resident_ms": device_ms, "h2d_bytes": h2d,
                  "h2d_GBps_effective": h2d / max(dt - device_ms * 1e-3, 1e-9) / 1e9,
                  "matches_device_resident": bool(np.array_equal(aff, device_aff))}
    if ntt and not args.no_ntt:
        m = args.ntt_log
        x = zk.gen_fr("bls12_381", 0x5A4B0003, 1 << m)
        sg = zk.get_fft_subgroup("bls12_381", m)
        lib = zk.load()
        reused = np.zeros_like(x)
        reused.fill(1)  # pages resident
        g = sg.gen_array()
        for name, key in (("ntt_forward", "forward"), ("ntt_inverse", "inverse")):
            sym = getattr(lib, f"bls12_381_poly_mont_{name}")
            fn = zk.forward_ntt if key == "forward" else zk.inverse_ntt
            fn(sg, x)
            keep = []  # outputs stay alive: the timing holds the call, not freeing the previous output
            t0 = time.perf_counter()
            for _ in range(2):
                keep.append(fn(sg, x))  # fresh output array per call, as the Haskell binding allocates
            dt = (time.perf_counter() - t0) / 2
            del keep
            t0 = time.perf_counter()
            for _ in range(2):
                sym(m, zk._p(g), zk._p(x), zk._p(reused))
            dt2 = (time.perf_counter() - t0) / 2
            dev = ntt[key]["ms"]
            out[name] = {"symbol": f"bls12_381_poly_mont_{name}", "elems_per_s": x.shape[0] / dt, "ms": dt * 1e3,
                         "ms_reused_output": dt2 * 1e3, "elems_per_s_reused_output": x.shape[0] / dt2,
                         "device_resident_ms": dev, "pcie_bytes": 2 * x.nbytes,
                         "pcie_GBps_effective": 2 * x.nbytes / max(dt2 - dev * 1e-3, 1e-9) / 1e9,
                         "note": "ms: a fresh, uninitialised output array per call (np.empty, as the binding's "
                                 "mallocForeignPtrArray, Poly.hs:405): its first touch -- 512 MiB of new pages -- "
                                 "is paid inside the call: the library copies the result back through its own pinned "
                                 "double buffer (copy_to_host, zk_runtime.cpp: 32 MiB DMA pieces into one half while "
                                 "the host pool copies the other half into the caller's array, faulting its pages in "
                                 "as it goes); ms_reused_output: the same symbol into a resident buffer.  (Round 4 allocated with np.zeros inside the timing: +~25 ms of calloc "
                                 "zeroing that the Haskell binding never pays.)"}
    return out


def cpu_baseline(zk, curve, seed, msm_log, ntt_log):
    """The reference's own C (oracle/_ref: lib/cbits compiled in place) at the bench sizes: the
    MSM of the headline's 2^msm_log pairs (MSM_mont_coeff_affine_out, the reference's window rule)
    and the BLS12-381 NTT and iNTT at 2^ntt_log (24 = the GPU line's size).  Each is the
    reference's single-threaded C on ONE host core; the three run at the same time on three
    cores (ctypes releases the GIL), so the wall time is the slowest one (the 2^24 inverse,
    ~1 min), not the sum.  Falls back to our C restatement (oracle.Oracle) without oracle/_ref."""
    import threading
    import numpy as np
    from oracle.oracle import Oracle, Reference
    impl, kind = (Reference(), "reference") if Reference.available() else (Oracle(), "port")
    n = 1 << msm_log
    sc = zk.gen_fr(curve, seed, n)
    pts = zk.gen_points(curve, seed, n)
    m = ntt_log
    x = zk.gen_fr("bls12_381", 0x5A4B0003, 1 << m)
    sg = zk.get_fft_subgroup("bls12_381", m)
    g = sg.gen_array()
    got = {}

    def run(name, fn):
        t0 = time.perf_counter()
        y = fn()
        got[name] = (y, time.perf_counter() - t0)

    jobs = [("msm", lambda: impl.msm(curve, sc, pts, mont=True, out="affine")),
            ("forward", lambda: impl.ntt("bls12_381", m, g, x, inverse=False)),
            ("inverse", lambda: impl.ntt("bls12_381", m, g, x, inverse=True))]
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=j) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    out, dt = got["msm"]
    gpu = zk.msm_affine(curve, sc, pts)
    res = {"value": n / dt, "unit": "pairs/s", "cores": 1, "kind": kind,
           "sample": f"the whole 2^{msm_log}-pair {curve} G1 MSM of the headline through "
                     f"{'MSM_mont_coeff_affine_out of lib/cbits' if kind == 'reference' else 'the oracle restatement'}",
           "seconds": dt, "host_nproc": os.cpu_count(), "gpu_matches_cpu": bool(np.array_equal(out, gpu)),
           "concurrency": "MSM, NTT and iNTT each on one core, run at the same time (wall %.1f s)" % wall}
    ntt = {}
    for name in ("forward", "inverse"):
        y, dt = got[name]
        gy = zk.inverse_ntt(sg, x) if name == "inverse" else zk.forward_ntt(sg, x)
        ntt[name] = {"value": x.shape[0] / dt, "unit": "elems/s", "seconds": dt,
                     "gpu_matches_cpu": bool(np.array_equal(y, gy))}
    res["ntt"] = dict(ntt, cores=1, kind=kind,
                      sample=f"BLS12-381 Fr {'poly_mont_ntt_forward/_inverse of lib/cbits' if kind == 'reference' else 'oracle'}"
                             f" of the whole 2^{m}-element input of the GPU NTT line")
    return res


if __name__ == "__main__":
    main()
