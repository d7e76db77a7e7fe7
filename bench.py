#!/usr/bin/env python3
"""Benchmark of the MSM / NTT hot path (BASELINE.json metric: "BLS12-381 G1 MSM pairs/sec at
2^20; Fr NTT 2^24 elems/sec (1/2/4/8 GPU)").

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workloads (synthetic, deterministic generator zk_gen.cpp: uniform Fr scalars in Montgomery
form -- the Haskell `msm` path -- and an arithmetic progression of random order-r subgroup
points in affine Montgomery form; inputs resident in HBM when the timed region starts):
  * N = 1: BASELINE configs[1], BLS12-381 G1 MSM of 2^20 pairs.  A step is one complete MSM
    (digits, bucket sort, accumulation, bucket reduction, host finish, affine output).
  * N > 1: BASELINE configs[4], the 2^26-pair BLS12-381 MSM split into N contiguous shards
    (sharded.shard_range); a step is every rank's shard MSM plus the all-gather of the
    partial sums (torch.distributed "nccl" = RCCL over xGMI) and their rank-ordered sum.
    Total work is fixed ("strong"); rank 0 checks the affine result against the
    reference's own output for config 5 (tests/golden/baseline_configs.json).
  * NTT (configs[2]): BLS12-381 Fr NTT and iNTT of 2^24 elements on every rank (replicas:
    a single 2^24 transform is a few ms on one GPU); aggregate elems/s over ranks.
  * config4 (configs[3], N = 1 only): the BN128 G1 MSM of 2^24 pairs (KZG-commit shaped), a
    secondary line with its own parity check against the reference's output.
Rank 0 at N = 1 also reports the rate through the reference-named entry points with host
buffers (what the Haskell binding pays: PCIe included) and the reference's own C
(oracle/_ref, lib/cbits compiled in place) timed on one host core.
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
    ap.add_argument("--log-n", type=int, default=0,
                    help="log2 pairs: per GPU at N = 1 (default 20), total at N > 1 (default 26)")
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--ntt-log", type=int, default=24)
    ap.add_argument("--ntt-steps", type=int, default=5)
    ap.add_argument("--no-ntt", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-buffer (PCIe-inclusive) rates")
    ap.add_argument("--no-config4", action="store_true", help="skip the secondary BN128 2^24 (config 4) MSM line")
    ap.add_argument("--cpu-msm-log", type=int, default=20, help="log2 pairs of the CPU baseline MSM")
    ap.add_argument("--cpu-ntt-log", type=int, default=20, help="log2 size of the CPU baseline NTT sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for the partial-sum exchange (nccl = RCCL over xGMI)")
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


def valu_ceiling():
    src, d = latest_profile("*valu_ceiling*.json")
    if not d:
        return None
    return {"source": src, "mad_rate": d["rates"]["v_mad_u64_u32"]["lane_ops_per_s"],
            "mad_clock_mhz": d["rates"]["v_mad_u64_u32"]["clock_mhz"]}


class Dist:
    """torch.distributed plumbing: init, barrier, max over ranks, all-gather of tiny payloads"""

    def __init__(self, args, device):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.dist = None
        self.xdev = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            if args.backend == "nccl":
                torch.cuda.set_device(device)
                self.xdev = "cuda"
            dist.init_process_group(args.backend)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device=self.xdev or "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def sharded_msm_step(zk, curve, n_local, d_s, d_p, window, dist, msm_fn=None):
    """One step of the multi-GPU MSM: this rank's shard on its GPU, all-gather of the partial
    projective sums, rank-ordered sum on every rank.  msm_fn lets the CPU (gloo) test stand
    in for the GPU kernel; everything else is this exact code path."""
    from sharded import allgather_partials, combine_partials
    partial = msm_fn() if msm_fn else zk.msm_device(curve, n_local, d_s, d_p, mont=True, window=window)
    if dist.world > 1:
        parts = allgather_partials(partial, device=dist.xdev)
        _, aff = combine_partials(curve, parts)
    else:
        aff = zk.g1_to_affine(curve, partial)
    return aff


def main():
    args = parse()
    import numpy as np
    import zkalgebra as zk
    from sharded import shard_range

    local = int(os.environ.get("LOCAL_RANK", "0"))
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and args.backend == "nccl":
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so, libhsa-runtime64.so).  Loaded
        # after the library's (/opt/rocm), it finds no GPU (two HSA runtimes in one process); loaded
        # first, the library binds to the same runtime by soname (profiles/r03y_torch_runtime_order.txt).
        import torch
        torch.cuda.set_device(local % torch.cuda.device_count())
    zk.require_gpu()
    device = local % zk.device_count()  # (several ranks share a GPU only in single-GPU rehearsals)
    dist = Dist(args, device)
    world, rank = dist.world, dist.rank
    zk.load().zkg_set_device(device)

    curve = args.curve
    if world == 1:
        log_n = args.log_n or 20
        n_total = 1 << log_n
        seed = SEED[curve]
        workload = f"{curve}_g1_msm_2^{log_n}"
        scaling = "weak"
    else:
        log_n = args.log_n or 26
        n_total = 1 << log_n
        seed = SEED_CONFIG5 if curve == "bls12_381" else SEED[curve]
        workload = f"{curve}_g1_msm_2^{log_n}_sharded{world}"
        scaling = "strong"
    lo, hi = shard_range(n_total, rank, world)
    n_local = hi - lo
    t = time.time()
    scalars = zk.gen_fr(curve, seed, n_local, start=lo)
    points = zk.gen_points(curve, seed, n_local, start=lo)
    gen_s = time.time() - t
    d_s, d_p = zk.DeviceBuffer(scalars), zk.DeviceBuffer(points)

    def step():
        return sharded_msm_step(zk, curve, n_local, d_s, d_p, args.window, dist)

    def sync():
        zk.load().zkg_device_synchronize()
        dist.barrier()

    for _ in range(args.warmup):
        aff = step()
    sync()
    zk.timer(enable=True, reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        aff = step()
    sync()
    elapsed = dist.max(time.perf_counter() - t0)
    kt_ms, kt_n = zk.timer(enable=False)

    ms_per_step = elapsed / args.steps * 1e3
    value = n_total / (elapsed / args.steps)
    c = args.window if args.window else zk.load().zkg_msm_default_window(n_local)
    accum_s = (kt_ms / kt_n) / 1e3 if kt_n else float("nan")

    # parity of the timed result against the reference's own output (tests/golden)
    parity = None
    cfgs = baseline()
    key = ("config2_bls12_381_msm_2^20" if world == 1 else "config5_bls12_381_msm_2^26") \
        if curve == "bls12_381" else "config4_bn128_msm_2^24"
    cfg = cfgs.get(key)
    if cfg and cfg["log_n"] == log_n and cfg["seed"] == seed:
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
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32-limb Montgomery Fp (381-bit)" if curve == "bls12_381" else "u32-limb Montgomery Fp (254-bit)",
        "data": "synthetic (deterministic generator zk_gen.cpp: uniform Fr scalars in Montgomery form, "
                "random order-r subgroup points P0+i*H in affine Montgomery form)",
        "config": {"workload": workload, "curve": curve, "pairs_total": n_total, "pairs_per_gpu_max": n_local,
                   "scalars": "Fr Montgomery (Haskell msm path)", "window_c": c,
                   "parallelism": f"shard{world} (contiguous chunks, RCCL all-gather of partials)"
                   if world > 1 else "single"},
        "parity_vs_reference": parity,
        "parity_key": key if parity is not None else None,
        "input_gen_s": gen_s,
    }
    result.update(msm_rooflines(curve, n_local, c, accum_s))

    if not args.no_ntt:
        result["ntt"] = bench_ntt(zk, args, dist)
    if rank == 0 and world == 1 and curve == "bls12_381" and not args.no_config4:
        result["config4"] = bench_config4(zk)
    if rank == 0 and world == 1 and not args.no_e2e:
        result["end_to_end"] = end_to_end(zk, curve, scalars, points, ms_per_step, result.get("ntt"), args, aff)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(zk, curve, seed, args.cpu_msm_log, args.cpu_ntt_log)
    d_s.free()
    d_p.free()
    if rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()


def msm_rooflines(curve, n, c, accum_s):
    """HBM roofline (the contract's) and VALU-issue roofline of the dominant kernel, k_accum.
    Work per launch: one XYZZ mixed add per nonzero signed digit, ~n * ceil(255/c) madds
    (BLS12-381 / BN128 scalars are < 2^255 after REDC)."""
    windows = -(-255 // c)
    madds = windows * n
    algo_bytes = MSM_BYTES_PER_PAIR[curve] * n
    pmc = load_pmc("k_accum")
    out = {"roofline": {"bound": "hbm", "achieved": algo_bytes / accum_s / 1e9, "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": algo_bytes / accum_s / 1e9 / HBM_PEAK_GBPS,
                        "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
                        "traffic_source": (pmc or {}).get("source"),
                        "kernel": "k_accum (bucket accumulation)", "kernel_ms": accum_s * 1e3,
                        "kernel_ms_source": "HIP events recorded around every k_accum launch on the library's "
                                            "own stream (zkg_timer_*), averaged over the timed steps",
                        "algorithmic_bytes_per_launch": algo_bytes,
                        "note": "MSM is VALU-issue bound (integer multiply-add), see valu_roofline"}}
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
            "warmup": warmup, "window_c": zk.load().zkg_msm_default_window(n), "parity_vs_reference": parity,
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
                         "note": "ms: fresh numpy output per call (its first touch -- 512 MiB of new pages -- is "
                                 "paid inside the call); ms_reused_output: the same symbol into a resident buffer"}
    return out


def cpu_baseline(zk, curve, seed, msm_log, ntt_log):
    """The reference's own C (oracle/_ref: lib/cbits compiled in place) on one host core:
    the MSM at the bench's own size (2^20 by default, the reference's window rule c = 17)
    and the NTT / iNTT on a bounded 2^ntt_log sample; falls back to our C restatement."""
    import numpy as np
    from oracle.oracle import Oracle, Reference
    impl, kind = (Reference(), "reference") if Reference.available() else (Oracle(), "port")
    n = 1 << msm_log
    sc = zk.gen_fr(curve, seed, n)
    pts = zk.gen_points(curve, seed, n)
    t0 = time.perf_counter()
    out = impl.msm(curve, sc, pts, mont=True, out="affine")
    dt = time.perf_counter() - t0
    gpu = zk.msm_affine(curve, sc, pts)
    res = {"value": n / dt, "unit": "pairs/s", "cores": 1, "kind": kind,
           "sample": f"the first 2^{msm_log} pairs of the {curve} G1 MSM workload through "
                     f"{'MSM_mont_coeff_affine_out of lib/cbits' if kind == 'reference' else 'the oracle restatement'}",
           "seconds": dt, "host_nproc": os.cpu_count(),
           "gpu_matches_cpu": bool(np.array_equal(out, gpu))}
    m = ntt_log
    x = zk.gen_fr("bls12_381", 0x5A4B0003, 1 << m)
    sg = zk.get_fft_subgroup("bls12_381", m)
    g = sg.gen_array()
    ntt = {}
    for name, inv in (("forward", False), ("inverse", True)):
        t0 = time.perf_counter()
        y = impl.ntt("bls12_381", m, g, x, inverse=inv)
        dt = time.perf_counter() - t0
        gy = zk.inverse_ntt(sg, x) if inv else zk.forward_ntt(sg, x)
        ntt[name] = {"value": x.shape[0] / dt, "unit": "elems/s", "seconds": dt,
                     "gpu_matches_cpu": bool(np.array_equal(y, gy))}
    res["ntt"] = dict(ntt, cores=1, kind=kind,
                      sample=f"BLS12-381 Fr {'poly_mont_ntt_forward/_inverse of lib/cbits' if kind == 'reference' else 'oracle'}"
                             f" at 2^{m} (bench size 2^24: the reference takes ~27 s / ~78 s there, BASELINE.md)")
    return res


if __name__ == "__main__":
    main()
