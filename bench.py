#!/usr/bin/env python3
"""Benchmark: BLS12-381 G1 MSM pairs/s at 2^20 per GPU (BASELINE.json configs[1]),
plus the Fr NTT/iNTT at 2^24 (configs[2]) as a secondary line item.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one complete MSM over the rank's 2^20 (scalar, point) pairs -- digits,
counting sort, bucket accumulation, bucket reduction, host Horner -- with the inputs
already resident in HBM; for N > 1 it also includes the RCCL all-gather of the partial
sums and their combination (weak scaling: every GPU owns 2^20 pairs, the job is the
N*2^20-pair MSM).  Data are synthetic (deterministic generator, zk_gen.cpp): scalars are
uniform Fr in Montgomery form (the Haskell `msm` path), points an arithmetic
progression of random subgroup points in affine Montgomery form.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zikkurat-algebra_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
MSM_BYTES_PER_PAIR = {"bls12_381": 128, "bn128": 96}  # scalar 32 B + affine point
NTT_BYTES_PER_ELEM = 64  # read + write 32 B per transform
SEED = {"bls12_381": 0x5A4B0002, "bn128": 0x5A4B0004}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--curve", default="bls12_381", choices=["bls12_381", "bn128"])
    ap.add_argument("--log-n", type=int, default=20, help="log2 pairs per GPU")
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--ntt-log", type=int, default=24)
    ap.add_argument("--ntt-steps", type=int, default=5)
    ap.add_argument("--no-ntt", action="store_true")
    ap.add_argument("--cpu-sample-log", type=int, default=18, help="log2 pairs in the bounded CPU sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for the partial-sum exchange (nccl = RCCL over xGMI)")
    return ap.parse_args()


def baseline():
    """expected outputs of the BASELINE configs, produced by the reference (tools/make_golden.py)"""
    p = os.path.join(ROOT, "tests", "golden", "baseline_configs.json")
    return json.load(open(p)) if os.path.exists(p) else {}


def windows_used(c, bits=255):
    # signed c-bit digits of < 2^255 scalars: the carry window is (nearly) empty
    return -(-bits // c)


def load_pmc(kernel):
    """HBM traffic per launch from a committed rocprofv3 PMC summary (profiles/*pmc*.json)."""
    pdir = os.path.join(ROOT, "profiles")
    best = None
    if os.path.isdir(pdir):
        for f in sorted(os.listdir(pdir)):
            if f.endswith(".json") and "pmc" in f:
                try:
                    d = json.load(open(os.path.join(pdir, f)))
                    if kernel in d:
                        best = d[kernel]
                except (OSError, ValueError):
                    pass
    return best


def main():
    args = parse()
    import numpy as np
    import zkalgebra as zk
    from sharded import allgather_partials, combine_partials

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    zk.require_gpu()
    device = local % zk.device_count()  # (several ranks share a GPU only in single-GPU rehearsals)
    if world > 1:
        import torch
        import torch.distributed as dist
        if args.backend == "nccl":
            torch.cuda.set_device(device)
        dist.init_process_group(args.backend)
    zk.load().zkg_set_device(device)
    xdev = "cuda" if args.backend == "nccl" else None

    curve = args.curve
    n_local = 1 << args.log_n
    n_total = n_local * world
    lo = rank * n_local
    seed = SEED[curve]
    t = time.time()
    scalars = zk.gen_fr(curve, seed, n_local, start=lo)
    points = zk.gen_points(curve, seed, n_local, start=lo)
    gen_s = time.time() - t
    d_s, d_p = zk.DeviceBuffer(scalars), zk.DeviceBuffer(points)

    def step():
        partial = zk.msm_device(curve, n_local, d_s, d_p, mont=True, window=args.window)
        if world > 1:
            parts = allgather_partials(partial, device=xdev)
            _, aff = combine_partials(curve, parts)
        else:
            aff = zk.g1_to_affine(curve, partial)
        return aff

    def sync():
        zk.load().zkg_device_synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        aff = step()
    sync()
    zk.timer(enable=True, reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        aff = step()
    sync()
    elapsed = time.perf_counter() - t0
    kt_ms, kt_n = zk.timer(enable=False)
    if world > 1:
        import torch
        e = torch.tensor([elapsed], dtype=torch.float64, device=xdev or "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    ms_per_step = elapsed / args.steps * 1e3
    value = n_total / (elapsed / args.steps)
    c = args.window if args.window else zk.load().zkg_msm_default_window(n_local)
    accum_s = (kt_ms / kt_n) / 1e3 if kt_n else float("nan")
    algo_bytes = MSM_BYTES_PER_PAIR[curve] * n_local
    achieved = algo_bytes / accum_s / 1e9
    madds = windows_used(c) * n_local
    pmc = load_pmc("k_accum")
    mul_peak = zk.field_mul_rate(curve, "fp")

    # parity of the timed result against the reference's own output (tests/golden)
    parity = None
    if world == 1 and lo == 0:
        key = {"bls12_381": "config2_bls12_381_msm_2^20", "bn128": "config4_bn128_msm_2^24"}[curve]
        cfg = baseline().get(key)
        if cfg and cfg["log_n"] == args.log_n:
            parity = [int(x) for x in aff] == cfg["affine"]

    result = {
        "metric": "BLS12-381 G1 MSM pairs/sec at 2^20; Fr NTT 2^24 elems/sec (1/2/4/8 GPU)",
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
        "config": {"workload": f"{curve}_g1_msm_2^{args.log_n}_per_gpu", "curve": curve,
                   "pairs_per_gpu": n_local, "pairs_total": n_total, "scalars": "Fr Montgomery (Haskell msm path)",
                   "window_c": c, "parallelism": f"shard{world}" if world > 1 else "single"},
        "parity_vs_reference": parity,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
                     "kernel": "k_accum (bucket accumulation)",
                     "kernel_ms": accum_s * 1e3,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "note": "MSM is VALU integer-multiply bound; see valu_roofline"},
        "valu_roofline": {"bound": "valu (v_mad_u64_u32)", "madds_per_launch": madds,
                          "fp_muls_per_launch": 10 * madds, "unit": "Fp products/s",
                          "achieved": 10 * madds / accum_s, "peak": mul_peak,
                          "frac": 10 * madds / accum_s / mul_peak,
                          "peak_source": "zkg_field_mul_rate: live probe of the same fe_mul on this GPU"},
        "input_gen_s": gen_s,
    }

    if rank == 0 and world == 1 and not args.no_ntt:
        result["ntt"] = bench_ntt(zk, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(zk, curve, seed, args.cpu_sample_log)
    d_s.free()
    d_p.free()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_ntt(zk, args):
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
    res = {}
    fr_peak = zk.field_mul_rate(curve, "fr")
    for name, src, dst, inv in (("forward", d_x, d_f, False), ("inverse", d_f, d_i, True)):
        zk.timer(enable=True, reset=True)
        t0 = time.perf_counter()
        for _ in range(args.ntt_steps):
            zk.ntt_device(curve, m, g, src, dst, inverse=inv)
        zk.load().zkg_device_synchronize()
        dt = (time.perf_counter() - t0) / args.ntt_steps
        kms, kn = zk.timer(enable=False)
        kt = kms / kn / 1e3
        muls = n // 2 * m + 2 * n  # butterfly products + two inter-pass twiddle products per element
        res[name] = {"elems_per_s": n / dt, "ms": dt * 1e3, "kernel_ms": kt * 1e3,
                     "valu_roofline": {"fr_muls": muls, "achieved": muls / kt, "peak": fr_peak,
                                       "frac": muls / kt / fr_peak, "unit": "Fr products/s"},
                     "roofline": {"bound": "hbm", "achieved": NTT_BYTES_PER_ELEM * n / kt / 1e9,
                                  "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                  "frac": NTT_BYTES_PER_ELEM * n / kt / 1e9 / HBM_PEAK_GBPS}}
    f = d_f.to_host(x)
    back = d_i.to_host(x)
    cfg = baseline().get("config3_bls12_381_ntt_2^24")
    res["parity_vs_reference"] = {
        "forward_sha256_match": (hashlib.sha256(f.tobytes()).hexdigest() == cfg["forward_sha256"])
        if cfg and cfg["log_n"] == m else None,
        "roundtrip_exact": bool(np.array_equal(back, x)),
    }
    res["workload"] = f"bls12_381_fr_ntt_2^{m}"
    for b in (d_x, d_f, d_i):
        b.free()
    return res


def cpu_baseline(zk, curve, seed, log_sample):
    """The reference's own C (oracle/_ref) on one host core, on a bounded sample of the
    same workload (the first 2^log_sample pairs); falls back to our C restatement."""
    import numpy as np
    from oracle.oracle import Oracle, Reference
    n = 1 << log_sample
    sc = zk.gen_fr(curve, seed, n)
    pts = zk.gen_points(curve, seed, n)
    if Reference.available():
        impl, kind = Reference(), "reference"
    else:
        impl, kind = Oracle(), "port"
    t0 = time.perf_counter()
    out = impl.msm(curve, sc, pts, mont=True, out="affine")
    dt = time.perf_counter() - t0
    gpu = zk.msm_affine(curve, sc, pts)
    return {"value": n / dt, "unit": "pairs/s", "cores": 1, "kind": kind,
            "sample": f"first 2^{log_sample} pairs of the same {curve} G1 MSM workload "
                      f"({'MSM_mont_coeff_affine_out of lib/cbits' if kind == 'reference' else 'oracle restatement'})",
            "seconds": dt, "host_nproc": os.cpu_count(),
            "gpu_matches_cpu_on_sample": bool(np.array_equal(out, gpu))}


if __name__ == "__main__":
    import numpy as np  # noqa: F401
    main()
