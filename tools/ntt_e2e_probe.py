#!/usr/bin/env python3
"""Where a host-buffer NTT into a FRESH output array spends its time (GPU box):
   python tools/ntt_e2e_probe.py [m]
Times, for 2^m BLS12-381 Fr elements (32 B each): MADV_POPULATE_WRITE of a fresh buffer on 1 and
8 threads; a synchronous device-to-host copy into fresh / populated / resident pages; and the
reference symbol bls12_381_poly_mont_ntt_forward into a fresh and a resident output (the library
prefaults the caller's output on 8 threads unless ZK_PREFAULT=0)."""
import ctypes
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zikkurat-algebra_amd"))
import numpy as np  # noqa: E402
import zkalgebra as zk  # noqa: E402

MADV_POPULATE_WRITE = 23
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def populate(buf, threads, huge=False):
    addr, nbytes = buf.ctypes.data, buf.nbytes
    page = 4096
    if huge:  # transparent huge pages for the whole range first
        a = addr & ~(page - 1)
        libc.madvise(a, addr + nbytes - a, 14)  # MADV_HUGEPAGE
    chunk = (nbytes // threads + (2 << 20) - 1) & ~((2 << 20) - 1)
    rcs = []

    def run(lo, hi):
        a = lo & ~(page - 1)
        rcs.append(libc.madvise(a, hi - a, MADV_POPULATE_WRITE))
    th = [threading.Thread(target=run, args=(addr + o, addr + min(nbytes, o + chunk))) for o in range(0, nbytes, chunk)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    return (time.perf_counter() - t) * 1e3, rcs


def ms(fn):
    t = time.perf_counter()
    fn()
    return (time.perf_counter() - t) * 1e3


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    n = 1 << m
    zk.require_gpu()
    x = zk.gen_fr("bls12_381", 0x5A4B0003, n)
    print(f"prefault {'off' if os.environ.get('ZK_PREFAULT') == '0' else 'on'}, 2^{m} x 32 B = {x.nbytes >> 20} MiB", flush=True)
    hold = []
    for alloc in ("zeros", "empty"):
        for th in (1, 8, 16):
            b = np.zeros_like(x) if alloc == "zeros" else np.empty_like(x)
            t, rcs = populate(b, th)
            print(f"populate ({alloc:5s} buffer) {th:2d} threads: {t:7.2f} ms (rc {set(rcs)})", flush=True)
            hold.append(b)  # kept: a freed mapping could come back populated
    try:
        print("THP:", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(),
              "defrag:", open("/sys/kernel/mm/transparent_hugepage/defrag").read().strip(), flush=True)
    except OSError as e:
        print("THP settings unreadable:", e)
    for th in (1, 8, 16):
        b = np.empty_like(x)
        t, rcs = populate(b, th, huge=True)
        print(f"populate (empty buffer, MADV_HUGEPAGE) {th:2d} threads: {t:7.2f} ms (rc {set(rcs)})", flush=True)
        hold.append(b)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    for _ in range(2):
        b = np.empty_like(x)
        t = time.perf_counter()
        rc = hip.hipHostRegister(b.ctypes.data, b.nbytes, 0)
        tr = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        rc2 = hip.hipHostUnregister(b.ctypes.data)
        tu = (time.perf_counter() - t) * 1e3
        print(f"hipHostRegister fresh empty buffer: {tr:7.2f} ms (rc {rc}), unregister {tu:6.2f} ms (rc {rc2})", flush=True)
        hold.append(b)
    del hold
    d = zk.DeviceBuffer(x)
    res = np.zeros_like(x)
    res.fill(1)
    lib = zk.load()
    for name in ("fresh", "populated", "resident"):
        b = res if name == "resident" else np.zeros_like(x)
        if name == "populated":
            populate(b, 8)
        t = ms(lambda: lib.zkg_memcpy_dtoh(b.ctypes.data, d.ptr, x.nbytes))
        print(f"D2H {name:9s}: {t:7.2f} ms", flush=True)
    sg = zk.get_fft_subgroup("bls12_381", m)
    g = sg.gen_array()
    sym = lib.bls12_381_poly_mont_ntt_forward
    sym(m, zk._p(g), zk._p(x), zk._p(res))  # warm
    keep = []
    for _ in range(3):
        b = np.zeros_like(x)
        keep.append(b)
        print(f"ntt_forward fresh output   : {ms(lambda: sym(m, zk._p(g), zk._p(x), zk._p(b))):7.2f} ms", flush=True)
    for _ in range(3):
        print(f"ntt_forward resident output: {ms(lambda: sym(m, zk._p(g), zk._p(x), zk._p(res))):7.2f} ms", flush=True)
    b = np.zeros_like(x)
    tp, _ = populate(b, 8)
    print(f"ntt_forward populated first ({tp:.1f} ms populate): "
          f"{ms(lambda: sym(m, zk._p(g), zk._p(x), zk._p(b))):7.2f} ms", flush=True)
    for name, alloc in (("np.zeros_like", np.zeros_like), ("np.empty_like", np.empty_like)):
        for _ in range(2):
            t = time.perf_counter()
            b = alloc(x)
            ta = (time.perf_counter() - t) * 1e3
            keep.append(b)
            tc = ms(lambda: sym(m, zk._p(g), zk._p(x), zk._p(b)))
            print(f"{name}: alloc {ta:7.2f} ms, then ntt_forward into it {tc:7.2f} ms", flush=True)
    for _ in range(2):
        print(f"zk.forward_ntt (wrapper, empty output): {ms(lambda: keep.append(zk.forward_ntt(sg, x))):7.2f} ms",
              flush=True)


if __name__ == "__main__":
    main()
