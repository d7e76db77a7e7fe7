#!/usr/bin/env python3
"""Brute-force LDS bank-conflict check of the NTT pass kernel's tile swizzle (zk_ntt.hip
lds_slot): for every wave-level access pattern of a pass (bit-reversed tile load, every
radix-4 / radix-2 round, tile store) and each tile shape, the worst number of lanes that hit
one of the 64 banks with 9-word elements.  CPU only:  python tools/ntt_lds_banks.py"""
import itertools, sys
def rev(x, r):
    return int(format(x, f'0{r}b')[::-1], 2) if r else 0
def swz_old(I):
    m1 = (I >> 6) & 3; m2 = (I >> 8) & 3; x = m1 ^ m2
    return I ^ (m1 | (x << 2) | (x << 4))
def swz_new(I):
    m1 = (I >> 6) & 3; m2 = (I >> 8) & 3; m3 = (I >> 10) & 3; x = m1 ^ m2; y = x ^ m3
    return I ^ (m1 | (x << 2) | (y << 4))
def degree(slots):
    b = {}
    for s in slots:
        k = (s * 9) % 64
        b[k] = b.get(k, 0) + 1
    return max(b.values())
def patterns(r, G, NT):
    R = 1 << r
    nel = G * R
    # load (non-last): g = e % G, k = e / G ; last: g = e / R, k = e % R
    for kind in ("nonlast", "last"):
        for base in range(0, nel, NT):
            for w in range(0, NT, 64):
                sl = []
                for lane in range(64):
                    e = base + w + lane
                    if e >= nel: continue
                    if kind == "nonlast": g, k = e % G, e // G
                    else: g, k = e // R, e % R
                    sl.append(g * R + rev(k, r))
                if sl: yield ("load_" + kind, sl)
    # rounds
    q4 = R >> 2
    s = 0
    while s + 1 < r:
        half = 1 << s
        for base in range(0, G * q4, NT):
            for w in range(0, NT, 64):
                for a in range(4):
                    sl = []
                    for lane in range(64):
                        u = base + w + lane
                        if u >= G * q4: continue
                        g, j = u // q4, u % q4
                        if s == 0:
                            i0 = g * R + j * 4; sl.append(i0 + a)
                        else:
                            blk, off = j >> s, j & (half - 1)
                            i0 = g * R + blk * 4 * half + off; sl.append(i0 + a * half)
                    if sl: yield (f"round{s}_a{a}", sl)
        s += 2
    if s < r:  # radix-2
        half = 1 << s
        q2 = R >> 1
        for base in range(0, G * q2, NT):
            for w in range(0, NT, 64):
                for a in range(2):
                    sl = []
                    for lane in range(64):
                        u = base + w + lane
                        if u >= G * q2: continue
                        g, j = u // q2, u % q2
                        blk, off = j >> s, j & (half - 1)
                        sl.append(g * R + blk * 2 * half + off + a * half)
                    if sl: yield (f"r2_{s}_a{a}", sl)
    # store: g = e % G, k = e / G -> slot g*R + k
    for base in range(0, nel, NT):
        for w in range(0, NT, 64):
            sl = [ (e % G) * R + e // G for e in range(base + w, min(base + w + 64, nel))]
            yield ("store", sl)
for name, f in (("bits 6..9 (round 2 early)", swz_old), ("bits 6..11 (lds_slot)", swz_new)):
    for (r, G, NT) in [(8, 4, 256), (7, 8, 256), (6, 16, 256), (9, 8, 1024), (10, 4, 1024), (11, 2, 1024), (12, 1, 1024), (11, 1, 256), (10, 1, 256)]:
        worst = {}
        for kind, sl in patterns(r, G, NT):
            d = degree([f(x) for x in sl])
            k = kind.split("_a")[0]
            worst[k] = max(worst.get(k, 0), d)
        print(name, (r, G, NT), max(worst.values()), {k: v for k, v in worst.items() if v > 1})
