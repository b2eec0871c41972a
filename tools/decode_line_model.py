#!/usr/bin/env python3
"""Line model of the single-launch decode's reads.

For records of the generator (CPU: oracle marshal + decode of the default
forms), lists the 128-byte lines each phase of the walk (win.h win_walk)
touches: the tile head's header blocks, window 1 at the tail's start, the ACL
flag burst, window 2 after the list, direct reads past window 2, window 3
after the signature. `sum` counts a line once per phase (every phase fetches
its lines again: the L2 kept nothing between phases), `union` once per record
(perfect reuse); the measured read bytes per record (PMC, 1.625 GB / 1M) lie
between them, near `sum`. Pairwise overlaps name the lines fetched twice.

  python tools/decode_line_model.py [--n 4000] [--align 64] [--skip-window-flags] [--skip-window2-flags]

(The model has no cache: the nt policy of the window refills and bursts,
which lets the L2 keep the tile head's lines, is outside it.)
"""
import argparse
import itertools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = 128


def lines(a, b):
    return set(range(a // L, (b - 1) // L + 1)) if b > a else set()


def uvlen(x):
    k = 1
    while x >= 128:
        x >>= 7
        k += 1
    return k


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4000)
    ap.add_argument("--shape", default="small")
    ap.add_argument("--align", type=int, default=16, help="window base alignment (HONU_WIN_ALIGN)")
    ap.add_argument("--skip-window-flags", action="store_true",
                    help="the burst skips the flags window 1 holds (HONU_GATHER_SKIP_WIN)")
    ap.add_argument("--skip-window2-flags", action="store_true",
                    help="... and the last ones window 2 holds (HONU_GATHER_SKIP_WIN2)")
    a = ap.parse_args()
    from oracle import oracle as O
    from honu_amd.workload import gen_host_batch
    hb = gen_host_batch(1, a.shape, 0, a.n)
    rec, off, _ = O.marshal_batch(hb)
    meta, info, _, _, _, _ = O.decode_batch(rec, off)
    base = lambda p: p & ~(a.align - 1)  # noqa: E731
    phases = ["head", "w1", "acl", "w2", "direct2", "w3"]
    tot = dict.fromkeys(phases, 0)
    uni = need = 0
    per = []
    for i in range(a.n):
        beg, end = int(off[i]), int(off[i + 1])
        m, inf = meta[i], info[i]
        tstart = int(inf["data_off"]) + int(inf["data_len"]) if int(inf["data_len"]) else beg + 2
        S = {}
        A = beg & ~15
        S["head"] = lines(A, A + 16) | (lines(A + 16, A + 32) if (beg & 15) > 5 and A + 16 < end else set())
        w1 = base(tstart)
        S["w1"] = lines(w1, min(w1 + 256, end))
        na, ap_ = int(m["acl_count"]), int(m["acl_off"])
        S["acl"] = set()
        if na:
            j0 = 0
            if a.skip_window_flags and ap_ < w1 + 256:
                j0 = min(na, (w1 + 256 - ap_ + 17) // 18)
            j1 = na
            if a.skip_window2_flags:
                w2b = base(ap_ + 18 * na)
                j1 = max(j0, min(na, (w2b - ap_ + 17) // 18)) if w2b > ap_ else j0
            for j in range(j0, min(j1, j0 + 64)):
                q = (ap_ + 18 * j) & ~3
                S["acl"] |= lines(q, q + 4)
            p2 = ap_ + 18 * na
        else:
            nr = int(m["regions_count"])
            p2 = int(m["regions_off"]) - uvlen(nr) if nr else w1 + 200
        w2 = base(p2)
        S["w2"] = lines(w2, min(w2 + 256, end))
        so, sl = int(m["signature"]["off"]), int(m["signature"]["len"])
        if sl:
            S["direct2"] = lines(w2 + 256, so) if so > w2 + 256 else set()
            p3 = so + sl
        else:
            S["direct2"] = set()
            p3 = end - 40
        w3 = base(p3)
        S["w3"] = lines(w3, min(w3 + 256, end))
        U = set()
        for k, v in S.items():
            tot[k] += len(v) * L
            U |= v
        uni += len(U) * L
        need += end - tstart + 16
        per.append(S)
    ov = {}
    for i, S in enumerate(per):
        for x, y in itertools.combinations(phases, 2):
            ov[f"{x}&{y}"] = ov.get(f"{x}&{y}", 0) + len(S[x] & S[y]) * L
        if i + 1 < len(per):
            for x in ("w2", "w3"):
                ov[f"{x}&next head"] = ov.get(f"{x}&next head", 0) + len(S[x] & per[i + 1]["head"]) * L
    n = a.n
    print("bytes per record by phase:", {k: round(v / n) for k, v in tot.items()})
    print(f"sum {sum(tot.values()) / n:.0f} + 8 (offsets)  union {uni / n:.0f}  tail + header bytes {need / n:.0f}")
    print("lines fetched by two phases (bytes per record):", {k: round(v / n) for k, v in ov.items() if v})


if __name__ == "__main__":
    main()
