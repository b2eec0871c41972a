#!/usr/bin/env python3
"""Timed launches of `bench.py --mode decode` cut out of its rocprofv3 kernel
trace, so the committed stats reproduce the line's rooflines:

  zero copy      k_decode_fused launches over the whole batch: the first is the
                 untimed warm-up, the next `reps` are timed (bench.py
                 DecodeBench.zero_copy: max(3, steps) reps)
  materialising  k_copy_segments<DecodeSegments>: `warmup` untimed passes of C
                 chunk launches, then `steps` timed passes, then the untimed
                 verification pass (whose digest kernels run beside it)

usage: python tools/decode_timed_stats.py KERNEL_TRACE.csv BENCH.json
Prints one JSON object: per leg the launches taken, their average duration
and the roofline recomputed from it (algorithmic bytes from the bench line).
"""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1:3]
    b = json.load(open(bench))
    d = b["decode"]
    with open(trace, newline="") as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # noqa: E731
    out = {"bench": bench}
    g = [r for r in rows if "k_decode_fused<2" in r["Kernel_Name"] or "k_decode_guard" in r["Kernel_Name"]]
    if g:
        out["guarded_launches"] = {"count": len(g),
                                   "avg_us": sum(dur(r) for r in g) / len(g) * 1e3}
    zc = d.get("zero_copy")
    if zc:
        # the speculative launches (k_decode_fused<1>; each is followed by a
        # guarded <2> that returns at once), else the plain ones (<0>)
        fused = [r for r in rows if "k_decode_fused<1" in r["Kernel_Name"]] or \
            [r for r in rows if "k_decode_fused<0" in r["Kernel_Name"]]
        reps = zc["reps"]
        timed = fused[1:1 + reps]
        ms = sum(dur(r) for r in timed) / len(timed)
        alg = zc["roofline"]["algorithmic_bytes_per_launch"]
        out["zero_copy"] = {"kernel": "k_decode_fused", "launches": len(timed),
                            "avg_ms_trace": ms, "avg_ms_events": zc["ms"],
                            "achieved_gbs": alg / ms / 1e6, "frac": alg / ms / 1e6 / 8000.0}
    mat = d.get("materialising")
    if mat:
        copies = [r for r in rows if "k_copy_segments<honu::DecodeSegments" in r["Kernel_Name"]]
        C, W, K = mat["chunks"], b["warmup"], mat["steps"]
        timed = copies[W * C:(W + K) * C]
        ms = sum(dur(r) for r in timed) / len(timed)
        alg = mat["roofline"]["algorithmic_bytes_per_launch"]
        out["materialising"] = {"kernel": "k_copy_segments<DecodeSegments>", "launches": len(timed),
                                "avg_ms_trace": ms, "avg_ms_events": mat["roofline"]["avg_launch_ms"],
                                "achieved_gbs": alg / ms / 1e6, "frac": alg / ms / 1e6 / 8000.0}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
