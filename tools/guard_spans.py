#!/usr/bin/env python3
"""Spans of the single-launch decode's launches in a rocprofv3 kernel trace
(a guarded launch that queues for CUs): for every
k_decode_fused<MODE,...> / k_decode_guard<...> instantiation the count,
median, mean and max duration, and for guarded launches (MODE 2: the
k_decode_guard kernel since round 5) longer than --slow-us the
kernels that ran beside them.

  python tools/guard_spans.py <run_results.db | *_kernel_trace.csv> [--slow-us 20]
"""
import argparse
import collections
import csv
import json
import sqlite3
import statistics


def load(path):
    """[(name, start_ns, end_ns)] sorted by start."""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
        return [(n, int(s), int(e)) for n, s, e in rows]
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(rows, key=lambda x: x[1])


def short(n):
    return n.split("(")[0].replace("void ", "").replace("honu::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--slow-us", type=float, default=20.0)
    a = ap.parse_args()
    rows = load(a.trace)
    spans = collections.defaultdict(list)
    for n, s, e in rows:
        if "k_decode_fused<" in n or "k_decode_guard<" in n:
            spans[short(n)].append((e - s) / 1e3)
    out = {"trace": a.trace, "launches": {}}
    for k, v in sorted(spans.items()):
        out["launches"][k] = {"n": len(v), "median_us": round(statistics.median(v), 1),
                              "mean_us": round(sum(v) / len(v), 1), "max_us": round(max(v), 1)}
    slow = []
    for n, s, e in rows:
        if ("k_decode_fused<2" in n or "k_decode_guard<" in n) and (e - s) / 1e3 > a.slow_us:
            beside = sorted({short(n2) for n2, s2, e2 in rows if s2 < e and e2 > s and (n2, s2) != (n, s)})
            slow.append({"us": round((e - s) / 1e3, 1), "beside": beside})
    out["guards_over_slow_us"] = len(slow)
    out["slow_guards"] = slow[:12]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
