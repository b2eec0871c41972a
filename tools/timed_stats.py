"""Per-kernel statistics of a bench run's TIMED steps only, from the
rocprofv3 kernel trace of that run.

`rocprofv3 --kernel-trace --stats` summarises every launch of the process:
the warmup step, the timed steps, and the untimed verification step, whose
digest and row-check kernels run beside the next chunk's payload copies and
slow them (up to 5.5 ms against 4.0-4.4 ms per 1M-Large copy launch). The
bench line's `roofline.avg_launch_ms` covers the timed steps only, so this
tool cuts the same window out of the trace:

  window start = end of the last warmup decode copy (the timed region starts
                 after a barrier + synchronize that follow it), or the trace
                 start when warmup = 0
  window end   = end of the last timed decode copy

Each step launches exactly one encode copy and one decode copy per chunk, so
the decode-copy launch index bounds the window: launches [W*C, (W+K)*C).

usage: python tools/timed_stats.py KERNEL_TRACE.csv BENCH.json [OUT.csv]
Prints the roofline of the dominant kernel recomputed from the trace, and
writes the stats (rocprofv3 --stats column layout) to OUT.csv when given.
"""
import csv
import json
import statistics
import sys

DEC = "k_copy_segments<honu::DecodeSegments"
ENC = "k_copy_segments<honu::EncodeSegments"


def load(path):
    with open(path, newline="") as f:
        rows = list(csv.DictReader(f))
    ks = []
    for r in rows:
        ks.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    ks.sort(key=lambda k: k[1])
    return ks


def window(ks, warmup, steps, chunks):
    dec = [k for k in ks if DEC in k[0]]
    need = (warmup + steps) * chunks
    if len(dec) < need:
        raise SystemExit(f"trace holds {len(dec)} decode copies, the run needs {need}")
    t0 = dec[warmup * chunks - 1][2] if warmup else ks[0][1]
    t1 = dec[need - 1][2]
    return t0, t1


def stats(ks, t0, t1):
    by = {}
    for name, s, e in ks:
        if s >= t0 and e <= t1:
            by.setdefault(name, []).append(e - s)
    tot = sum(sum(v) for v in by.values())
    out = []
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        out.append({"Name": name, "Calls": len(d), "TotalDurationNs": sum(d),
                    "AverageNs": sum(d) / len(d), "Percentage": 100.0 * sum(d) / tot,
                    "MinNs": min(d), "MaxNs": max(d),
                    "StdDev": statistics.pstdev(d) if len(d) > 1 else 0.0})
    return out


def main(argv):
    trace, bench_json = argv[0], argv[1]
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    chunks = b["config"]["chunks"]
    ks = load(trace)
    t0, t1 = window(ks, b["warmup"], b["steps"], chunks)
    st = stats(ks, t0, t1)
    if len(argv) > 2:
        with open(argv[2], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0].keys()), quoting=csv.QUOTE_NONNUMERIC)
            w.writeheader()
            w.writerows(st)
    rl = b["roofline"]
    alg = rl["algorithmic_bytes_per_launch"]
    print(f"timed window {(t1 - t0) / 1e6:.3f} ms = {(t1 - t0) / 1e6 / b['steps']:.3f} ms/step "
          f"(bench under the profiler: {b['ms_per_step']:.3f} ms/step)")
    for key in (ENC, DEC):
        for r in st:
            if key in r["Name"]:
                gbs = alg / r["AverageNs"]
                print(f"{key}: {r['Calls']} launches, avg {r['AverageNs'] / 1e6:.3f} ms, "
                      f"{gbs:.1f} GB/s algorithmic = {gbs / rl['peak']:.3f} of {rl['peak']:.0f}")
    dom = st[0]
    print(f"dominant by time: {dom['Name'][:80]} ({dom['Percentage']:.1f} %)")


if __name__ == "__main__":
    main(sys.argv[1:])
