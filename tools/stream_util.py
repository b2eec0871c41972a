#!/usr/bin/env python3
"""How busy each hardware queue of a bench run is inside its timed steps, from
a rocprofv3 kernel trace (csv): the window is the last --steps x chunks copy
launches on the copy queue (the queue that runs k_copy_segments); per queue
the busy time (union of its kernels' spans) and the share of the window, and
for the copy queue its idle gaps with the kernel it waited for (the last one
to end on another queue before the next copy started).

  python tools/stream_util.py run_kernel_trace.csv --copies 40
"""
import argparse
import collections
import csv
import json


def short(n):
    return n.split("(")[0].replace("void ", "").replace("honu::", "")


def union(spans):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(spans):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--copies", type=int, required=True,
                    help="copy launches in the timed steps (steps x chunks x copies per chunk)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                         short(r["Kernel_Name"])))
    rows.sort()
    copies = [x for x in rows if x[3].startswith("k_copy_segments")]
    cq = collections.Counter(x[2] for x in copies).most_common(1)[0][0]
    timed = [x for x in copies if x[2] == cq][-a.copies:]
    w0, w1 = timed[0][0], timed[-1][1]
    inwin = [x for x in rows if x[1] > w0 and x[0] < w1]
    out = {"window_ms": (w1 - w0) / 1e6, "copy_queue": cq, "queues": {}}
    for q in sorted({x[2] for x in inwin}):
        spans = [(max(s, w0), min(e, w1)) for s, e, qq, _ in inwin if qq == q]
        kern = collections.Counter(n for s, e, qq, n in inwin if qq == q)
        out["queues"][q] = {"busy_ms": union(spans) / 1e6, "busy_frac": union(spans) / (w1 - w0),
                            "kernels": dict(kern.most_common(8))}
    gaps = []
    for prev, nxt in zip(timed, timed[1:]):
        g = nxt[0] - prev[1]
        if g > 20000:  # > 20 us
            before = [x for x in inwin if x[2] != cq and x[1] <= nxt[0]]
            last = max(before, key=lambda x: x[1]) if before else None
            gaps.append({"us": round(g / 1e3, 1), "after": prev[3][:40], "before": nxt[3][:40],
                         "waited_for": (last[3][:40], last[2]) if last else None})
    out["copy_gaps_over_20us"] = len(gaps)
    out["copy_gap_ms_total"] = sum(x["us"] for x in gaps) / 1e3
    out["gaps"] = gaps[:12]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
