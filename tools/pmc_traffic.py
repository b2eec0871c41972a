#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two rocprofv3 PMC passes
(--pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs of the same command),
corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide
coalesced streaming read (16 B per lane), so it is doubled; WRITE_SIZE is exact
for 16-B-per-lane streaming stores.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV WORKLOAD OUT_JSON
OUT_JSON holds one entry per workload ({"workloads": {WORKLOAD: ...}}); an
existing file is updated in place, so the bench lines of several commands
share it (bench.py reads the entry of its own workload).
"""
import os
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0]
            acc[name].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch_csv, write_csv, workload, out = sys.argv[1:5]
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    res = {"workload": workload, "source": [fetch_csv, write_csv],
           "correction": "bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024",
           # the commit the measured tree was (HONU_COMMIT, set by the caller:
           # the GPU box has no .git), read back by bench.py (roofline.traffic_commit)
           "commit": os.environ.get("HONU_COMMIT"), "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fv, wv = f.get(k, []), w.get(k, [])
        fb = 2 * 1024 * sum(fv) / max(1, len(fv))
        wb = 1024 * sum(wv) / max(1, len(wv))
        res["kernels"][k] = {"launches": max(len(fv), len(wv)), "read_bytes_per_launch": fb,
                             "write_bytes_per_launch": wb, "traffic_per_launch": fb + wb}
    allw = {"workloads": {}}
    if os.path.exists(out):
        old = json.load(open(out))
        allw["workloads"] = old.get("workloads", {})
    allw["workloads"][workload] = res
    json.dump(allw, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k[:60]:60s} {v['traffic_per_launch'] / 1e9:10.3f} GB/launch")


if __name__ == "__main__":
    main()
