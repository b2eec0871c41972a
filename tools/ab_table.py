#!/usr/bin/env python3
"""Summary of tools/r06_ab.sh runs: per tag, the runs' ms_per_step (or a
dotted key path, e.g. decode.zero_copy.ms) in run order, mean and range.
usage: tools/ab_table.py OUT/ab.jsonl [key.path]"""
import collections
import json
import sys


def get(d, path):
    for k in path.split("."):
        d = d[k]
    return d


def main():
    path = sys.argv[2] if len(sys.argv) > 2 else "ms_per_step"
    by = collections.defaultdict(list)
    for ln in open(sys.argv[1]):
        if ln.strip():
            r = json.loads(ln)
            by[r["tag"]].append(get(r["line"], path))
    for tag, v in by.items():
        print(f"{tag:24s} n={len(v)} mean={sum(v) / len(v):.4f} min={min(v):.4f} max={max(v):.4f} "
              f"runs={[round(x, 4) for x in v]}")


if __name__ == "__main__":
    main()
