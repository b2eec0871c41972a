#!/usr/bin/env python3
"""Median-per-round summary of tools/decode_ab.py output: one line per
(workload, lib) with the per-round medians in microseconds."""
import collections
import json
import sys

r = collections.defaultdict(list)
for line in open(sys.argv[1]):
    d = json.loads(line)
    if "error" in d:
        print(d)
        continue
    r[(d["workload"], d["lib"].split("/")[-1])].append(round(d["ms_median"] * 1000, 1))
for k, v in sorted(r.items()):
    print(f"{k[0]:>16} {k[1]:>14} " + " ".join(f"{x:8.1f}" for x in v))
