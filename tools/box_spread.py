#!/usr/bin/env python3
"""Box-to-box spread of the default bench line: one directory per fresh GPU
box (each gpurun call takes a new one), each holding bench_default.json and
bench_small.json; prints one row per box and the range of every column.

  python tools/box_spread.py profiles/r04/box_spread/box*
"""
import json
import sys


def last_json(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def row(d):
    big = last_json(d + "/bench_default.json")
    rl = big["roofline"]
    zc = big.get("decode", {}).get("zero_copy")
    zc_rps = zc.get("records_per_s") if isinstance(zc, dict) else None
    probe = big.get("kernels", {}).get("hbm_probe", {})
    out = {"box": d.rstrip("/").split("/")[-1], "large_gibs": big["value"], "large_ms": big["ms_per_step"],
           "frac": rl["frac"], "frac_of_achievable": rl.get("frac_of_achievable"),
           "probe_copy_gbs": probe.get("copy_gbs"), "zero_copy_grec_s": zc_rps and zc_rps / 1e9,
           "verified": big.get("verified")}
    try:
        small = last_json(d + "/bench_small.json")
        out.update(small_gibs=small["value"], small_ms=small["ms_per_step"])
    except (OSError, ValueError):
        pass
    return out


def main(dirs):
    rows = [row(d) for d in dirs]
    cols = [k for k in rows[0] if k != "box"]
    print("\t".join(["box"] + cols))
    for r in rows:
        print("\t".join([r["box"]] + [f"{r.get(k):.4g}" if isinstance(r.get(k), float) else str(r.get(k))
                                      for k in cols]))
    for k in cols:
        v = [r[k] for r in rows if isinstance(r.get(k), (int, float)) and not isinstance(r.get(k), bool)]
        if v:
            print(f"# {k}: {min(v):.4g} .. {max(v):.4g} over {len(v)} boxes")


if __name__ == "__main__":
    main(sys.argv[1:])
