#!/usr/bin/env python3
"""One line per bench JSON of an A/B directory (profiles/r05/pipeline_ab/box*):
ms per step, GiB/s, the dominant copy's roofline.frac and the whole step's
algorithmic HBM rate as a fraction of the 8 TB/s spec, verified.

  python tools/pipeline_ab_summary.py profiles/r05/pipeline_ab/boxH
"""
import glob
import json
import os
import sys


def main():
    for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        if "ms_per_step" not in d:
            continue
        k = d.get("kernels", {})
        step = k.get("step_hbm_gbs_algorithmic")
        print(f"{os.path.basename(f):28s} {d['ms_per_step']:8.3f} ms {d['value']:8.1f} GiB/s "
              f"frac {d['roofline']['frac']:.3f} step {step / 8000 if step else float('nan'):.3f} "
              f"verified {d.get('verified')}")


if __name__ == "__main__":
    main()
