#!/usr/bin/env python3
"""Where does the bench's run-to-run spread come from? Builds one Bench (the
default 1M Large workload) and times several rounds of --steps steps in the
same process; run it in several processes to compare the spread within a
process (same allocations) with the spread between processes."""
import sys
import time
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
    args = bench.parse_args()
    torch.cuda.set_device(0)
    b = bench.Bench(args, 0, 0)
    b.step()
    torch.cuda.synchronize()
    vals = []
    for _ in range(5):
        b.events = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            b.step(timed=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        vals.append(b.total_rec_bytes / dt / 2**30)
    print("rounds GiB/s:", " ".join(f"{v:.1f}" for v in vals), flush=True)


if __name__ == "__main__":
    main()
