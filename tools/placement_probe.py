#!/usr/bin/env python3
"""Does the relative placement of the copy's source and destination matter?
One Bench (1M Large); the two output slots are re-allocated with the records
arena and the data arena shifted by each pad (bytes) inside their
allocations, and a round of --steps steps is timed per pad. Rates within one
process are stable to 0.1 %, so differences between pads are placement."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

PADS = [(0, 0), (1 << 20, 0), (0, 1 << 20), (4096, 4096), (2 << 20, 3 << 20), (0, 0),
        (256, 0), (65536, 131072), (0, 0)]


def main():
    sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
    args = bench.parse_args()
    torch.cuda.set_device(0)
    b = bench.Bench(args, 0, 0)
    ncu = torch.cuda.get_device_properties(b.dev).multi_processor_count
    for pad in PADS:
        b.slots = None
        torch.cuda.empty_cache()
        b.slots = [bench.Slot(b.dev, b.C, b.out_cap, b.acl_cap, b.reg_cap, b.data_cap, pad)
                   for _ in range(2)]
        for sl in b.slots:
            b.lib.honu_ctx_set_param(sl.codec.ctx, b"record_blocks", args.meta_blocks * ncu)
            b.lib.honu_ctx_set_param(sl.codec.ctx, b"lane_blocks", b.lane_blocks * ncu)
        b.step()
        torch.cuda.synchronize()
        b.events = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            b.step(timed=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        addr = (b.slots[0].out.data_ptr() & 0xFFFFFFF, b.slots[0].data.data_ptr() & 0xFFFFFFF)
        print(f"pad {pad}: {b.total_rec_bytes / dt / 2**30:.1f} GiB/s  (low bits of out/data {addr[0]:#x} {addr[1]:#x})",
              flush=True)


if __name__ == "__main__":
    main()
