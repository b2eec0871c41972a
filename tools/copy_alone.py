#!/usr/bin/env python3
"""The materialising decode's payload copy ALONE on the chip, and the part's
own streaming copy at the same bytes, for the counter passes of
tools/copy_attr.sh (attribute the gap between the codec's
decode copy in the pipelined bench step, the same copy alone, and the box's
streaming probe).

One 1M-Large-sized chunk (--records records of --shape, default 61,680 Large:
the bench's chunk) is generated, encoded and decoded once (single-launch
decode, materialising offsets); then honu_decode_payloads is launched --reps
times back to back with nothing beside it, and the library's probe copies
(honu_hbm_probe mode 4: wave ranges with non-temporal loads and stores; mode
2: the same with the default cache policy) move the same number of bytes at
--probe-blocks workgroups per CU. Prints one JSON line: per-launch ms and
GB/s (read + write bytes) of each form, events on the launch stream.

  python tools/copy_alone.py [--records N] [--reps R]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from honu_amd import _lib  # noqa: E402
from honu_amd.object import Codec  # noqa: E402
from honu_amd.workload import gen_meta  # noqa: E402


def P(t):
    return t.data_ptr()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=61680)
    ap.add_argument("--shape", default="large")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--probe-blocks", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = a.records
    meta, var, acl, reg, off = gen_meta(a.seed, a.shape, 0, n)
    E = lambda nb: torch.empty(int(max(nb, 16)), dtype=torch.uint8, device=dev)  # noqa: E731

    def D(x):
        x = np.ascontiguousarray(x)
        t = E(x.nbytes)
        t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
        return t

    c = Codec(0, n)
    L, ctx = c.lib, c.ctx
    s = torch.cuda.current_stream(dev).cuda_stream
    dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(off)
    pay = E(int(off[n]) + 16)
    _lib.check(L.honu_gen_payload(ctx, a.seed, 0, n, P(do), P(pay), s), "gen")
    out_off, st = E(8 * (n + 1)), E(4 * n)
    _lib.check(L.honu_encode_sizes(ctx, P(dm), len(var), P(da), len(acl), P(dr), len(reg), P(do), n,
                                   P(out_off), P(st), s), "sizes")
    _lib.check(L.honu_exclusive_scan(ctx, P(out_off), n, P(out_off), s), "scan")
    total = int(out_off.view(torch.int64)[n].item())
    rec = E(total + 16)
    _lib.check(L.honu_encode(ctx, P(dm), P(dv), len(var), P(da), len(acl), P(dr), len(reg), P(pay), P(do), n,
                             P(rec), total + 16, P(out_off), P(st), s), "encode")
    del pay
    torch.cuda.empty_cache()
    lens = np.diff(off.astype(np.int64))
    data_cap = int(((lens + 15) // 16 * 16).sum()) + 16
    rows, info, tot = E(352 * n), E(32 * n), E(32)
    dacl, dreg, data = E(20 * (len(acl) + 1)), E(4 * (len(reg) + 1)), E(data_cap)
    _lib.check(L.honu_decode_records(ctx, P(rec), P(out_off), n, P(rows), P(info), P(dacl), len(acl) + 1,
                                     P(dreg), len(reg) + 1, 1, data_cap, P(tot), s), "decode")
    copy_bytes = 2 * int(lens.sum())

    def timed(fn, reps):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    res = {"records": n, "shape": a.shape, "reps": a.reps, "copy_bytes": copy_bytes}
    ms = timed(lambda: _lib.check(L.honu_decode_payloads(ctx, P(rec), n, P(info), P(data), P(tot), s),
                                  "payloads"), a.reps)
    res["decode_copy_alone"] = {"ms": ms, "gbs": copy_bytes / ms / 1e6,
                                "kernel": "k_copy_segments<honu::DecodeSegments>"}
    # the probe: the same bytes (half read, half written), 16-byte aligned
    half = copy_bytes // 2 // 16 * 16
    del rows, dacl, dreg
    torch.cuda.empty_cache()
    src, dst = rec[:half], data[:half]
    for mode, name in ((4, "probe_nt_copy"), (2, "probe_copy")):
        ms = timed(lambda: _lib.check(L.honu_hbm_probe(ctx, mode, P(src), P(dst), half, a.probe_blocks, s),
                                      "probe"), a.reps)
        res[name] = {"ms": ms, "gbs": 2 * half / ms / 1e6, "blocks_per_cu": a.probe_blocks,
                     "kernel": f"k_hbm_probe<{mode}>"}
    print(json.dumps(res), flush=True)
    c.close()


if __name__ == "__main__":
    main()
