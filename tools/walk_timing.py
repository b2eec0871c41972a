#!/usr/bin/env python3
"""Where one wave's Metadata walk spends its time: stage timestamps recorded by
lane 0 of every wave (timing build: make -C honu_amd EXTRA=-DHONU_WALK_TIMING,
copied to a separate path and loaded with HONU_LIB_PATH). Runs the split parse
(honu_decode_parse) once on an encoded batch and prints the median and p90 of
every stage over the waves, in microseconds (100 MHz clock)."""
import argparse
import ctypes as C
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

STAGES = ["rec_off", "header", "window1", "to_acl_count", "acl_flags", "window_after_acl",
          "regions_to_sig", "window_after_sig", "tail_end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="large")
    ap.add_argument("--records", type=int, default=61845)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = a.records
    codec = Codec(0, n)
    L, c = codec.lib, codec.ctx
    P = lambda t: t.data_ptr()  # noqa: E731
    meta, var, acl, reg, off = gen_meta(1, a.shape, 0, n)

    def D(x):
        x = np.ascontiguousarray(x)
        t = torch.empty(max(x.nbytes, 16), dtype=torch.uint8, device=dev)
        t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
        return t
    dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(off)
    s = torch.cuda.current_stream().cuda_stream
    pay = torch.empty(int(off[n]) + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_gen_payload(c, 1, 0, n, P(do), P(pay), s), "gen")
    out_off = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
    st = torch.empty(4 * n + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_encode_sizes(c, P(dm), len(var), P(da), len(acl), P(dr), len(reg), P(do), n,
                                   P(out_off), P(st), s), "sizes")
    _lib.check(L.honu_exclusive_scan(c, P(out_off), n, P(out_off), s), "scan")
    total = int(out_off.view(torch.int64)[n].item())
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_encode(c, P(dm), P(dv), len(var), P(da), len(acl), P(dr), len(reg), P(pay),
                             P(do), n, P(out), total, P(out_off), P(st), s), "encode")
    dmeta = torch.empty(352 * n, dtype=torch.uint8, device=dev)
    dinfo = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    for _ in range(3):
        _lib.check(L.honu_decode_parse(c, P(out), P(out_off), n, P(dmeta), P(dinfo), s), "parse")
    torch.cuda.synchronize()
    waves = min((n + 63) // 64, 1 << 16)
    buf = np.zeros((waves, 10), np.uint64)
    fn = L.honu_debug_walk_stamps
    fn.restype = C.c_int32
    fn.argtypes = [C.c_void_p, C.c_uint64]
    assert fn(buf.ctypes.data, waves) == 0
    t = buf.astype(np.int64)
    t0 = t[:, 0].min()
    res = {"shape": a.shape, "records": n, "waves": waves,
           "first_wave_start_us": 0.0, "last_wave_end_us": float((t[:, 9].max() - t0) / 100)}
    for k, name in enumerate(STAGES):
        d = (t[:, k + 1] - t[:, k]) / 100.0
        res[name] = {"median_us": float(np.median(d)), "p90_us": float(np.percentile(d, 90))}
    res["walk_total"] = {"median_us": float(np.median((t[:, 9] - t[:, 0]) / 100.0))}
    res["start_spread_us"] = float((np.percentile(t[:, 0], 90) - t0) / 100)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
