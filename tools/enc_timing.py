#!/usr/bin/env python3
"""Where one wave's header/tail encode (k_encode_meta_lane) spends its time:
stage timestamps recorded by lane 0 of every wave (timing build: make -C
honu_amd EXTRA=-DHONU_ENC_TIMING, loaded with HONU_LIB_PATH). Runs
honu_encode_records on a sized batch and prints the median and p90 of every
stage over the waves, in microseconds (100 MHz clock)."""
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

STAGES = ["row_load", "header_to_mime", "owner_to_acl_count", "acl_ends", "regions",
          "publisher", "encryption_to_end"]
NST = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="large")
    ap.add_argument("--records", type=int, default=61845)
    ap.add_argument("--no-stamps", action="store_true",
                    help="only run the encodes (counter passes on a non-timing build)")
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
    for _ in range(3):
        _lib.check(L.honu_encode_records(c, P(dm), P(dv), P(da), P(dr), P(do), n, P(out), total,
                                         P(out_off), P(st), s), "records")
    torch.cuda.synchronize()
    if a.no_stamps:
        return
    waves = min((n + 63) // 64, 1 << 16)
    buf = np.zeros((waves, NST), np.uint64)
    fn = L.honu_debug_enc_stamps
    fn.restype = C.c_int32
    fn.argtypes = [C.c_void_p, C.c_uint64]
    assert fn(buf.ctypes.data, waves) == 0
    t = buf.astype(np.int64)
    t0 = t[:, 0].min()
    t = t[t[:, 7] > 0]  # waves whose lane 0 encoded a record
    res = {"shape": a.shape, "records": n, "waves": int(len(t)),
           "last_wave_end_us": float((t[:, 7].max() - t0) / 100)}
    for k, name in enumerate(STAGES):
        d = (t[:, k + 1] - t[:, k]) / 100.0
        res[name] = {"median_us": float(np.median(d)), "p90_us": float(np.percentile(d, 90))}
    res["total"] = {"median_us": float(np.median((t[:, 7] - t[:, 0]) / 100.0))}
    res["start_spread_us"] = float((np.percentile(t[:, 0], 90) - t0) / 100)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
