#!/usr/bin/env python3
"""Sweep the payload-copy launch geometry / variants on one chunk of records
(interleaved rounds in one process; GB/s = 2 x payload bytes / kernel time)."""
import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from honu_amd import _lib  # noqa: E402
from honu_amd.object import Codec  # noqa: E402
from honu_amd.workload import gen_meta  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=65536)
    ap.add_argument("--shape", default="large")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--blocks", default="1,2,4,8")
    ap.add_argument("--variants", default="0,6,7")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = Codec(0, a.records)
    L, c = codec.lib, codec.ctx
    P = lambda t: t.data_ptr()  # noqa: E731
    meta, var, acl, reg, off = gen_meta(1, a.shape, 0, a.records)

    def D(x):
        x = np.ascontiguousarray(x)
        t = torch.empty(max(x.nbytes, 16), dtype=torch.uint8, device=dev)
        t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
        return t
    dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(off)
    n = a.records
    pay = torch.empty(int(off[n]) + 16, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(L.honu_gen_payload(c, 1, 0, n, P(do), P(pay), s), "gen")
    out_off = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
    st = torch.empty(4 * n, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_encode_sizes(c, P(dm), len(var), P(da), len(acl), P(dr), len(reg), P(do), n,
                                   P(out_off), P(st), s), "sizes")
    _lib.check(L.honu_exclusive_scan(c, P(out_off), n, P(out_off), s), "scan")
    total = int(out_off.view(torch.int64)[n].item())
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_encode(c, P(dm), P(dv), len(var), P(da), len(acl), P(dr), len(reg), P(pay),
                             P(do), n, P(out), total, P(out_off), P(st), s), "encode")
    dmeta = torch.empty(352 * n, dtype=torch.uint8, device=dev)
    dinfo = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    cap = total
    dacl = torch.empty(20 * cap // 16, dtype=torch.uint8, device=dev)
    dreg = torch.empty(4 * cap // 16, dtype=torch.uint8, device=dev)
    data = torch.empty(total + 16 * n, dtype=torch.uint8, device=dev)
    tot = torch.empty(32, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_decode_parse(c, P(out), P(out_off), n, P(dmeta), P(dinfo), s), "parse")
    _lib.check(L.honu_decode_tables(c, P(out), n, P(dmeta), P(dinfo), P(dacl), cap // 16, P(dreg),
                                    cap // 16, P(data), total + 16 * n, P(tot), s), "tables")
    torch.cuda.synchronize()
    nbytes = 2 * int(off[n])
    cfgs = [(b, v) for b in map(int, a.blocks.split(",")) for v in map(int, a.variants.split(","))]
    res = {cfg: ([], []) for cfg in cfgs}
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for _ in range(a.rounds):
        for (b, v) in cfgs:
            _lib.check(L.honu_ctx_set_param(c, b"copy_blocks", b * ncu), "p")
            _lib.check(L.honu_ctx_set_param(c, b"copy_variant", v), "p")
            for k, fn in enumerate((
                lambda: L.honu_encode_payloads(c, P(pay), P(do), n, P(out), out.numel(), P(out_off), P(st), s),
                lambda: L.honu_decode_payloads(c, P(out), n, P(dinfo), P(data), P(tot), s))):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.check(fn(), "copy")
                e1.record()
                torch.cuda.synchronize()
                res[(b, v)][k].append(nbytes / (e0.elapsed_time(e1) / 1e3) / 1e9)
    # memcpy reference of the same byte count
    x = torch.empty(int(off[n]), dtype=torch.uint8, device=dev)
    ref = []
    for _ in range(a.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        data[: x.numel()].copy_(x)
        e1.record()
        torch.cuda.synchronize()
        ref.append(nbytes / (e0.elapsed_time(e1) / 1e3) / 1e9)
    rows = []
    for (b, v), (enc, dec) in res.items():
        rows.append({"blocks_per_cu": b, "variant": v, "enc_med": statistics.median(enc),
                     "dec_med": statistics.median(dec), "enc_max": max(enc), "dec_max": max(dec)})
    rows.sort(key=lambda r: -(r["enc_med"] + r["dec_med"]))
    for r in rows:
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}))
    print(json.dumps({"torch_copy_med": round(statistics.median(ref), 1)}))


if __name__ == "__main__":
    main()
