#!/usr/bin/env python3
"""Time each codec stage in isolation over a sweep of batch sizes, to separate
the latency floor of the per-record kernels from their throughput slope.
Prints one JSON line per (records, variant) with the median microseconds of
every stage and ns/record."""
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

P = lambda t: t.data_ptr()  # noqa: E731


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="small")
    ap.add_argument("--sizes", default="4096,16384,65536,262144")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--params", default="", help="name=value,... ctx params")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sizes = [int(x) for x in a.sizes.split(",")]
    N = max(sizes)
    codec = Codec(0, N)
    L, c = codec.lib, codec.ctx
    for kv in filter(None, a.params.split(",")):
        k, v = kv.split("=")
        _lib.check(L.honu_ctx_set_param(c, k.encode(), int(v)), "param")
    meta, var, acl, reg, off = gen_meta(1, a.shape, 0, N)

    def D(x):
        x = np.ascontiguousarray(x)
        t = torch.empty(max(x.nbytes, 16), dtype=torch.uint8, device=dev)
        if x.nbytes:
            t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
        return t
    dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(off)
    s = torch.cuda.current_stream().cuda_stream
    pay = torch.empty(int(off[N]) + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_gen_payload(c, 1, 0, N, P(do), P(pay), s), "gen")
    out_off = torch.empty(8 * (N + 1), dtype=torch.uint8, device=dev)
    st = torch.empty(4 * N + 16, dtype=torch.uint8, device=dev)
    cap = int(off[N]) + 4096 * N
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    dmeta = torch.empty(352 * N, dtype=torch.uint8, device=dev)
    dinfo = torch.empty(32 * N, dtype=torch.uint8, device=dev)
    acl_cap = int(meta["acl_count"].astype(np.int64).sum()) + 1
    reg_cap = int(meta["regions_count"].astype(np.int64).sum()) + 1
    dacl = torch.empty(20 * acl_cap, dtype=torch.uint8, device=dev)
    dreg = torch.empty(4 * reg_cap, dtype=torch.uint8, device=dev)
    data = torch.empty(int(off[N]) + 16 * N + 16, dtype=torch.uint8, device=dev)
    tot = torch.empty(32, dtype=torch.uint8, device=dev)
    for v in map(int, a.variants.split(",")):
        _lib.check(L.honu_ctx_set_param(c, b"record_variant", v), "p")
        for n in sizes:
            stages = {
                "sizes": lambda: L.honu_encode_sizes(c, P(dm), len(var), P(da), len(acl), P(dr),
                                                     len(reg), P(do), n, P(out_off), P(st), s),
                "scan": lambda: L.honu_exclusive_scan(c, P(out_off), n, P(out_off), s),
                "encode_meta": lambda: L.honu_encode_records(c, P(dm), P(dv), P(da), P(dr), P(do), n,
                                                             P(out), cap, P(out_off), P(st), s),
                "encode_copy": lambda: L.honu_encode_payloads(c, P(pay), P(do), n, P(out), cap,
                                                              P(out_off), P(st), s),
                "parse": lambda: L.honu_decode_parse(c, P(out), P(out_off), n, P(dmeta), P(dinfo), s),
                "tables": lambda: L.honu_decode_tables(c, P(out), n, P(dmeta), P(dinfo), P(dacl),
                                                       acl_cap, P(dreg), reg_cap, P(data),
                                                       data.numel(), P(tot), s),
                "decode_copy": lambda: L.honu_decode_payloads(c, P(out), n, P(dinfo), P(data),
                                                              P(tot), s),
                # single-launch decode (fused.hip): zero-copy, then materialising
                "fused_zc": lambda: L.honu_decode_records(c, P(out), P(out_off), n, P(dmeta), P(dinfo),
                                                          P(dacl), acl_cap, P(dreg), reg_cap, 0, 0,
                                                          P(tot), s),
                "fused_mat": lambda: L.honu_decode_records(c, P(out), P(out_off), n, P(dmeta),
                                                           P(dinfo), P(dacl), acl_cap, P(dreg),
                                                           reg_cap, 1, data.numel(), P(tot), s),
            }
            times = {k: [] for k in stages}
            for r in range(a.reps + 1):
                for k, fn in stages.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    _lib.check(fn(), k)
                    e1.record()
                    torch.cuda.synchronize()
                    if r:
                        times[k].append(e0.elapsed_time(e1) * 1e3)
            ok = bool((st[: 4 * n].view(torch.int32) == 0).all())
            info = dinfo[: 32 * n].view(torch.int64).view(n, 4)
            ok &= bool((info[:, 2].contiguous().view(torch.int32) == 0).all())
            med = {k: round(statistics.median(t), 1) for k, t in times.items()}
            meta_us = sum(med[k] for k in ("sizes", "scan", "encode_meta", "parse", "tables"))
            print(json.dumps({"records": n, "variant": v, "us": med,
                              "ns_per_record": {k: round(1e3 * t / n, 3) for k, t in med.items()},
                              "metadata_us": round(meta_us, 1), "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
