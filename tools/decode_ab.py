#!/usr/bin/env python3
"""A/B timing of the zero-copy decode (honu_decode_batch without a data
arena: Object.Metadata() + Data()) across library builds, interleaved: each
`--libs` entry runs in its own child process (HONU_LIB_PATH) over the same
seeded batches, `--rounds` times in alternation, so box-to-box and
process-to-process spread hits every build alike. One JSON line per
(round, lib, workload) with the median of --reps launches.

  python tools/decode_ab.py --libs tools/tmp/base.so,honu_amd/libhonu_codec.so
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from honu_amd import _lib
    from honu_amd.object import Codec
    from honu_amd.workload import gen_meta
    P = lambda t: t.data_ptr()  # noqa: E731
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    out_lines = []
    for wl in a.workloads.split(","):
        shape, n = wl.split(":")
        n = int(n)
        codec = Codec(0, n)
        L, c = codec.lib, codec.ctx
        if a.lane_blocks_per_cu:  # grid of the single-launch decode (workgroups per CU)
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            _lib.check(L.honu_ctx_set_param(c, b"lane_blocks", a.lane_blocks_per_cu * ncu), "param")
        meta, var, acl, reg, off = gen_meta(1, shape, 0, n)

        def D(x):
            x = np.ascontiguousarray(x)
            t = torch.empty(max(x.nbytes, 16), dtype=torch.uint8, device=dev)
            t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
            return t
        dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(off)
        pay = torch.empty(int(off[n]) + 16, dtype=torch.uint8, device=dev)
        _lib.check(L.honu_gen_payload(c, 1, 0, n, P(do), P(pay), s), "gen")
        oo = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
        st = torch.empty(4 * n + 16, dtype=torch.uint8, device=dev)
        _lib.check(L.honu_encode_sizes(c, P(dm), len(var), P(da), len(acl), P(dr), len(reg), P(do),
                                       n, P(oo), P(st), s), "sizes")
        _lib.check(L.honu_exclusive_scan(c, P(oo), n, P(oo), s), "scan")
        total = int(oo.view(torch.int64)[n].item())
        rec = torch.empty(total + 16, dtype=torch.uint8, device=dev)
        _lib.check(L.honu_encode(c, P(dm), P(dv), len(var), P(da), len(acl), P(dr), len(reg),
                                 P(pay), P(do), n, P(rec), total, P(oo), P(st), s), "encode")
        del pay
        acl_cap = int(meta["acl_count"].astype(np.int64).sum()) + 1
        reg_cap = int(meta["regions_count"].astype(np.int64).sum()) + 1
        E = lambda nb: torch.empty(int(nb), dtype=torch.uint8, device=dev)  # noqa: E731
        dmeta, dinfo, dacl, dreg, tot = E(352 * n), E(32 * n), E(20 * acl_cap), E(4 * reg_cap), E(32)
        scrub = E(1 << 30) if a.cold else None
        data_cap = total + 16 * n
        data = E(data_cap) if a.what == "mat" else None

        def once():
            if a.what == "encode":  # header/tail encoder (honu_encode_records), payload copy apart
                _lib.check(L.honu_encode_records(c, P(dm), P(dv), P(da), P(dr), P(do), n, P(rec),
                                                 total, P(oo), P(st), s), "encode_records")
                return
            if a.what == "mat":  # materialising: single-launch decode, then the copy kernel
                _lib.check(L.honu_decode_records(c, P(rec), P(oo), n, P(dmeta), P(dinfo), P(dacl),
                                                 acl_cap, P(dreg), reg_cap, 1, data_cap, P(tot), s), "dec")
                _lib.check(L.honu_decode_payloads(c, P(rec), n, P(dinfo), P(data), P(tot), s), "copy")
                return
            _lib.check(L.honu_decode_batch(c, P(rec), P(oo), n, P(dmeta), P(dinfo), P(dacl), acl_cap,
                                           P(dreg), reg_cap, 0, 0, P(tot), s), "decode")
        once()
        ms = []
        for _ in range(a.reps):
            if scrub is not None:
                scrub.fill_(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            once()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        ms.sort()
        out_lines.append({"what": a.what, "workload": wl, "ms_median": ms[len(ms) // 2], "ms_min": ms[0],
                          "records_per_s": n / (ms[len(ms) // 2] / 1e3)})
        codec.close()
        del rec, dmeta, dinfo, dacl, dreg, scrub, data
        torch.cuda.empty_cache()
    print(json.dumps(out_lines), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--workloads", default="small:1048576,large:61845")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--cold", action="store_true", help="1 GiB write before every launch")
    ap.add_argument("--what", choices=["decode", "encode", "mat"], default="decode",
                    help="decode: zero copy; encode: header/tail encoder; mat: materialising "
                         "decode (single launch + copy kernel)")
    ap.add_argument("--lane-blocks-per-cu", type=int, default=0)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a)
        return
    libs = [x for x in a.libs.split(",") if x]
    for r in range(a.rounds):
        for lib in libs:  # PATH or PATH@K: K workgroups per CU for the single-launch decode
            path, _, lbk = lib.partition("@")
            env = dict(os.environ, HONU_LIB_PATH=os.path.abspath(path))
            cmd = [sys.executable, os.path.abspath(__file__), "--child", "--workloads", a.workloads,
                   "--reps", str(a.reps), "--what", a.what] + (["--cold"] if a.cold else []) + \
                (["--lane-blocks-per-cu", lbk] if lbk else [])
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if p.returncode:
                print(json.dumps({"round": r, "lib": lib, "error": p.stderr[-2000:]}), flush=True)
                sys.exit(p.returncode)
            for x in json.loads(p.stdout.strip().splitlines()[-1]):
                print(json.dumps({"round": r, "lib": lib, **x}), flush=True)


if __name__ == "__main__":
    main()
