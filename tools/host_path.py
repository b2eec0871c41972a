#!/usr/bin/env python3
"""Host-inclusive codec rate: records start and end in host memory (Honu's
bbolt pages / replication socket), so this times pinned host -> device copies,
the codec and device -> host copies, pipelined over three HIP streams (H2D,
codec, D2H) with two device slots. Reported in DESIGN.md next to the
device-resident bench; never the bench `value`.

  encode: H2D(rows, CSR payload offsets, payload) -> marshal -> D2H(records)
  decode: H2D(records, record offsets) -> decode, materialising -> D2H(rows, data)
The small tables (var arena, ACL and region tables) are uploaded once.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from honu_amd import _lib  # noqa: E402
from honu_amd.object import Codec  # noqa: E402
from honu_amd.workload import gen_meta  # noqa: E402

P = lambda t: t.data_ptr()  # noqa: E731


def pinned(nbytes):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, pin_memory=True)


def dev(nbytes, d):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=d)


def measure(shape="large", records=65536, chunk=4096, reps=3, device=0, first=0):
    """Host-path encode and decode rates of records [first, first + records)
    of the seed-1 synthetic batch on cuda:device (one JSON-able dict)."""
    d = torch.device("cuda", device)
    N, C = records, chunk
    meta, var, acl, reg, off = gen_meta(1, shape, first, N)
    off64 = off.astype(np.int64)
    chunks = [(s, min(s + C, N)) for s in range(0, N, C)]
    rng = np.random.default_rng(1)

    h_meta = pinned(meta.nbytes)
    h_meta.numpy()[: meta.nbytes] = meta.view(np.uint8)
    pay_n = int(off[N])
    h_pay = pinned(pay_n)
    # payload bytes do not change the codec's work: a random 1 MiB block, tiled
    blk = torch.from_numpy(rng.integers(0, 256, 1 << 20, dtype=np.uint8))
    hv = h_pay[:pay_n]
    for o in range(0, pay_n, 1 << 20):
        hv[o:o + (1 << 20)].copy_(blk[: min(1 << 20, pay_n - o)])
    h_poff = []  # per-chunk relative payload offsets, pinned
    for s, e in chunks:
        t = pinned(8 * (e - s + 1))
        t.numpy()[: 8 * (e - s + 1)] = (off64[s:e + 1] - off64[s]).astype(np.uint64).view(np.uint8)
        h_poff.append(t)

    def up(arr):
        t = dev(arr.nbytes, d)
        if arr.nbytes:
            t[: arr.nbytes].copy_(torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1)))
        return t
    d_var, d_acl, d_reg = up(var), up(acl), up(reg)

    lens = np.diff(off64)
    cmax = max(int(lens[s:e].sum()) for s, e in chunks)
    acl_cap = max(int(meta["acl_count"][s:e].sum()) for s, e in chunks) + 1
    reg_cap = max(int(meta["regions_count"][s:e].sum()) for s, e in chunks) + 1
    slots = []
    for _ in range(2):
        slots.append({
            "codec": Codec(device, C), "meta": dev(352 * C, d), "poff": dev(8 * (C + 1), d),
            "pay": dev(cmax, d), "roff": dev(8 * (C + 1), d), "st": dev(4 * C, d),
            "rec": dev(cmax + 2048 * C, d), "dmeta": dev(352 * C, d), "dinfo": dev(32 * C, d),
            "dacl": dev(20 * acl_cap, d), "dreg": dev(4 * reg_cap, d), "data": dev(cmax + 16 * C, d),
            "tot": dev(32, d), "done": None})

    # untimed sizing pass: exact record bytes and offsets per chunk (host copies)
    h_roff, rec_bytes = [], []
    sl = slots[0]
    for k, (s, e) in enumerate(chunks):
        n = e - s
        L, c = sl["codec"].lib, sl["codec"].ctx
        sl["meta"][: 352 * n].copy_(h_meta[352 * s:352 * e])
        sl["poff"][: 8 * (n + 1)].copy_(h_poff[k][: 8 * (n + 1)])
        _lib.check(L.honu_encode_sizes(c, P(sl["meta"]), len(var), P(d_acl), len(acl), P(d_reg),
                                       len(reg), P(sl["poff"]), n, P(sl["roff"]), P(sl["st"]), 0), "sz")
        _lib.check(L.honu_exclusive_scan(c, P(sl["roff"]), n, P(sl["roff"]), 0), "scan")
        t = pinned(8 * (n + 1))
        t[: 8 * (n + 1)].copy_(sl["roff"][: 8 * (n + 1)])
        h_roff.append(t)
        rec_bytes.append(int(t[: 8 * (n + 1)].view(torch.int64)[n].item()))
    rec_pos = np.concatenate([[0], np.cumsum(rec_bytes)])
    h_rec = pinned(int(rec_pos[-1]))
    h_rows = pinned(352 * N)
    dcap = max(int(((lens[s:e] + 15) // 16 * 16).sum()) for s, e in chunks)
    h_data = [pinned(dcap) for _ in range(2)]
    s_in, s_k, s_out = (torch.cuda.Stream(d) for _ in range(3))

    def run(encode):
        for sl in slots:
            sl["done"] = None
        for k, (s, e) in enumerate(chunks):
            n = e - s
            sl = slots[k % 2]
            L, c = sl["codec"].lib, sl["codec"].ctx
            r0, r1 = int(rec_pos[k]), int(rec_pos[k + 1])
            with torch.cuda.stream(s_in):
                if sl["done"] is not None:
                    s_in.wait_event(sl["done"])
                if encode:
                    p0, p1 = int(off64[s]), int(off64[e])
                    sl["meta"][: 352 * n].copy_(h_meta[352 * s:352 * e], non_blocking=True)
                    sl["poff"][: 8 * (n + 1)].copy_(h_poff[k][: 8 * (n + 1)], non_blocking=True)
                    sl["pay"][: p1 - p0].copy_(h_pay[p0:p1], non_blocking=True)
                else:
                    sl["rec"][: r1 - r0].copy_(h_rec[r0:r1], non_blocking=True)
                    sl["roff"][: 8 * (n + 1)].copy_(h_roff[k][: 8 * (n + 1)], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s_in)
            s_k.wait_event(ev)
            ks = s_k.cuda_stream
            if encode:
                _lib.check(L.honu_marshal_batch(c, P(sl["meta"]), P(d_var), len(var), P(d_acl),
                                                len(acl), P(d_reg), len(reg), P(sl["pay"]),
                                                P(sl["poff"]), n, P(sl["rec"]), r1 - r0,
                                                P(sl["roff"]), P(sl["st"]), ks), "marshal")
            else:
                _lib.check(L.honu_decode_batch(c, P(sl["rec"]), P(sl["roff"]), n, P(sl["dmeta"]),
                                               P(sl["dinfo"]), P(sl["dacl"]), acl_cap, P(sl["dreg"]),
                                               reg_cap, P(sl["data"]), dcap, P(sl["tot"]), ks), "decode")
            ev2 = torch.cuda.Event()
            ev2.record(s_k)
            with torch.cuda.stream(s_out):
                s_out.wait_event(ev2)
                if encode:
                    h_rec[r0:r1].copy_(sl["rec"][: r1 - r0], non_blocking=True)
                else:
                    db = int(((lens[s:e] + 15) // 16 * 16).sum())
                    h_rows[352 * s:352 * e].copy_(sl["dmeta"][: 352 * n], non_blocking=True)
                    h_data[k % 2][:db].copy_(sl["data"][:db], non_blocking=True)
                sl["done"] = torch.cuda.Event()
                sl["done"].record(s_out)
        torch.cuda.synchronize()

    run(True)
    run(False)
    te, td = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        run(True)
        te.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        run(False)
        td.append(time.perf_counter() - t0)
    # check: decoded rows equal the input rows on the fields the host knows
    rows = h_rows.numpy()[: 352 * N].view(meta.dtype)
    ok = bool(np.array_equal(rows["pid"], meta["pid"]) and np.array_equal(rows["created"], meta["created"]))
    total = int(rec_pos[-1])
    for sl in slots:
        sl["codec"].close()
    res = {"records": N, "shape": shape, "chunk_records": C, "record_bytes": total,
           "encode_host_path_gbs": total / min(te) / 1e9,
           "decode_host_path_gbs": total / min(td) / 1e9,
           "encode_s": min(te), "decode_s": min(td), "rows_match": ok,
           "note": "pinned host buffers, 3 streams (H2D / codec / D2H), 2 device slots; "
                   "encode moves payload+rows in and records out, decode moves records in "
                   "and rows+payloads out"}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=65536)
    ap.add_argument("--chunk", type=int, default=4096)
    ap.add_argument("--shape", default="large")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    print(json.dumps(measure(a.shape, a.records, a.chunk, a.reps)))


if __name__ == "__main__":
    main()
