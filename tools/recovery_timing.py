#!/usr/bin/env python3
"""What a misspeculated single-launch decode costs with a guarded launch of
G one-wave workgroups (context param guard_blocks; 0 = as many waves as the
speculative launch has). A Small batch (ticket tiles) is encoded on the
device, records whose ACL lists hold a nil entry (tests/corpora.random_metas,
encoded by the same codec) are spliced in, and honu_decode_records is timed
with HIP events on the context's stream: speculation on (back-off cleared
before every call), so every call misspeculates and the guarded launch redoes
the batch; the clean batch beside it for the no-op guard.

  python tools/recovery_timing.py [--records 262144] [--guards 0,256,512,1024]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from honu_amd import _lib  # noqa: E402
from honu_amd import object as hobj  # noqa: E402
from honu_amd.metadata import pack_batch  # noqa: E402
from honu_amd.workload import gen_host_batch  # noqa: E402


def param(c, name, v):
    _lib.check(c.lib.honu_ctx_set_param(c.ctx, name.encode(), v), name)


def get(c, name):
    v = C.c_int64(-1)
    _lib.check(c.lib.honu_ctx_get_param(c.ctx, name.encode(), C.byref(v)), name)
    return v.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 18)
    ap.add_argument("--guards", default="0,256,512,1024")
    ap.add_argument("--bad", type=int, default=1, help="records with a nil ACL entry")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from corpora import random_metas
    n = a.records
    c = hobj.Codec(0, n)
    enc = c.marshal(hobj.DeviceBatch.from_host(gen_host_batch(43, "small", 0, n)))
    rec, off, st = enc.host()
    assert (st == 0).all()
    metas, datas = random_metas(4 * a.bad + 40, 77)
    pick = [i for i, m in enumerate(metas) if m.ACL and any(x is None for x in m.ACL) and datas[i]][:a.bad]
    e2 = c.marshal(hobj.DeviceBatch.from_host(pack_batch([metas[i] for i in pick], [datas[i] for i in pick])))
    r2, o2, st2 = e2.host()
    assert (st2 == 0).all()
    at = {int(x): j for j, x in enumerate(np.linspace(3, n - 1, a.bad).astype(np.int64))}
    pieces, lens = [], np.empty(n, np.uint64)
    for i in range(n):
        j = at.get(i)
        r = r2[int(o2[j]):int(o2[j + 1])] if j is not None else rec[int(off[i]):int(off[i + 1])]
        pieces.append(r)
        lens[i] = len(r)
    boff = np.zeros(n + 1, np.uint64)
    boff[1:] = np.cumsum(lens)
    batches = {"clean": (rec, off), "misspec": (np.concatenate(pieces), boff)}
    cap = int(max(off[-1], boff[-1]))
    e = c._empty
    meta, info, acl, reg, tot = e(352 * n), e(32 * n), e(20 * cap), e(4 * cap), e(32)
    dev = {k: (hobj._dev_bytes(r, c.torch_device), hobj._dev_bytes(o, c.torch_device))
           for k, (r, o) in batches.items()}
    s = torch.cuda.current_stream()
    out = {"records": n, "bad": a.bad, "ms": {}}
    for g in [int(x) for x in a.guards.split(",")]:
        param(c, "guard_blocks", g)
        for k, (dr, do) in dev.items():
            ts = []
            for rep in range(a.reps + 1):
                param(c, "speculate_backoff", 0)
                r0 = get(c, "recoveries")
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record(s)
                _lib.check(c.lib.honu_decode_records(
                    c.ctx, _lib.ptr(dr), _lib.ptr(do), n, _lib.ptr(meta), _lib.ptr(info), _lib.ptr(acl), cap,
                    _lib.ptr(reg), cap, 0, 0, _lib.ptr(tot), c.stream), "decode")
                t1.record(s)
                torch.cuda.synchronize()
                rec_ran = get(c, "recoveries") - r0
                assert rec_ran == (1 if k == "misspec" else 0), (k, rec_ran)
                if rep:
                    ts.append(t0.elapsed_time(t1))
            out["ms"][f"g{g}_{k}"] = round(float(np.median(ts)), 4)
    print(json.dumps(out))
    c.close()


if __name__ == "__main__":
    main()
