#!/usr/bin/env python3
"""Do two single-launch decodes on two contexts and two streams, running at
once, misspeculate? Each round launches K decodes per context back to back on
its own stream, then checks each context's speculate_backoff (a recovery ran)
and compares the outputs with a solo decode's.

  python tools/decode_overlap_probe.py SHAPE RECORDS [two|one]
(DESIGN §3 "A guarded launch that waits for CUs"; results in
profiles/r04/final3/probes/)"""
import ctypes as C, json, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from honu_amd import _lib
from honu_amd.object import Codec
from honu_amd.workload import gen_meta

P = lambda t: t.data_ptr()  # noqa: E731
shape, n = sys.argv[1], int(sys.argv[2])
mode = sys.argv[3] if len(sys.argv) > 3 else "two"  # two | one (same context twice, serial)
dev = torch.device("cuda", 0)
s0 = torch.cuda.current_stream().cuda_stream
ca, cb = Codec(0, n), Codec(0, n)
L = ca.lib
meta, var, acl, reg, off = gen_meta(1, shape, 0, n)


def D(x):
    x = np.ascontiguousarray(x)
    t = torch.empty(max(x.nbytes, 16), dtype=torch.uint8, device=dev)
    t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
    return t


dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(off)
pay = torch.empty(int(off[n]) + 16, dtype=torch.uint8, device=dev)
c = ca.ctx
_lib.check(L.honu_gen_payload(c, 1, 0, n, P(do), P(pay), s0), "gen")
oo = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
st = torch.empty(4 * n + 16, dtype=torch.uint8, device=dev)
_lib.check(L.honu_encode_sizes(c, P(dm), len(var), P(da), len(acl), P(dr), len(reg), P(do), n, P(oo), P(st), s0), "sz")
_lib.check(L.honu_exclusive_scan(c, P(oo), n, P(oo), s0), "scan")
total = int(oo.view(torch.int64)[n].item())
rec = torch.empty(total + 16, dtype=torch.uint8, device=dev)
_lib.check(L.honu_encode(c, P(dm), P(dv), len(var), P(da), len(acl), P(dr), len(reg), P(pay), P(do), n, P(rec),
                         total, P(oo), P(st), s0), "enc")
del pay
acl_cap = int(meta["acl_count"].astype(np.int64).sum()) + 1
reg_cap = int(meta["regions_count"].astype(np.int64).sum()) + 1
E = lambda nb: torch.empty(int(nb), dtype=torch.uint8, device=dev)  # noqa: E731


class Out:
    def __init__(self):
        self.m, self.i, self.a, self.r, self.t = E(352 * n), E(32 * n), E(20 * acl_cap), E(4 * reg_cap), E(32)

    def dec(self, ctx, s):
        _lib.check(L.honu_decode_records(ctx, P(rec), P(oo), n, P(self.m), P(self.i), P(self.a), acl_cap,
                                         P(self.r), reg_cap, 0, 0, P(self.t), s), "dec")

    def same(self, o):
        t = o.t[:24].view(torch.int64).tolist()
        return all(torch.equal(x, y) for x, y in ((self.m, o.m), (self.i, o.i), (self.a[:20 * t[0]], o.a[:20 * t[0]]),
                                                   (self.r[:4 * t[1]], o.r[:4 * t[1]]), (self.t[:24], o.t[:24])))


def backoff(ctx):
    v = C.c_int64(-1)
    _lib.check(L.honu_ctx_get_param(ctx, b"speculate_backoff", C.byref(v)), "get")
    _lib.check(L.honu_ctx_set_param(ctx, b"speculate_backoff", 0), "set")
    return v.value


ref = Out()
ref.dec(ca.ctx, s0)
torch.cuda.synchronize()
assert backoff(ca.ctx) == 0
oa, ob = Out(), Out()
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
res = []
for r in range(int(os.environ.get("ROUNDS", "10"))):
    for k in range(int(os.environ.get("K", "3"))):
        if mode == "two":
            oa.dec(ca.ctx, sa.cuda_stream)
            ob.dec(cb.ctx, sb.cuda_stream)
        else:
            oa.dec(ca.ctx, s0)
            ob.dec(ca.ctx, s0)
    torch.cuda.synchronize()
    res.append([backoff(ca.ctx), backoff(cb.ctx), oa.same(ref), ob.same(ref)])
print(json.dumps({"shape": shape, "n": n, "mode": mode, "rounds": res}), flush=True)
