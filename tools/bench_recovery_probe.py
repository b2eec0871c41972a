#!/usr/bin/env python3
"""Do the bench pipeline's single-launch decodes recover (misspeculate)?
Groups of PROBE_GROUP steps run back to back, then each output slot's context
is asked whether a recovery launch ran (speculate_backoff), PROBE_STEPS times.

  python tools/bench_recovery_probe.py META_STREAMS SHAPE [bench args...]
(DESIGN §3 "A guarded launch that waits for CUs"; results in
profiles/r04/final3/probes/)"""
import ctypes as C, json, sys, os
sys.path.insert(0, os.getcwd())
import torch
import bench
from honu_amd import _lib
ms = sys.argv[1]
args = bench.parse_args(["--shape", sys.argv[2], "--meta-streams", ms] + sys.argv[3:])
b = bench.Bench(args, 0, 0)
L = b.lib
def get(ctx):
    v = C.c_int64(-1)
    _lib.check(L.honu_ctx_get_param(ctx, b"speculate_backoff", C.byref(v)), "get")
    return v.value
res = []
G = int(os.environ.get("PROBE_GROUP", "4"))  # steps back to back, then one check
for step in range(int(os.environ.get("PROBE_STEPS", "8"))):
    for _ in range(G):
        b.step()
    torch.cuda.synchronize()
    r = [get(sl.codec.ctx) for sl in b.slots]
    for sl in b.slots:
        _lib.check(L.honu_ctx_set_param(sl.codec.ctx, b"speculate_backoff", 0), "set")
    res.append(r)
ok = b.verify()
print(json.dumps({"meta_streams": ms, "shape": sys.argv[2], "recoveries_per_step": res, "verified": ok}), flush=True)
