#!/usr/bin/env python3
"""Copy-engine rate vs segment size: honu_encode_payloads over uniform
synthetic segments (payload arena CSR -> records arena with a fixed gap per
record, as the Metadata tail leaves), for a fixed total of bytes. Separates
per-segment overhead from streaming bandwidth. One JSON line per size."""
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

P = lambda t: t.data_ptr()  # noqa: E731


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-gib", type=float, default=2.0)
    ap.add_argument("--sizes", default="512,1024,2048,2560,4096,8192,16384,32768,65536,262144")
    ap.add_argument("--gap", type=int, default=1027, help="record bytes between payloads")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--params", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    total = int(a.total_gib * 2**30)
    nmax = total // min(int(x) for x in a.sizes.split(","))
    codec = Codec(0, nmax)
    L, c = codec.lib, codec.ctx
    for kv in filter(None, a.params.split(",")):
        k, v = kv.split("=")
        _lib.check(L.honu_ctx_set_param(c, k.encode(), int(v)), "param")
    pay = torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device=dev)
    out = torch.empty(total + nmax * (a.gap + 8) + 64, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for sz in map(int, a.sizes.split(",")):
        n = total // sz
        poff = torch.arange(n + 1, dtype=torch.int64, device=dev) * sz
        ooff = torch.arange(n + 1, dtype=torch.int64, device=dev) * (sz + a.gap)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        _lib.check(L.honu_encode_payloads(c, P(pay), P(poff), n, P(out), out.numel(), P(ooff), P(st), s), "copy")
        e0.record()
        for _ in range(a.reps):
            _lib.check(L.honu_encode_payloads(c, P(pay), P(poff), n, P(out), out.numel(), P(ooff), P(st), s), "copy")
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / a.reps
        print(json.dumps({"seg_bytes": sz, "segments": n, "us": round(t * 1e6, 1),
                          "tbs": round(2 * n * sz / t / 1e12, 3),
                          "ns_per_segment": round(t * 1e9 / n, 2)}), flush=True)


if __name__ == "__main__":
    main()
