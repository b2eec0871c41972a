#!/usr/bin/env python3
"""Device-resident scatter of an encoded batch from a staging GPU (SURVEY
§8e): rank 0 marshals a synthetic batch on its GPU, then sends every rank a
contiguous byte-balanced sub-batch with RCCL point-to-point sends batched in
one group (honu_amd.shard.scatter_records); each rank decodes what it got
(zero copy) and checks every record. Prints one JSON line on rank 0 with the
scatter rate (bytes leaving rank 0 / time) and the per-rank decode rate.

Not part of bench.py: in Honu the records start in host memory, so each GPU's
own H2D is the production feed; this measures the xGMI path for a batch that
is already on one GPU.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port 29511 tools/scatter_bench.py --gib 8
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from honu_amd import _lib  # noqa: E402
from honu_amd.object import Codec  # noqa: E402
from honu_amd.shard import scatter_records  # noqa: E402
from honu_amd.workload import gen_meta  # noqa: E402

P = lambda t: t.data_ptr()  # noqa: E731


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0, help="encoded GiB on the staging GPU")
    ap.add_argument("--shape", default="large")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", local)
    s = torch.cuda.current_stream().cuda_stream
    arena = off = None
    if rank == 0:
        avg = {"small": 3600, "medium": 26000, "large": 198000, "xlarge": 3.2e6, "mixed": 80000}[a.shape]
        n = max(world, int(a.gib * 2**30 / avg))
        meta, var, acl, reg, poff = gen_meta(1, a.shape, 0, n)
        codec = Codec(local, n)

        def D(x):
            x = np.ascontiguousarray(x)
            t = torch.empty(max(x.nbytes, 16), dtype=torch.uint8, device=dev)
            if x.nbytes:
                t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
            return t
        dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(poff)
        pay = torch.empty(int(poff[n]) + 16, dtype=torch.uint8, device=dev)
        _lib.check(codec.lib.honu_gen_payload(codec.ctx, 1, 0, n, P(do), P(pay), s), "gen")
        cap = int(poff[n]) + 2048 * n
        arena = torch.empty(cap, dtype=torch.uint8, device=dev)
        off_b = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
        st = torch.empty(4 * n + 16, dtype=torch.uint8, device=dev)
        _lib.check(codec.lib.honu_marshal_batch(codec.ctx, P(dm), P(dv), len(var), P(da), len(acl),
                                                P(dr), len(reg), P(pay), P(do), n, P(arena), cap,
                                                P(off_b), P(st), s), "marshal")
        torch.cuda.synchronize()
        off = off_b.view(torch.int64)[: n + 1]
        del pay
    times = []
    for _ in range(a.reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mine, moff, first, cnt, sent = scatter_records(arena, off, src=0)
        torch.cuda.synchronize()
        dist.barrier()
        times.append(time.perf_counter() - t0)
    # decode what arrived (headers + Metadata walk, zero copy) and check it
    c = Codec(local, max(cnt, 1))
    rows = torch.empty(352 * max(cnt, 1), dtype=torch.uint8, device=dev)
    info = torch.empty(32 * max(cnt, 1), dtype=torch.uint8, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.check(c.lib.honu_decode_parse(c.ctx, P(mine), P(moff), cnt, P(rows), P(info), s), "parse")
    e1.record()
    torch.cuda.synchronize()
    inf = info[: 32 * cnt].view(torch.int64).view(cnt, 4)
    st32 = inf[:, 2].contiguous().view(torch.int32).view(cnt, 2)
    ok = torch.tensor([int(bool((st32 == 0).all()))], device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    ms = torch.tensor([e0.elapsed_time(e1)], dtype=torch.float64, device=dev)
    dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    if rank == 0:
        t = min(times)
        print(json.dumps({
            "metric": "device-resident scatter of encoded records from a staging GPU (RCCL p2p group)",
            "n_gpus": world, "shape": a.shape, "records": int(off.numel() - 1),
            "bytes_sent": sent, "scatter_ms": t * 1e3, "scatter_gbs": sent / t / 1e9,
            "per_link_gbs": sent / t / 1e9 / max(1, world - 1),
            "decode_parse_ms_max": float(ms.item()), "verified": bool(ok.item()),
        }), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
