#!/usr/bin/env python3
"""Host-path rates of the two storage feeds (include/honu_codec.h, "Read feed"
and "Write feed"): records start and end in host memory, as in Honu's
local-storage path (store Put -> object.Marshal; cursor scan -> Metadata()).

Write feed: a host batch (rows + var arena + tables + payloads) is appended
with honu_put_feed_append_batch (host memcpy into pinned slots), submitted
(H2D, marshal, D2H) and waited for, two slots in flight.
Read feed: the encoded records are appended with honu_feed_append_batch and
decoded (zero copy, keys) on the GPU, two slots in flight.

Prints one JSON line: records/s and GB/s of encoded records for both feeds,
the batch geometry, and a bit-exactness check of a sample against the oracle.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (loads the HIP runtime first)

from honu_amd.feed import PutFeed, RecordFeed  # noqa: E402
from honu_amd.workload import gen_host_batch  # noqa: E402


def put_pass(feed, hb, collect):
    first, prev, out, nrec, nbytes = 0, None, [], 0, 0

    def take(t):
        nonlocal nrec, nbytes
        r = feed.wait(t)
        n = len(r.status)
        nrec += n
        nbytes += int(r.rec_off[n])
        if collect:
            out.append((r.records.copy(), r.rec_off.copy(), r.status.copy()))

    while first < len(hb):
        st, got = feed.append_batch(hb, first)
        if got == 0:
            raise RuntimeError(f"record {first} does not fit a batch (status {st})")
        first += got
        t = feed.submit()
        if prev is not None:
            take(prev)
        prev = t
    take(prev)
    return out, nrec, nbytes


def read_pass(feed, arena, off):
    first, prev, nrec, bad = 0, None, 0, 0

    def take(t):
        nonlocal nrec, bad
        r = feed.wait(t)
        nrec += len(r.info)
        bad += int((r.info["meta_status"] != 0).sum())

    n = len(off) - 1
    while first < n:
        st, got = feed.append_batch(arena, off, first)
        if got == 0:
            raise RuntimeError(f"record {first} does not fit a batch (status {st})")
        first += got
        t = feed.submit()
        if prev is not None:
            take(prev)
        prev = t
    take(prev)
    return nrec, bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="small")
    ap.add_argument("--records", type=int, default=262144)
    ap.add_argument("--batch-records", type=int, default=32768)
    ap.add_argument("--batch-mib", type=int, default=512)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=3)
    a = ap.parse_args()
    hb = gen_host_batch(a.seed, a.shape, 0, a.records)
    bb = a.batch_mib << 20
    put = PutFeed(0, a.batch_records, bb)
    batches, n, total = put_pass(put, hb, collect=True)  # warm-up + records for the read pass
    arena = np.concatenate([b[0] for b in batches])
    sizes = np.concatenate([np.diff(b[1].astype(np.int64)) for b in batches])
    off = np.zeros(len(sizes) + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    ok = all(int((b[2] != 0).sum()) == 0 for b in batches)
    # bit-exactness of a sample against the oracle
    sys.path.insert(0, ROOT)
    from honu_amd.metadata import HostBatch
    from oracle import oracle
    k = min(512, a.records)
    sub = HostBatch(hb.meta[:k], hb.var, hb.acl, hb.regions, hb.payload, hb.payload_off[:k + 1])
    orec, ooff, _ = oracle.marshal_batch(sub)
    ok &= arena[: int(off[k])].tobytes() == orec[: int(ooff[k])].tobytes()
    t_put = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        _, n, total = put_pass(put, hb, collect=False)
        t_put.append(time.perf_counter() - t0)
    put.close()
    rd = RecordFeed(0, a.batch_records, bb)
    read_pass(rd, arena, off)
    t_rd = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        nr, bad = read_pass(rd, arena, off)
        t_rd.append(time.perf_counter() - t0)
        ok &= bad == 0 and nr == n
    rd.close()
    tp, tr = min(t_put), min(t_rd)
    print(json.dumps({
        "shape": a.shape, "records": n, "encoded_bytes": total,
        "batch_records": a.batch_records, "batch_mib": a.batch_mib,
        "put_records_per_s": n / tp, "put_gbs": total / tp / 1e9,
        "read_records_per_s": n / tr, "read_gbs": total / tr / 1e9,
        "verified": bool(ok),
        "note": "host arrays -> pinned slots -> GPU -> pinned results; two slots in flight; "
                "best of reps; read feed decodes zero copy + keys",
    }), flush=True)


if __name__ == "__main__":
    main()
