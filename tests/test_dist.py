"""The N>1 path on CPU: world-size-2 gloo process group. Sharded encode (each
rank its own byte-balanced range, offsets made global by the shard-totals
all-gather) must reproduce the single-process encoding of the whole batch
byte for byte (CPU oracle as the codec here; the GPU path is the same
per-rank code)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from honu_amd.metadata import HostBatch
    from honu_amd.shard import byte_balanced_ranges, global_base, weak_range
    from honu_amd.workload import gen_host_batch
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 300
        full = gen_host_batch(5, "mixed", 0, n)
        sizes = np.diff(full.payload_off.astype(np.int64)) + 1000
        lo, hi = byte_balanced_ranges(sizes, world)[rank]
        mine = gen_host_batch(5, "mixed", lo, hi - lo)  # records are f(seed, index)
        out, off, st = oracle.marshal_batch(mine)
        base, total = global_base(int(off[-1]))
        # weak scaling ranges are disjoint and contiguous
        first, cnt = weak_range(rank, world, 128)
        q.put((rank, lo, hi, base, total, out.tobytes(), (st == 0).all(), first, cnt))
    finally:
        dist.destroy_process_group()


def test_sharded_encode_matches_single_process(oracle_lib):
    from honu_amd.workload import gen_host_batch
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    full = gen_host_batch(5, "mixed", 0, 300)
    ref, ref_off, _ = oracle_lib.marshal_batch(full)
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == 300
    assert res[0][3] == 0 and res[1][3] == len(res[0][5])      # global bases
    assert res[0][4] == res[1][4] == len(ref)                  # total bytes
    assert res[0][5] + res[1][5] == ref.tobytes()              # sharded == single process
    assert all(r[6] for r in res)
    assert (res[0][7], res[1][7]) == (0, 128) and res[0][8] == 128


def test_byte_balanced_ranges_balance():
    from honu_amd.shard import byte_balanced_ranges
    rng = np.random.default_rng(0)
    sizes = np.where(rng.random(10000) < 0.01, 5_000_000, 3_000)
    r = byte_balanced_ranges(sizes, 8)
    assert r[0][0] == 0 and r[-1][1] == 10000
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
    tot = [sizes[a:b].sum() for a, b in r]
    assert max(tot) - min(tot) <= 2 * sizes.max()


def _scatter_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from honu_amd.shard import scatter_records
    from honu_amd.workload import gen_host_batch
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arena = off = None
        if rank == 0:
            rec, o, _ = oracle.marshal_batch(gen_host_batch(6, "mixed", 0, 257))
            arena = torch.from_numpy(rec.copy())
            off = torch.from_numpy(o.astype(np.int64))
        a, o, first, n, sent = scatter_records(arena, off, src=0)
        o = o.numpy().astype(np.uint64)
        meta, info, *_ = oracle.decode_batch(a.numpy()[: int(o[-1])], o)
        q.put((rank, first, n, a.numpy()[: int(o[-1])].tobytes(), bool((info["meta_status"] == 0).all()), sent))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_records(oracle_lib, world):
    """Staging-rank scatter of an encoded batch (the device-resident scaling
    experiment of SURVEY §8e): every rank gets a contiguous byte-balanced
    sub-batch that decodes cleanly, and the pieces concatenate to the batch."""
    from honu_amd.workload import gen_host_batch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(6, "mixed", 0, 257))
    assert b"".join(r[3] for r in res) == rec.tobytes()
    assert sum(r[2] for r in res) == 257 and res[0][1] == 0
    assert all(res[k][1] + res[k][2] == res[k + 1][1] for k in range(world - 1))
    assert all(r[4] for r in res)
    assert res[0][5] == len(rec) - len(res[0][3])
