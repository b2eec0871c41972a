"""The bench's N>1 legs on CPU at world size 2 (gloo): the scatter leg
(rank 0's encoded records sent as byte-balanced sub-batches, every rank checks
what arrived) and the host-path leg's aggregation over ranks, through the same
bench.py functions the GPU run calls (bench.scatter_leg, bench.host_path_leg,
bench.make_reducers). The CPU oracle encodes and checks here; on the GPU the
codec does."""
import os
import socket
import sys

import numpy as np
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
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from honu_amd.workload import gen_host_batch
        from oracle import oracle

        gather_max, all_ok = bench.make_reducers(dist, world, torch.device("cpu"))
        arena = off = None
        if rank == 0:
            hb = gen_host_batch(3, "mixed", 0, 120)
            out, ooff, st = oracle.marshal_batch(hb)
            assert (st == 0).all()
            arena = torch.from_numpy(out.copy())
            off = torch.from_numpy(ooff.astype(np.int64))

        def check(mine, moff, cnt):
            rec = mine.numpy()[: int(moff[-1])] if cnt else np.zeros(1, np.uint8)
            _, info, _, _, _, _ = oracle.decode_batch(rec, moff.numpy().astype(np.uint64))
            return cnt > 0 and bool((info["meta_status"] == 0).all()) and bool(
                (info["data_status"] == 0).all())

        sc = bench.scatter_leg(arena, off, dist, world, all_ok, check)

        class B:  # the Bench attributes host_path_leg reads
            total_rec_bytes = 10 * 4096
            N = 10
            first = 10 * rank

        class A:
            shape = "mixed"

        def fake_measure(shape, n, chunk, reps, device, first):
            assert (shape, first) == ("mixed", 10 * rank) and 256 <= n and chunk >= 256
            return {"record_bytes": 1000, "encode_s": 0.1 * (rank + 1), "decode_s": 0.25,
                    "rows_match": rank == 0}

        hp = bench.host_path_leg(B, A, 0, world, gather_max, all_ok, measure=fake_measure)
        mx, vals = gather_max(float(rank + 3))
        q.put((rank, sc, hp, mx, vals))
    finally:
        dist.destroy_process_group()


def test_scatter_and_host_path_legs_world2(oracle_lib):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sc, hp, mx, vals in res:
        assert sc["verified"] is True
        assert sc["bytes_sent_by_rank0"] > 0 and sc["scatter_gbs"] > 0
        assert mx == 4.0 and vals == [3.0, 4.0]
        agg = hp["all_ranks"]
        # all ranks' bytes over the slowest rank's time
        assert abs(agg["encode_host_path_gbs"] - 2 * 1000 / 0.2 / 1e9) < 1e-15
        assert abs(agg["decode_host_path_gbs"] - 2 * 1000 / 0.25 / 1e9) < 1e-15
        assert hp["rows_match"] is False  # AND over ranks
