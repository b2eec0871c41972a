"""Sharding of a record batch across ranks (one process per GPU).

Records are independent (object.go:24-45 encodes one record; decode is a pure
function of one Object), so the only cross-rank information is bookkeeping:
  - weak scaling: rank r owns records [r*N, (r+1)*N) of the synthetic batch;
  - a fixed batch split for strong scaling: contiguous ranges balanced by
    BYTES (exclusive scan of record sizes cut at byte quantiles), because a
    count split is unbalanced by heavy-tailed mixes (XLarge);
  - one all-gather of per-rank byte totals turns each rank's local output
    offsets into offsets of a single logical output arena.
No payload crosses ranks. Works with any torch.distributed
backend (gloo on CPU in the tests, nccl = RCCL on the GPUs).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def weak_range(rank: int, world: int, per_rank: int) -> Tuple[int, int]:
    """(first, n) of rank's shard when every rank processes per_rank records."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return rank * per_rank, per_rank


def byte_balanced_ranges(sizes: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Split records into `world` contiguous ranges of ~equal total bytes."""
    sizes = np.asarray(sizes, dtype=np.int64)
    n = len(sizes)
    cum = np.concatenate([[0], np.cumsum(sizes)])
    total = int(cum[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        cuts.append(int(np.searchsorted(cum, target, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts), n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def global_base(local_total: int, group=None) -> Tuple[int, int]:
    """All-gather the per-rank byte totals; returns (this rank's base offset in
    the logical output arena, total bytes of all ranks)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.tensor([local_total], dtype=torch.int64, device=dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    totals = [int(x.item()) for x in out]
    return sum(totals[:rank]), sum(totals)


def scatter_records(arena, off, src: int = 0, group=None):
    """Scatter a CSR records batch held by rank `src` as byte-balanced
    contiguous sub-batches: rank r receives records ranges[r] as its own
    (arena, off) with offsets rebased to 0. Point-to-point sends batched into
    one group (batch_isend_irecv: ncclGroupStart/End over RCCL, so every
    destination link is busy at once on xGMI; gloo on CPU). Non-source ranks
    pass arena=off=None. Tensors live on the backend's device (cuda for nccl).

    Returns (arena, off, first, n, bytes_sent_by_src)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    off_t = None
    if rank == src:  # offsets as int64 on the backend's device (a uint8 byte view is accepted)
        off_t = off if isinstance(off, torch.Tensor) else torch.from_numpy(np.asarray(off).astype(np.int64))
        off_t = off_t.to(dev)
        if off_t.dtype != torch.int64:
            off_t = off_t.view(torch.int64)
    # 1. geometry: [first, n, bytes] per rank, broadcast from src
    geo = torch.zeros(3 * world, dtype=torch.int64, device=dev)
    if rank == src:
        o = off_t.cpu().numpy()
        g = []
        for a, b in byte_balanced_ranges(np.diff(o), world):
            g += [a, b - a, int(o[b] - o[a])]
        geo.copy_(torch.tensor(g, dtype=torch.int64))
    dist.broadcast(geo, src, group=group)
    g = geo.cpu().tolist()
    first, n, nbytes = g[3 * rank: 3 * rank + 3]
    # 2. payloads: offsets (rebased) and record bytes, all destinations at once
    if rank == src:
        ops, keep = [], []
        for r in range(world):
            a, cnt, nb = g[3 * r: 3 * r + 3]
            lo = int(off_t[a].item())
            if r == src:
                my_off = (off_t[a: a + cnt + 1] - lo).contiguous()
                my_arena = arena[lo: lo + nb].clone() if nb else torch.zeros(16, dtype=torch.uint8, device=dev)
                continue
            o_r = (off_t[a: a + cnt + 1] - lo).contiguous()
            keep.append(o_r)
            ops.append(dist.P2POp(dist.isend, o_r, r, group=group))
            if nb:
                ops.append(dist.P2POp(dist.isend, arena[lo: lo + nb], r, group=group))
        sent = sum(g[3 * r + 2] for r in range(world) if r != src)
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return my_arena, my_off, first, n, sent
    my_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    my_arena = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=dev)
    ops = [dist.P2POp(dist.irecv, my_off, src, group=group)]
    if nbytes:
        ops.append(dist.P2POp(dist.irecv, my_arena[:nbytes], src, group=group))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return my_arena, my_off, first, n, 0
