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
