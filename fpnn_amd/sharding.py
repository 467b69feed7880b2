"""Multi-GPU sharding of a packet batch.

Packets and streams are independent CFB chains, so a batch splits across GPUs by
packet (or stream) index with no data-path collective: every rank encrypts /
decrypts its own contiguous range.  Ranges are balanced by payload bytes (prefix sum
over lengths), never splitting a packet or a stream.  torch.distributed is used only
for the barrier and the max-over-ranks timing reduction.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np


def shard_range(count: int, world: int, rank: int, lengths: Optional[Sequence[int]] = None) -> Tuple[int, int]:
    """Contiguous [begin, end) packet range of `rank`.

    Uniform packets: equal counts (the first count % world ranks get one more).
    Ragged packets: cut at the packet whose byte prefix sum crosses rank/world of the
    total, so every rank gets ~total/world bytes (byte-balanced)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    if lengths is None:
        base, extra = divmod(count, world)
        begin = rank * base + min(rank, extra)
        return begin, begin + base + (1 if rank < extra else 0)
    lens = np.asarray(lengths, dtype=np.uint64)
    if len(lens) != count:
        raise ValueError("lengths must have one entry per packet")
    csum = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)])
    total = int(csum[-1])

    def cut(r):
        if r == 0:
            return 0
        if r == world:
            return count
        target = (total * r + world - 1) // world
        return int(np.searchsorted(csum, np.uint64(target), side="left"))

    return cut(rank), cut(rank + 1)


def max_over_ranks(value: float, world: int, device=None) -> float:
    """Max of a per-rank scalar (the bench contract's timing reduction)."""
    if world <= 1:
        return float(value)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
