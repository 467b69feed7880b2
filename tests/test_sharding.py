"""Multi-GPU sharding logic (CPU): shard plans and the N>1 bench reductions over a
real world_size-2 gloo process group."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from fpnn_amd.sharding import max_over_ranks, shard_range
import workloads as W


@pytest.mark.parametrize("count,world", [(1 << 20, 8), (10, 3), (7, 8), (0, 2)])
def test_uniform_shards_cover_disjoint(count, world):
    got = [shard_range(count, world, r) for r in range(world)]
    assert got[0][0] == 0 and got[-1][1] == count
    for (a, b), (c, d) in zip(got, got[1:]):
        assert b == c and a <= b
    sizes = [b - a for a, b in got]
    assert max(sizes) - min(sizes) <= 1


def test_ragged_shards_are_byte_balanced():
    sizes = W.zipf_sizes(dict(W.C4, total_bytes=64 << 20))
    n = len(sizes)
    for world in (2, 4, 8):
        parts = [shard_range(n, world, r, sizes) for r in range(world)]
        assert parts[0][0] == 0 and parts[-1][1] == n
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        bytes_per = [int(sizes[a:b].sum()) for a, b in parts]
        assert sum(bytes_per) == int(sizes.sum())
        # every rank within one maximal packet of the ideal share
        ideal = sizes.sum() / world
        assert max(abs(x - ideal) for x in bytes_per) <= int(sizes.max())


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        count = 1 << 20
        b, e = shard_range(count, world, rank)
        # each rank's shard is the slice of one global synthetic batch (bench.py fills
        # its payload from byte offset rank * P * L)
        t = torch.tensor([b, e], dtype=torch.int64)
        allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, t)
        ranges = sorted(tuple(x.tolist()) for x in allr)
        covered = ranges[0][0] == 0 and ranges[-1][1] == count and all(
            ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
        m = max_over_ranks(1.5 + rank, world)
        dist.barrier()
        q.put((rank, covered, m))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shards_and_max_reduction():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, covered, m in res:
        assert covered
        assert m == 2.5  # max over ranks of 1.5 + rank
