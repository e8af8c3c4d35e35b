"""CPU tests of the N>1 path: fid-range sharding balanced by bytes, and the
bench's rank protocol (barrier + MAX-over-ranks timing, per-rank fid offsets)
with a world_size-2 gloo group."""
import os
import random
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from couloydb_amd.shard import partition_by_bytes, shard_for_rank


def test_partition_properties():
    rng = random.Random(1)
    for trial in range(200):
        n = rng.randrange(0, 40)
        sizes = [rng.choice([0, 1, 1 << 20, 256 << 20, rng.randrange(1, 300 << 20)]) for _ in range(n)]
        k = rng.randrange(1, 9)
        parts = partition_by_bytes(sizes, k)
        assert len(parts) == k
        # contiguous cover of [0, n)
        assert parts[0][0] == 0 and parts[-1][1] == n
        for (a, b), (c, d) in zip(parts, parts[1:]):
            assert b == c and a <= b
        if n >= k and sum(sizes) and len(set(sizes)) == 1:
            counts = [b - a for a, b in parts]
            assert max(counts) - min(counts) <= 1


def test_partition_balanced_bytes():
    sizes = [256 << 20] * 1024            # config 5: 1024 files over 8 GPUs
    parts = partition_by_bytes(sizes, 8)
    assert [b - a for a, b in parts] == [128] * 8
    files = [(fid, s) for fid, s in enumerate(sizes)]
    assert [f for f, _ in shard_for_rank(files, 3, 8)] == list(range(384, 512))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    files = [(fid, (fid % 7 + 1) << 20) for fid in range(37)]
    mine = shard_for_rank(files, rank, world)
    # bench protocol: barrier, per-rank time, MAX over ranks, total work = sum
    dist.barrier()
    t = torch.tensor([0.5 + rank, float(sum(s for _, s in mine)), float(len(mine))], dtype=torch.float64)
    tmax = t.clone()
    dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
    dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
    gathered = [None] * world
    dist.all_gather_object(gathered, [f for f, _ in mine])
    if rank == 0:
        q.put((float(tmax[0]), float(t[1]), float(t[2]), gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_protocol():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    tmax, total_bytes, nfiles, gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert tmax == 1.5
    assert nfiles == 37 and total_bytes == sum((fid % 7 + 1) << 20 for fid in range(37))
    # union of shards is every fid, in order, contiguous per rank
    assert gathered[0] + gathered[1] == list(range(37))
