"""The N>1 path on CPU: world_size-2 gloo processes, each with its
round-robin shard (bench.py's partition), no data-path collective.  The
union of the shards' encodings, put back in global block order, must equal
the reference encoding of the unsharded stream (digest C1), and the timing
reduction must return the max over ranks."""
from __future__ import annotations

import hashlib
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from lcdb_amd import shard

WORLD = 2
PER_RANK = 512          # 2 x 512 = the 1024 blocks of digest C1


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        c = shard.fillseq_shard(PER_RANK, rank, WORLD)
        codec = oracle.best()
        encs = [codec.encode(b) for b in c.blocks()]   # no communication here
        gathered = [None] * WORLD
        dist.all_gather_object(gathered, encs)        # test-side check only
        tmax = shard.max_over_ranks(float(rank + 1), dist)
        if rank == 0:
            order = []
            for g in range(PER_RANK * WORLD):
                r = shard.owner(g, WORLD)
                order.append(gathered[r][g // WORLD])
            h = hashlib.sha256(b"".join(order)).hexdigest()
            q.put((h, sum(len(e) for e in order), tmax))
    finally:
        dist.destroy_process_group()


def test_round_robin_shards_reassemble_to_reference(digests):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    h, nbytes, tmax = q.get(timeout=10)
    d = digests["C1_fillseq_1024x4KiB"]
    assert (h, nbytes) == (d["comp_sha256"], d["comp_bytes"])
    assert tmax == float(WORLD)


def test_shard_index_maps():
    for world in (1, 2, 3, 8):
        seen = set()
        for r in range(world):
            for i in range(shard.local_count(100, r, world)):
                g = shard.global_index(i, r, world)
                assert shard.owner(g, world) == r
                seen.add(g)
        assert seen == set(range(100))


@pytest.mark.parametrize("world", [2, 4])
def test_shards_are_slices_of_one_stream(world):
    from lcdb_amd import corpus
    full = corpus.fillseq(8 * world)
    for r in range(world):
        s = shard.fillseq_shard(8, r, world)
        for i in range(8):
            assert s.block(i) == full.block(shard.global_index(i, r, world))
