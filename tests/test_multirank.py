"""The N>1 path on CPU: world_size-2 gloo processes, each with its
round-robin shard (bench.py's partition), no data-path collective.  The
union of the shards' encodings, put back in global block order, must equal
the reference encoding of the unsharded stream (digest C1), and the timing
reduction must return the max over ranks."""
from __future__ import annotations

import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from lcdb_amd import shard

WORLD = 2
BENCH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")
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


def _bench(*args: str, env=None) -> subprocess.CompletedProcess:
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True,
                          timeout=600, env=e)


def _last_json(out: str) -> dict:
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_bench_launcher_ws2_reassembles_c1(digests):
    """bench.py's own launcher (--gpus 2, no WORLD_SIZE) starts 2 gloo ranks;
    their round-robin shards, re-interleaved by the parity gather, are the
    C1 stream (per-block digests in global order == the pinned raw_dd)."""
    r = _bench("--gpus", "2", "--plan-only", "--total-blocks", "1024")
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["blocks_rank0"] == 512
    assert line["raw_dd"] == digests["C1_fillseq_1024x4KiB"]["raw_dd"]
    assert line["max_over_ranks"] == 2.0


@pytest.mark.slow
def test_bench_launcher_c4_default(digests):
    """At N > 1 the default workload is C4: 1 048 576 blocks dealt g -> g % N."""
    r = _bench("--gpus", "2", "--plan-only")
    assert r.returncode == 0, r.stderr[-2000:]
    line = _last_json(r.stdout)
    assert line["workload"].startswith("C4:")
    assert line["total_blocks"] == 1048576 and line["blocks_rank0"] == 524288
    assert line["raw_dd"] == digests["C4_fillseq_1048576x4KiB"]["raw_dd"]


def test_bench_rejects_world_mismatch():
    r = _bench("--gpus", "4", "--plan-only", "--total-blocks", "64",
               env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_oracle_shards_reassemble_to_reference_dd(digests):
    """comp_dd (digest of per-block digests) of C1 from ws=3 round-robin
    shards encoded by the reference codec equals the pinned comp_dd."""
    from lcdb_amd import corpus
    codec = oracle.best()
    per = []
    for r in range(3):
        c = shard.fillseq_total(1024, r, 3)
        out, ooff, olen = codec.encode_batch(c.buf, c.off, c.len, 2)
        per.append(corpus.block_digests(out, ooff, olen))
    allb = shard.interleave(per, 1024)
    assert corpus.digest_of_digests(allb) == digests["C1_fillseq_1024x4KiB"]["comp_dd"]


def test_bench_launcher_fails_fast_when_a_rank_dies():
    """A rank that exits non-zero ends the launch at once (the survivors are
    terminated, not left in gloo's rendezvous until its timeout)."""
    import time
    t0 = time.perf_counter()
    r = _bench("--gpus", "2", "--plan-only", "--total-blocks", "-5")
    assert r.returncode != 0
    assert time.perf_counter() - t0 < 120


def test_cpu_baseline_fields_on_cpu():
    """bench.py's cpu_baseline leg (no GPU needed): 1 thread, the per-GPU
    share and nproc threads, both partitions, the reference's bytes."""
    import argparse

    import bench
    from lcdb_amd import corpus
    c = corpus.fillseq(256)
    a = argparse.Namespace(cpu_threads=2, cpu_sample=256, cpu_reps=1)
    out, ooff, olen = oracle.best().encode_batch(c.buf, c.off, c.len, 1)

    class H:   # the GPU's compressed blocks, as bench.py holds them
        buf, off, len = out, ooff, olen
    cb = bench.cpu_baseline(c, a, H, 1)
    nproc = len(os.sched_getaffinity(0))
    assert cb["nproc"]["threads"] == nproc
    assert cb["single_thread"]["threads"] == 1 and cb["per_gpu_share"]["threads"] == 2
    assert 1 <= cb["cores"] <= nproc
    assert cb["same_bytes_as_gpu"] is True
    # the headline is the fastest of the three points (on a small sample or
    # under a CPU quota fewer threads can win), and says which one it is
    pts = [cb["single_thread"], cb["per_gpu_share"], cb["nproc"]]
    assert cb["value"] == max(x["roundtrip_GiBps"] for x in pts) > 0
    assert cb["threads"] in {x["threads"] for x in pts}
    if nproc > 1:
        assert set(cb["nproc"]["by_partition"]) == {"round-robin", "contiguous"}


@pytest.mark.gpu
def test_bench_two_ranks_on_the_gpu_c2(digests):
    """bench.py --gpus 2 on the GPU box (the ranks share its GPU): C2's 65 536
    blocks dealt g -> g % 2, every rank encodes and decodes its shard, and
    rank 0's re-interleaved per-block digests equal the pinned C2 comp_dd."""
    r = _bench("--gpus", "2", "--total-blocks", "65536", "--steps", "2", "--warmup", "1",
               "--no-c3", "--no-cpu-baseline", "--no-pipelined", "--no-copy-probe")
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["config"]["blocks_rank0"] == 32768
    assert line["parity"].startswith("compressed blocks == reference (C2_fillseq_65536x4KiB")
    assert len(line["per_rank_elapsed_s"]["ranks"]) == 2


@pytest.mark.gpu
def test_bench_c4_full_stream_on_one_gpu(digests):
    """C4 (BASELINE.json configs[3]): the whole 1 048 576-block stream encoded
    and decoded on one GPU; compressed blocks equal the pinned C4 comp_dd."""
    r = _bench("--gpus", "1", "--total-blocks", "1048576", "--steps", "1", "--warmup", "1",
               "--copies", "1", "--no-c3", "--no-cpu-baseline", "--no-pipelined",
               "--no-copy-probe")
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["config"]["workload"].startswith("C4:")
    assert line["parity"].startswith("compressed blocks == reference (C4_fillseq_1048576x4KiB")
