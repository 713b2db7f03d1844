#!/usr/bin/env python3
"""bench.py -- device-resident Snappy encode+decode throughput on MI355X.

Metric (BASELINE.json): device-resident GiB/s of Snappy encode+decode on
4 KiB SSTable blocks.  One *step* = one encode launch + one decode launch over
the GPU's whole batch of synthetic db_bench fillseq blocks (BASELINE config 2:
65 536 x 4 KiB blocks per GPU), inputs already resident in HBM.
``value`` = uncompressed bytes that went through encode AND decode, summed
over all ranks, / wall time of the K timed steps (max over ranks), in GiB/s.

Multi-GPU (``torch.distributed.run``, one process per GPU): blocks are a
round-robin partition of one fillseq stream (block g -> rank g % N), each
rank holds 65 536 blocks (weak scaling); no data-path collective -- only the
barrier and the max-over-ranks timing reduction.

Extra JSON fields: per-kernel HIP-event timings (``kernels``), the roofline
of the dominant kernel (algorithmic bytes = raw + compressed + 16 per block,
SURVEY §8d), the CPU baseline (reference snappy.c from oracle/_ref on a
bounded sample, rank 0 at N=1 only), and a parity check of this run's output
against the reference digest.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse() -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--blocks", type=int, default=65536, help="blocks per GPU")
    p.add_argument("--block-size", type=int, default=4096)
    p.add_argument("--copies", type=int, default=2,
                   help="independent corpus copies rotated per step (defeats the 256 MiB MALL)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, cpu_count)")
    p.add_argument("--cpu-sample", type=int, default=16384, help="blocks in the CPU sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--no-pipelined", action="store_true",
                   help="skip the extra concurrent encode||decode measurement")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                   help="PMC traffic summary (written by tools/profile_traffic.py)")
    return p.parse_args()


def main() -> None:
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from lcdb_amd import batch, shard, snappy  # noqa: F401  (loads the HIP library)

    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))

    # ---- workload: this rank's round-robin shard of one fillseq stream ----
    t_gen = time.perf_counter()
    c = shard.fillseq_shard(a.blocks, rank, world, a.block_size)
    t_gen = time.perf_counter() - t_gen
    n = c.n
    raw_bytes = c.raw_bytes

    raws = [batch.upload(c, dev) for _ in range(a.copies)]
    comps = [batch.encode_slots(r) for r in raws]
    outs = [batch.decode_slots(c.len, dev) for _ in range(a.copies)]
    stats = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(a.copies)]

    def step(k: int, ev=None) -> None:
        j = k % a.copies
        if ev is not None:
            ev[0].record()
        batch.encode(raws[j], comps[j])
        if ev is not None:
            ev[1].record()
        batch.decode(comps[j], outs[j], stats[j])
        if ev is not None:
            ev[2].record()

    for k in range(a.warmup):
        step(k)
    torch.cuda.synchronize()

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(a.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k, evs[k])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = shard.max_over_ranks(t1 - t0, dist, dev)

    # ---- extra (not `value`): encode and decode concurrently on two streams,
    # step k encoding copy k while decoding what step k-1 encoded -- the shape
    # of a store that compacts (writes) while serving reads.
    pipelined = None
    if not a.no_pipelined and a.copies >= 2:
        s_enc, s_dec = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
        enc_done = [torch.cuda.Event() for _ in range(a.copies)]
        dec_done = [torch.cuda.Event() for _ in range(a.copies)]
        batch.encode(raws[0], comps[0], s_enc)
        enc_done[0].record(s_enc)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        t0p = time.perf_counter()
        for k in range(1, a.steps + 1):
            j, jp = k % a.copies, (k - 1) % a.copies
            if k >= a.copies:
                s_enc.wait_event(dec_done[j])        # the decode reading slot j is done
            batch.encode(raws[j], comps[j], s_enc)
            enc_done[j].record(s_enc)
            s_dec.wait_event(enc_done[jp])           # decode what step k-1 encoded
            batch.decode(comps[jp], outs[jp], stats[jp], s_dec)
            dec_done[jp].record(s_dec)
        torch.cuda.synchronize()
        tp = shard.max_over_ranks(time.perf_counter() - t0p, dist, dev)
        pipelined = {"GiBps": raw_bytes * world * a.steps / tp / 2**30,
                     "ms_per_step": tp / a.steps * 1e3,
                     "note": "encode(step k) || decode(step k-1) on two streams; extra field, "
                             "not value"}

    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    comp_bytes = int(comps[0].len.sum(dtype=torch.int64).item())

    # ---- parity of this run's output ----
    parity = None
    if not a.no_parity:
        ok = all(bool((s == 1).all()) for s in stats)
        dec_sha, _ = batch.digest(outs[0])
        ok = ok and dec_sha == c.sha256()
        comp_sha, _ = batch.digest(comps[0])
        ok = ok and all(batch.digest(x)[0] == comp_sha for x in comps[1:])
        dg = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
        ref = dg.get("C2_fillseq_65536x4KiB", {})
        if world == 1 and a.blocks == 65536 and a.block_size == 4096 and ref:
            same = comp_sha == ref["comp_sha256"]
            parity = ("compressed corpus sha256 == reference digest, round trip exact"
                      if (ok and same) else "MISMATCH")
        else:
            parity = "round trip exact, status all ok" if ok else "MISMATCH"

    tot_units = raw_bytes * world * a.steps
    value = tot_units / elapsed / 2**30
    enc_alg = raw_bytes + comp_bytes + 16 * n   # SURVEY §8d per-block bytes x blocks
    kern = {
        "encode": {"avg_ms": enc_ms, "alg_bytes": enc_alg,
                   "achieved_GBps": enc_alg / (enc_ms * 1e-3) / 1e9,
                   "GiBps_uncompressed": raw_bytes / (enc_ms * 1e-3) / 2**30},
        "decode": {"avg_ms": dec_ms, "alg_bytes": enc_alg,
                   "achieved_GBps": enc_alg / (dec_ms * 1e-3) / 1e9,
                   "GiBps_uncompressed": raw_bytes / (dec_ms * 1e-3) / 2**30},
    }
    dom = "encode" if enc_ms >= dec_ms else "decode"
    traffic = None
    try:
        tr = json.load(open(a.traffic))
        if tr.get("blocks") == n and dom in tr.get("kernels", {}):
            traffic = tr["kernels"][dom].get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    roof = {"bound": "hbm", "kernel": dom, "achieved": kern[dom]["achieved_GBps"],
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": kern[dom]["achieved_GBps"] / HBM_PEAK_GBS, "traffic": traffic}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(c, a)

    if rank == 0:
        line = {
            "metric": baseline["metric"], "value": value, "unit": "GiB/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"C2: {a.blocks} x {a.block_size // 1024} KiB db_bench "
                                   f"fillseq blocks per GPU, encode+decode round trip",
                       "blocks_per_gpu": n, "raw_bytes_per_gpu": raw_bytes,
                       "comp_bytes_per_gpu": comp_bytes, "ratio": comp_bytes / raw_bytes,
                       "partition": "round-robin block g -> rank g % N, no collective",
                       "copies_rotated": a.copies},
            "encode_GiBps": raw_bytes * world / (enc_ms * 1e-3) / 2**30,
            "decode_GiBps": raw_bytes * world / (dec_ms * 1e-3) / 2**30,
            "kernels": kern, "roofline": roof, "cpu_baseline": cpu, "parity": parity,
            "pipelined": pipelined,
            "gen_seconds": t_gen,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline(c, a) -> dict:
    """Reference snappy.c (oracle/_ref) on a bounded sample of the same blocks."""
    import oracle
    codec = oracle.reference()
    kind = "reference"
    if codec is None:
        codec, kind = oracle.restatement(), "port"
    threads = a.cpu_threads or min(16, os.cpu_count() or 1)
    m = min(a.cpu_sample, c.n)
    buf, off, ln = c.buf, c.off[:m].copy(), c.len[:m].copy()
    raw = int(ln.sum(dtype=np.uint64))
    comp = codec.encode_batch(buf, off, ln, threads)            # warm + inputs for decode
    caps = ln.copy()
    codec.decode_batch(comp[0], comp[1], comp[2], caps, threads)
    t_enc, t_dec, reps = [], [], 0
    t_stop = time.perf_counter() + a.cpu_seconds
    while reps < 3 or time.perf_counter() < t_stop:
        t0 = time.perf_counter()
        codec.encode_batch(buf, off, ln, threads)
        t1 = time.perf_counter()
        codec.decode_batch(comp[0], comp[1], comp[2], caps, threads)
        t2 = time.perf_counter()
        t_enc.append(t1 - t0)
        t_dec.append(t2 - t1)
        reps += 1
    te, td = float(np.median(t_enc)), float(np.median(t_dec))
    return {"value": raw / (te + td) / 2**30, "unit": "GiB/s", "cores": threads, "kind": kind,
            "encode_GiBps": raw / te / 2**30, "decode_GiBps": raw / td / 2**30,
            "sample": f"first {m} of the GPU's blocks ({raw} B raw), encode+decode pass, "
                      f"median of {reps} reps, {threads} threads round-robin"}


if __name__ == "__main__":
    main()
