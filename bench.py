#!/usr/bin/env python3
"""bench.py -- device-resident Snappy encode+decode throughput on MI355X.

Metric (BASELINE.json): device-resident GiB/s of Snappy encode+decode on
4 KiB SSTable blocks at 1/2/4/8 MI355X.  One *step* = one encode launch + one
decode launch over a GPU's whole share of synthetic db_bench fillseq blocks,
inputs already resident in HBM.  ``value`` = uncompressed bytes that went
through encode AND decode, summed over all ranks, / wall time of the K timed
steps (max over ranks), in GiB/s.

Workloads (BASELINE.json ``configs``):
  * N = 1 (default): C2, 65 536 x 4 KiB blocks on one GPU.
  * N > 1 (default): C4, 1 048 576 x 4 KiB blocks dealt round-robin
    (block g -> rank g % N), strong scaling: each rank holds 1 048 576 / N.
  * ``--total-blocks T`` picks any stream length (``--total-blocks 1048576``
    at N = 1 is C4's one-GPU point).

Multi-GPU: one process per GPU.  Under ``torch.distributed.run`` the ranks
come from RANK / LOCAL_RANK / WORLD_SIZE, which must agree with ``--gpus``.
Without them, ``--gpus N`` (N > 1) starts the N rank processes itself
before anything touches a GPU (127.0.0.1 rendezvous) and exits with their
status.  The process group is gloo: ranks only meet at the timing barriers,
the max-over-ranks reduction and, after timing, the parity gather of
per-block digests -- no data-path collective, no RCCL.

Extra JSON fields: per-kernel HIP-event timings (``kernels``), the roofline
of the dominant kernel (algorithmic bytes = raw + compressed + 16 per block,
SURVEY §8d), the CPU baseline (the reference snappy.c from oracle/_ref, rank 0
at N = 1 only, BASELINE.md's plan: 1 thread and the host's thread share, same
blocks, median of 5) and the parity of this run's output against the
reference digests.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
C2_BLOCKS, C4_BLOCKS = 65536, 1048576


def parse(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--total-blocks", type=int, default=0,
                   help="blocks in the whole stream, dealt round-robin over the ranks "
                        "(0: C2 = 65 536 at N = 1, C4 = 1 048 576 at N > 1)")
    p.add_argument("--blocks", type=int, default=0,
                   help="blocks per GPU (weak scaling); overrides --total-blocks")
    p.add_argument("--block-size", type=int, default=4096)
    p.add_argument("--copies", type=int, default=2,
                   help="independent corpus copies rotated per step (defeats the 256 MiB MALL)")
    p.add_argument("--cpu-reps", type=int, default=5)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="the multi-thread CPU point (0: this host's CPU share, <= 16)")
    p.add_argument("--cpu-sample", type=int, default=C2_BLOCKS,
                   help="blocks in the CPU sample (the first of the GPU's blocks)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--no-copy-probe", action="store_true",
                   help="skip the 1 GiB copy that measures the achievable HBM rate")
    p.add_argument("--no-pipelined", action="store_true",
                   help="skip the extra concurrent encode||decode measurement")
    p.add_argument("--no-table", action="store_true",
                   help="skip the batched table write/read extra field")
    p.add_argument("--no-c3", action="store_true",
                   help="skip the extra C3 (mixed 4/16/64 KiB) measurement at N = 1")
    p.add_argument("--c3-scale", type=int, default=32,
                   help="C3 scale: 512/128/32 blocks per half-class x this")
    p.add_argument("--plan-only", action="store_true",
                   help="no GPU: launch, partition and digest-gather only (CPU tests)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                   help="PMC traffic summary (tools/traffic_json.py)")
    return p.parse_args(argv)


def total_blocks(a, world: int) -> int:
    if a.blocks:
        return a.blocks * world
    if a.total_blocks:
        return a.total_blocks
    return C2_BLOCKS if world == 1 else C4_BLOCKS


def workload_name(total: int, a, world: int) -> str:
    kib = a.block_size // 1024
    if a.block_size == 4096 and not a.blocks:
        if total == C2_BLOCKS and world == 1:
            return f"C2: {total} x 4 KiB db_bench fillseq blocks on 1 GPU, encode+decode"
        if total == C4_BLOCKS:
            return (f"C4: {total} x 4 KiB db_bench fillseq blocks round-robin over {world} "
                    f"GPU{'s' if world > 1 else ''}, encode+decode")
    return (f"{total} x {kib} KiB db_bench fillseq blocks round-robin over {world} GPU(s), "
            f"encode+decode")


def reference_digest(total: int, a) -> dict | None:
    """The pinned reference digests of this exact stream, if any."""
    if a.block_size != 4096:
        return None
    dg = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    for key in ("C1_fillseq_1024x4KiB", "C2_fillseq_65536x4KiB", "C4_fillseq_1048576x4KiB"):
        d = dg.get(key)
        if d and d.get("blocks") == total and "comp_dd" in d:
            return dict(d, name=key)
    return None


# ---------------------------------------------------------------- launcher

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """Start n rank processes of this script (this process never touches a
    GPU) and return the first non-zero exit status, else 0.  The children
    are polled: once one fails the others are terminated at once (they
    would otherwise sit in gloo's rendezvous or a barrier until its
    timeout)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                      env=env))
    first_bad = 0
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad and not first_bad:
            first_bad = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
        if all(rc is not None for rc in rcs):
            return first_bad
        time.sleep(0.05)


# ---------------------------------------------------------------- ranks

def gather_digests(dist, rank: int, world: int, per_block: np.ndarray, total: int):
    """Rank 0 receives every rank's per-block digests and puts them back in
    global stream order (gloo, after the timed region)."""
    from lcdb_amd import shard
    if dist is None:
        return per_block
    got = [None] * world
    dist.all_gather_object(got, per_block)
    return shard.interleave(got, total) if rank == 0 else None


def run_plan_only(a, rank: int, world: int, dist) -> None:
    """Launcher + partition + digest path without a GPU: each rank builds its
    shard; rank 0 reassembles the raw stream's digest-of-digests."""
    from lcdb_amd import corpus, shard
    total = total_blocks(a, world)
    c = shard.fillseq_total(total, rank, world, a.block_size)
    per = corpus.block_digests(c.buf, c.off, c.len)
    allb = gather_digests(dist, rank, world, per, total)
    tmax = shard.max_over_ranks(float(rank + 1), dist)
    if rank == 0:
        print(json.dumps({"plan_only": True, "n_gpus": world, "total_blocks": total,
                          "blocks_rank0": c.n, "raw_dd": corpus.digest_of_digests(allb),
                          "max_over_ranks": tmax,
                          "workload": workload_name(total, a, world)}), flush=True)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return spawn_ranks(a.gpus, argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")

    dist = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        # A short timeout: a rank that died must not leave the others waiting
        # for gloo's default 30 minutes.
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=300))
    try:
        if a.plan_only:
            run_plan_only(a, rank, world, dist)
        else:
            run(a, rank, world, local, dist)
    finally:
        if dist is not None:
            dist.destroy_process_group()
    return 0


def run(a, rank: int, world: int, local: int, dist) -> None:
    import torch
    # One GPU per rank; with fewer visible GPUs than local ranks (a rehearsal
    # of the N > 1 path on a smaller box) ranks share devices round-robin and
    # the line says so -- such a value is not an N-GPU measurement.
    ndev = torch.cuda.device_count()
    dev_index = local % ndev if ndev else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    shared = ndev > 0 and world > ndev

    from lcdb_amd import batch, corpus, shard, snappy  # noqa: F401  (loads the HIP library)
    from lcdb_amd.build import kernel_sources_sha

    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    total = total_blocks(a, world)

    # ---- workload: this rank's round-robin share of one fillseq stream ----
    t_gen = time.perf_counter()
    c = shard.fillseq_total(total, rank, world, a.block_size)
    t_gen = time.perf_counter() - t_gen
    n = c.n
    raw_bytes = c.raw_bytes

    raws = [batch.upload(c, dev) for _ in range(a.copies)]
    comps = [batch.encode_slots(r) for r in raws]
    outs = [batch.decode_slots(c.len, dev) for _ in range(a.copies)]
    stats = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(a.copies)]
    stream = torch.cuda.current_stream(dev)    # the stream the codec launches on

    def step(k: int, ev=None) -> None:
        j = k % a.copies
        if ev is not None:
            ev[0].record(stream)
        batch.encode(raws[j], comps[j], stream)
        if ev is not None:
            ev[1].record(stream)
        batch.decode(comps[j], outs[j], stats[j], stream)
        if ev is not None:
            ev[2].record(stream)

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
    elapsed = shard.max_over_ranks(t1 - t0, dist)
    # every rank's own elapsed time (imbalance between GPUs is visible here)
    per_rank = [t1 - t0]
    if dist:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, t1 - t0)

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
        tp = shard.max_over_ranks(time.perf_counter() - t0p, dist)
        pipelined = {"GiBps": raw_bytes * world * a.steps / tp / 2**30,
                     "ms_per_step": tp / a.steps * 1e3,
                     "note": "encode(step k) || decode(step k-1) on two streams; extra field, "
                             "not value"}
        # The same on disjoint CU sets (hipExtStreamCreateWithCUMask): each
        # kernel keeps its own LDS occupancy instead of the two thrashing each
        # other's.  Workgroups go round-robin to the XCDs, so every XCD gets the
        # same decode share (cu_partition_streams); the share is the one whose
        # slower kernel, each timed alone on its CUs, is fastest (untimed).
        cu = choose_cu_partition(
            dev_index, lambda s: batch.encode(raws[0], comps[0], s),
            lambda s: batch.decode(comps[0], outs[0], stats[0], s))
        # Every rank runs the leg or none does (its barrier is collective).
        have = -shard.max_over_ranks(-(1.0 if cu is not None else 0.0), dist)
        if cu is not None and have < 1.0:
            import ctypes as C
            for st in cu[:2]:
                C.CDLL("libamdhip64.so").hipStreamDestroy(C.c_void_p(st.cuda_stream))
            cu = None
        if cu is not None:
            s_enc, s_dec, split, alone = cu
            batch.encode(raws[0], comps[0], s_enc)
            enc_done[0].record(s_enc)
            torch.cuda.synchronize()
            if dist:
                dist.barrier()
            t0p = time.perf_counter()
            for k in range(1, a.steps + 1):
                j, jp = k % a.copies, (k - 1) % a.copies
                if k >= a.copies:
                    s_enc.wait_event(dec_done[j])
                batch.encode(raws[j], comps[j], s_enc)
                enc_done[j].record(s_enc)
                s_dec.wait_event(enc_done[jp])
                batch.decode(comps[jp], outs[jp], stats[jp], s_dec)
                dec_done[jp].record(s_dec)
            torch.cuda.synchronize()
            tp = shard.max_over_ranks(time.perf_counter() - t0p, dist)
            pipelined["cu_partition"] = {
                "GiBps": raw_bytes * world * a.steps / tp / 2**30,
                "ms_per_step": tp / a.steps * 1e3, "cus_encode_decode": split,
                "alone_us_encode_decode": alone,
                "note": "encode and decode streams on disjoint CU sets (the same decode CUs "
                        "in every XCD), the split whose slower kernel alone is fastest"}
            # Release the masked queues: later legs' streams must not land on them.
            import ctypes as C
            hip = C.CDLL("libamdhip64.so")
            torch.cuda.synchronize()
            for st in (s_enc, s_dec):
                hip.hipStreamDestroy(C.c_void_p(st.cuda_stream))

    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    comp_bytes = int(comps[0].len.sum(dtype=torch.int64).item())

    # ---- parity of this run's output (after the timed region) ----
    parity = None
    hc = None
    if not a.no_parity:
        ok = all(bool((s == 1).all()) for s in stats)
        hc = batch.to_host(comps[0])
        ho = batch.to_host(outs[(a.warmup + a.steps - 1) % a.copies])
        ok = ok and np.array_equal(corpus.block_digests(ho.buf, ho.off, ho.len),
                                   corpus.block_digests(c.buf, c.off, c.len))
        per = corpus.block_digests(hc.buf, hc.off, hc.len)
        for x in comps[1:]:
            hx = batch.to_host(x)
            ok = ok and np.array_equal(corpus.block_digests(hx.buf, hx.off, hx.len), per)
        oks = [None] * world
        if dist:
            dist.all_gather_object(oks, ok)
        else:
            oks = [ok]
        allb = gather_digests(dist, rank, world, per, total)
        if rank == 0:
            ref = reference_digest(total, a)
            dd = corpus.digest_of_digests(allb)
            if not all(oks):
                parity = "MISMATCH (a rank's round trip or status failed)"
            elif ref is None:
                parity = "round trip exact, status all ok (no pinned digest for this stream)"
            elif dd == ref["comp_dd"]:
                parity = (f"compressed blocks == reference ({ref['name']} digest of per-block "
                          f"digests, {world} rank(s) re-interleaved), round trip exact")
            else:
                parity = f"MISMATCH against {ref['name']}"

    tot_units = raw_bytes * world * a.steps
    value = tot_units / elapsed / 2**30
    alg = raw_bytes + comp_bytes + 16 * n   # SURVEY §8d per-block bytes x blocks, one launch
    kern = {
        "encode": {"avg_ms": enc_ms, "alg_bytes": alg,
                   "achieved_GBps": alg / (enc_ms * 1e-3) / 1e9,
                   "GiBps_uncompressed": raw_bytes / (enc_ms * 1e-3) / 2**30},
        "decode": {"avg_ms": dec_ms, "alg_bytes": alg,
                   "achieved_GBps": alg / (dec_ms * 1e-3) / 1e9,
                   "GiBps_uncompressed": raw_bytes / (dec_ms * 1e-3) / 2**30},
    }
    dom = "encode" if enc_ms >= dec_ms else "decode"
    traffic, traffic_note = None, "no PMC summary for this workload"
    try:
        tr = json.load(open(a.traffic))
        if tr.get("blocks") == n and dom in tr.get("kernels", {}):
            if tr.get("sources_sha") == kernel_sources_sha():
                traffic = tr["kernels"][dom].get("hbm_bytes_per_launch")
                traffic_note = (f"PMC profile {tr['kernels'][dom].get('profile')} of these "
                                f"kernel sources ({tr['sources_sha']}), 2*FETCH_SIZE+WRITE_SIZE")
            else:
                traffic_note = "PMC summary is from other kernel sources: dropped"
    except (OSError, ValueError):
        pass
    copy = achievable_copy_gbps(dev, stream) if not a.no_copy_probe else None
    copy_gbps = copy["best"] if copy else None
    roof = {"bound": "hbm", "kernel": dom, "achieved": kern[dom]["achieved_GBps"],
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": kern[dom]["achieved_GBps"] / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_note": traffic_note,
            "alg_bytes_per_block": "raw_len + comp_len + 16 (SURVEY §8d)",
            # both directions' algorithmic bytes over both kernels' time
            "combined_encode_decode": {"achieved": 2 * alg / ((enc_ms + dec_ms) * 1e-3) / 1e9,
                                       "frac": 2 * alg / ((enc_ms + dec_ms) * 1e-3) / 1e9
                                       / HBM_PEAK_GBS},
            # the same box's measured HBM ceiling: a 1 GiB device-to-device copy
            "achievable_copy_GBps": copy_gbps, "copy_probes_GBps": copy,
            "frac_of_achievable": (kern[dom]["achieved_GBps"] / copy_gbps) if copy_gbps else None}

    cpu = None
    if rank == 0 and not a.no_cpu_baseline:
        cpu = cpu_baseline(c, a, hc, world)

    # ---- extra (not `value`): SURVEY §8(f) rows 2-3 on the same C2 blocks,
    # the batched table write (encode + 12.5 % rule + trailers + packing)
    # and read (truncation + checksums + decode), against the codec kernels.
    tables = None
    if world == 1 and not a.no_table:
        tables = table_paths(c, raws[0], stream, enc_ms, dec_ms)

    # ---- extra (not `value`): BASELINE.json configs[2] on this GPU, after
    # everything above, with its own buffers (the C2 ones are freed first).
    c3 = None
    if world == 1 and not a.no_c3:
        del raws, comps, outs, stats
        torch.cuda.empty_cache()
        c3 = c3_mixed(a, dev, stream)

    if rank == 0:
        line = {
            "metric": baseline["metric"], "value": value, "unit": "GiB/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "weak" if a.blocks else "strong", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": workload_name(total, a, world),
                       "total_blocks": total, "blocks_rank0": n,
                       "raw_bytes_rank0": raw_bytes, "comp_bytes_rank0": comp_bytes,
                       "ratio": comp_bytes / raw_bytes,
                       "partition": "round-robin block g -> rank g % N, no collective",
                       "process_group": "gloo (barrier, max-over-ranks, parity gather)",
                       "devices": ("%d ranks SHARE %d visible GPU(s): a rehearsal, not an "
                                   "N-GPU measurement" % (world, ndev)) if shared
                                  else "one GPU per rank",
                       "copies_rotated": a.copies},
            "per_rank_elapsed_s": {"min": min(per_rank), "max": max(per_rank),
                                   "ranks": [round(x, 6) for x in per_rank]},
            "encode_GiBps": raw_bytes * world / (enc_ms * 1e-3) / 2**30,
            "decode_GiBps": raw_bytes * world / (dec_ms * 1e-3) / 2**30,
            "kernels": kern, "roofline": roof, "cpu_baseline": cpu, "parity": parity,
            "pipelined": pipelined, "c3": c3, "table": tables,
            "gen_seconds": t_gen,
        }
        print(json.dumps(line), flush=True)


def table_paths(c, raw, stream, enc_ms: float, dec_ms: float) -> dict:
    """lgs_table_write_dev / lgs_table_read_dev (verify_checksums on) over the
    C2 blocks, buffers allocated once, HIP events on the launch stream, median
    of 10 after 2 warm-ups; the read-back is checked against the raw blocks."""
    import torch
    from lcdb_amd import batch, table
    n = c.n
    raw_bytes = c.raw_bytes
    max_len = int(c.len.max())

    def timed(fn) -> float:
        ts = []
        for k in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            if k >= 2:
                ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    bufs = table.write_buffers(n, raw_bytes, raw.buf.device)
    w_ms = timed(lambda: table.write_blocks(raw.buf, raw.off, raw.len, 1, 0, max_len, raw_bytes,
                                            stream, bufs))
    d_file, hoff, hsize, end, _ = bufs
    file_len = int(end.cpu()[0])
    dec = batch.decode_slots(c.len, raw.buf.device)
    olen = torch.zeros(n, dtype=torch.int32, device=raw.buf.device)
    st = torch.zeros(n, dtype=torch.uint8, device=raw.buf.device)
    scr = torch.empty(max(int(table._L.lgs_table_read_scratch(n)), 1), dtype=torch.uint8,
                      device=raw.buf.device)
    # lcdb's default ReadOptions do not verify checksums (util/options.c:43-47):
    # the same read without the trailer CRCs
    r0_ms = timed(lambda: table.read_blocks(d_file, file_len, hoff, hsize, dec.buf, dec.off,
                                            dec.cap, dec.max_cap, False, olen, st, stream, scr))
    ok = bool((st == 1).all()) and torch.equal(olen, raw.len)
    r_ms = timed(lambda: table.read_blocks(d_file, file_len, hoff, hsize, dec.buf, dec.off,
                                           dec.cap, dec.max_cap, True, olen, st, stream, scr))
    ok = ok and bool((st == 1).all()) and torch.equal(olen, raw.len)
    ho = batch.to_host(dec)
    ho.len = olen.cpu().numpy().astype(np.uint32)
    ok = ok and np.array_equal(corpus_digests(ho), corpus_digests(c))
    res = {"workload": f"C2 framing: {n} blocks, device-resident; read with verify_checksums on "
                       f"(read_ms) and off, lcdb's default (read_noverify_ms)",
           "file_bytes": file_len,
           "write_ms": w_ms, "write_GiBps_raw": raw_bytes / (w_ms * 1e-3) / 2**30,
           "read_ms": r_ms, "read_GiBps_raw": raw_bytes / (r_ms * 1e-3) / 2**30,
           "write_over_encode": w_ms / enc_ms, "read_over_decode": r_ms / dec_ms,
           "read_noverify_ms": r0_ms, "read_noverify_over_decode": r0_ms / dec_ms,
           "parity": "write -> read round trip exact, every checksum verified" if ok
                     else "MISMATCH",
           "note": "extra field (SURVEY §8(f) rows 2-3), not value"}
    del bufs, d_file, dec, scr
    torch.cuda.empty_cache()
    return res


def corpus_digests(c):
    from lcdb_amd import corpus
    return corpus.block_digests(c.buf, c.off, c.len)


N_XCD = 8        # MI355X: 8 XCDs of 32 CUs


def choose_cu_partition(dev_index: int, enc_fn, dec_fn, shares=range(8, 17)):
    """The decode share (CUs per XCD) whose slower kernel, each timed alone
    on its CU set with HIP events (best of 2 after a warm-up), is fastest.
    Returns (encode stream, decode stream, [n_encode_cus, n_decode_cus],
    [encode_us, decode_us]) or None where masks are refused.  The streams of
    the other shares are destroyed."""
    import ctypes as C
    import torch
    hip = C.CDLL("libamdhip64.so")

    def alone(fn, s):
        ts = []
        for k in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn(s)
            e1.record(s)
            e1.synchronize()
            if k:
                ts.append(e0.elapsed_time(e1) * 1e3)
        return min(ts)

    best = None
    for nx in shares:
        cu = cu_partition_streams(dev_index, nx)
        if cu is None:
            return None
        s_enc, s_dec, split = cu
        t = [round(alone(enc_fn, s_enc), 1), round(alone(dec_fn, s_dec), 1)]
        if best is None or max(t) < max(best[3]):
            if best is not None:
                hip.hipStreamDestroy(C.c_void_p(best[0].cuda_stream))
                hip.hipStreamDestroy(C.c_void_p(best[1].cuda_stream))
            best = (s_enc, s_dec, split, t)
        else:
            hip.hipStreamDestroy(C.c_void_p(s_enc.cuda_stream))
            hip.hipStreamDestroy(C.c_void_p(s_dec.cuda_stream))
    return best


def cu_partition_streams(dev_index: int, dec_per_xcd: int):
    """Two HIP streams on disjoint CUs of this GPU: dec_per_xcd CUs of every
    XCD for the decode stream, the rest for the encode stream.  Returns
    (encode stream, decode stream, [n_encode_cus, n_decode_cus]) as torch
    ExternalStreams, or None where the runtime refuses the mask.

    Mask bit i belongs to XCD i % N_XCD (measured, tools/cu_mask_map.py,
    profiles/r5y_cu_mask_map.json: bits [0, 8k) run a kernel on about 8k
    CUs, while one bit in eight -- all of one XCD -- runs it on the whole
    chip: an XCD left without a bit is not masked at all).  So the decode
    share is the contiguous bits [0, N_XCD * dec_per_xcd)."""
    import ctypes as C
    import torch
    try:
        hip = C.CDLL("libamdhip64.so")
    except OSError:
        return None
    ncu = torch.cuda.get_device_properties(dev_index).multi_processor_count
    words = (ncu + 31) // 32
    enc, dec = [0] * words, [0] * words
    for i in range(ncu):
        (dec if i < N_XCD * dec_per_xcd else enc)[i // 32] |= 1 << (i % 32)
    out = []
    for m in (enc, dec):
        s = C.c_void_p()
        if hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(words),
                                            (C.c_uint32 * words)(*m)) != 0:
            return None
        out.append(torch.cuda.ExternalStream(s.value, device=torch.device("cuda", dev_index)))
    return out[0], out[1], [sum(bin(x).count("1") for x in enc),
                            sum(bin(x).count("1") for x in dec)]


def c3_mixed(a, dev, stream) -> dict:
    """BASELINE.json configs[2] (C3): 4/16/64 KiB blocks, half db_bench
    fillseq, half uniform random (corpus.mixed), at --c3-scale.  Each class
    as its own batch and the whole mix as one batch (the split launch sorts
    it into classes on the device); HIP events on the launch stream, median
    of 10 after 2 warm-ups; every decode round-trip checked, the mix's
    compressed blocks diffed against the pinned reference digest."""
    import torch
    from lcdb_amd import batch, corpus
    scale = a.c3_scale

    def timed(fn) -> float:
        ts = []
        for k in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            if k >= 2:
                ts.append(e0.elapsed_time(e1) * 1e-3)
        return float(np.median(ts))

    def one(c) -> tuple[dict, object]:
        raw = batch.upload(c, dev)
        comp = batch.encode_slots(raw)
        out = batch.decode_slots(c.len, dev)
        st = torch.zeros(c.n, dtype=torch.uint8, device=dev)
        t_e = timed(lambda: batch.encode(raw, comp, stream))
        t_d = timed(lambda: batch.decode(comp, out, st, stream))
        ho = batch.to_host(out)
        ok = bool((st == 1).all()) and np.array_equal(
            corpus.block_digests(ho.buf, ho.off, ho.len), corpus.block_digests(c.buf, c.off, c.len))
        rb, cb = c.raw_bytes, int(comp.len.sum(dtype=torch.int64).item())
        hc = batch.to_host(comp)
        del raw, out, st, comp
        torch.cuda.empty_cache()
        return ({"blocks": c.n, "raw_bytes": rb, "ratio": cb / rb,
                 "encode_GiBps": rb / t_e / 2**30, "decode_GiBps": rb / t_d / 2**30,
                 "encode_ms": t_e * 1e3, "decode_ms": t_d * 1e3, "roundtrip_ok": ok}, hc)

    classes = {}
    for bs, n in ((4096, 512), (16384, 128), (65536, 32)):
        for kind in ("fillseq", "random"):
            c = (corpus.fillseq(n * scale, block_size=bs, key0=bs) if kind == "fillseq"
                 else corpus.random_blocks(n * scale, bs, seed=0x5EED + bs))
            classes[f"{kind}_{bs // 1024}K"] = one(c)[0]
    mix, hc = one(corpus.mixed(scale))
    dg = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
    ref = dg.get("C3_mixed" if scale == 1 else f"C3_mixed_x{scale}")
    ok = all(r["roundtrip_ok"] for r in classes.values()) and mix["roundtrip_ok"]
    if ref is None:
        parity = "round trips exact" if ok else "MISMATCH (round trip or status)"
    else:
        same = corpus.digest_of_digests(corpus.block_digests(hc.buf, hc.off, hc.len)) == \
            ref["comp_dd"]
        parity = ("round trips exact, mix's compressed blocks == reference digest"
                  if ok and same else "MISMATCH against the reference digest")
    return {"workload": f"C3: mixed 4/16/64 KiB, half fillseq / half random, scale {scale} "
                        f"({mix['blocks']} blocks, {mix['raw_bytes']} B)",
            "classes": classes, "mixed_one_launch": mix, "parity": parity,
            "note": "extra field (BASELINE.json configs[2]), not value"}


def achievable_copy_gbps(dev, stream) -> dict:
    """HBM bytes (read + write) per second of a 1 GiB device-to-device copy
    on this GPU (report an achievable rate beside the spec peak),
    median of 10, HIP events on the launch stream: the library's own
    16-bytes-per-lane streaming copy (lgs_hbm_copy_dev) and torch's copy_;
    the higher one is the yardstick."""
    import torch
    from lcdb_amd import _native
    n = 1 << 30
    src = torch.empty(n, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    src.fill_(1)
    lib = _native.lib()

    def lgs_copy():
        _native.check(lib.lgs_hbm_copy_dev(dst.data_ptr(), src.data_ptr(), n,
                                           stream.cuda_stream), "lgs_hbm_copy_dev")

    def med(fn) -> float:
        times = []
        with torch.cuda.stream(stream):
            for k in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                fn()
                e1.record(stream)
                e1.synchronize()
                if k >= 2:
                    times.append(e0.elapsed_time(e1) * 1e-3)
        return 2 * n / float(np.median(times)) / 1e9

    r = {"lgs_hbm_copy": med(lgs_copy), "torch_copy": med(lambda: dst.copy_(src))}
    if not torch.equal(dst[:1 << 20], src[:1 << 20]):
        raise RuntimeError("copy probe produced wrong bytes")
    del src, dst
    torch.cuda.empty_cache()
    r["best"] = max(r["lgs_hbm_copy"], r["torch_copy"])
    return r


def cpu_threads_share(a) -> int:
    if a.cpu_threads:
        return a.cpu_threads
    share = len(os.sched_getaffinity(0))
    for var in ("OMP_NUM_THREADS",):      # the GPU box sets the per-GPU CPU share here
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            share = min(share, int(v))
    return max(1, min(16, share))


def cpu_baseline(c, a, gpu_comp, world: int) -> dict:
    """BASELINE.md's CPU-baseline plan: the reference snappy.c (oracle/_ref,
    compiled unmodified) over the first `--cpu-sample` of this GPU's blocks
    (all of C2), at 1 thread, at the host's per-GPU thread share and at
    `nproc` threads (the process's affinity set: the whole node), warm-up +
    median of 5, compressed bytes checked against the GPU's.  Multi-thread
    points run with both block partitions of cpu_batch.c (static
    round-robin, as the plan says, and contiguous), each into fresh
    buffers first-touched by its own worker threads (NUMA-local pages);
    the headline is the `nproc` point's faster partition -- the node's
    CPUs against the node's GPUs (at N > 1 this is rank 0's node-level
    comparison).  `cores` = physical cores the threads occupy."""
    import oracle
    codec, kind = oracle.reference(), "reference"
    if codec is None:
        codec, kind = oracle.restatement(), "port"
    share = cpu_threads_share(a)
    nproc = len(os.sched_getaffinity(0))
    m = min(a.cpu_sample, c.n)
    off, ln = c.off[:m].copy(), c.len[:m].copy()
    counts = sorted({1, share, nproc})
    plan = oracle.baseline_plan(codec, c.buf, off, ln, counts, reps=a.cpu_reps, partitions=(0, 1))
    same = None
    if gpu_comp is not None:
        from lcdb_amd import corpus
        co, coo, col = plan["comp"]
        same = bool(np.array_equal(corpus.block_digests(co, coo, col),
                                   corpus.block_digests(gpu_comp.buf, gpu_comp.off[:m],
                                                        gpu_comp.len[:m])))
    pt = plan["per_threads"]
    pname = {0: "round-robin", 1: "contiguous"}

    def point(t: int) -> dict:
        parts = {pname[p]: {k: v[k] for k in ("roundtrip_GiBps", "encode_GiBps", "decode_GiBps")}
                 for (tt, p), v in pt.items() if tt == t}
        best = max(parts, key=lambda k: parts[k]["roundtrip_GiBps"])
        return dict(parts[best], threads=t, cores=oracle.cores_for_threads(t), partition=best,
                    by_partition=parts)

    pts = {t: point(t) for t in counts}
    # the headline: the fastest point (the whole node's CPUs, nproc, unless
    # fewer threads do better on this sample -- as on a shared GPU box whose
    # container is held to a CPU quota, reported as cgroup_cpu_quota)
    top = max(pts.values(), key=lambda x: x["roundtrip_GiBps"])
    host = oracle.cpu_model()
    return {"value": top["roundtrip_GiBps"], "unit": "GiB/s", "cores": top["cores"],
            "threads": top["threads"], "kind": kind, "partition": top["partition"],
            "encode_GiBps": top["encode_GiBps"], "decode_GiBps": top["decode_GiBps"],
            "nproc": pts[nproc], "per_gpu_share": pts[share], "single_thread": pts[1],
            "cpu_model": host["model"], "physical_cores": host["physical_cores"],
            "logical_cpus": host["logical_cpus"], "affinity_cpus": host["affinity_cpus"],
            "affinity_physical_cores": host["affinity_physical_cores"],
            "numa_nodes": host["numa_nodes"], "cgroup_cpu_quota": host["cgroup_cpu_quota"],
            "gpus_in_this_run": world, "same_bytes_as_gpu": same,
            "sample": f"first {m} of rank 0's blocks ({plan['raw_bytes']} B raw), encode then "
                      f"decode, warm-up + median of {a.cpu_reps} runs, at {counts} threads "
                      f"(round-robin and contiguous partitions, NUMA-local outputs)"}


if __name__ == "__main__":
    sys.exit(main())
