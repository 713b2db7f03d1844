#!/usr/bin/env python3
"""Concurrent encode || decode on C2 (bench.py's `pipelined` shape) under
stream-priority variants, against the sequential step (timing only).

Step k encodes copy k % 2 on one stream while decoding what step k-1 encoded
on another; each variant sets the two streams' priorities (torch: lower
number = higher priority).  Prints one JSON line per variant: GiB/s of raw
bytes through both directions per step, ms per step, and the statuses.

usage: python tools/pipe_ab.py [STEPS]
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    from lcdb_amd import batch, corpus
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    c = corpus.fillseq(65536)
    raws = [batch.upload(c) for _ in range(2)]
    comps = [batch.encode_slots(r) for r in raws]
    outs = [batch.decode_slots(c.len) for _ in range(2)]
    sts = [torch.zeros(c.n, dtype=torch.uint8, device="cuda") for _ in range(2)]
    s0 = torch.cuda.current_stream()
    for k in range(4):
        batch.encode(raws[k % 2], comps[k % 2], s0)
        batch.decode(comps[k % 2], outs[k % 2], sts[k % 2], s0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        batch.encode(raws[k % 2], comps[k % 2], s0)
        batch.decode(comps[k % 2], outs[k % 2], sts[k % 2], s0)
    torch.cuda.synchronize()
    seq = (time.perf_counter() - t0) / steps
    print(json.dumps({"variant": "sequential", "ms_per_step": seq * 1e3,
                      "GiBps": c.raw_bytes / seq / 2**30}), flush=True)
    for name, pe, pd in (("equal", 0, 0), ("decode_high", 0, -1), ("encode_high", -1, 0)):
        se = torch.cuda.Stream(priority=pe)
        sd = torch.cuda.Stream(priority=pd)
        enc_done = [torch.cuda.Event() for _ in range(2)]
        dec_done = [torch.cuda.Event() for _ in range(2)]
        for rep in range(2):          # the first pass warms up
            batch.encode(raws[0], comps[0], se)
            enc_done[0].record(se)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(1, steps + 1):
                j, jp = k % 2, (k - 1) % 2
                if k >= 2:
                    se.wait_event(dec_done[j])
                batch.encode(raws[j], comps[j], se)
                enc_done[j].record(se)
                sd.wait_event(enc_done[jp])
                batch.decode(comps[jp], outs[jp], sts[jp], sd)
                dec_done[jp].record(sd)
            torch.cuda.synchronize()
            tp = (time.perf_counter() - t0) / steps
        ok = all(bool((s == 1).all()) for s in sts)
        print(json.dumps({"variant": name, "ms_per_step": tp * 1e3,
                          "GiBps": c.raw_bytes / tp / 2**30, "status_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
