#!/usr/bin/env python3
"""Where a ring-decoder trip's cycles go (decode_ring_kernel on C2), from a
probe build with -DLGS_PROBE_RING_PHASES (lgs_probe_hooks.h): each wave sums
the shader-clock cycles (s_memtime) of its trip phases and lane k < 8 of the
wave writes phase k's sum into its block's out_len, lane 8 the trip count.

Phases: 0 first-slot piece (before the wait), 1 the trip's vmcnt(0),
2 far-copy and refill landing, 3 flush jobs, 4 first parse, 5 second slot
(piece + parse), 6 refill requests, 7 the loop test.  Each stamp is an
s_memtime whose use waits for every outstanding LDS operation too, so LDS
latency is charged to the phase whose operations are in flight at its end.

usage: python tools/ring_phases.py PROBE_SO [PRODUCT_SO]
Prints one JSON line: per-phase cycles per wave (median over waves), per
trip, the share of the wave's life, and the launch times of the probe and
(if given) the product library, HIP-event timed.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["piece1", "wait_vmcnt", "landing", "flush", "parse1", "slot2", "refill_req", "loop_test"]


def child(lib: str, phases: bool) -> dict:
    sys.path.insert(0, ROOT)
    import lcdb_amd.build as b
    b.LIB = os.path.abspath(lib)
    import numpy as np
    import torch
    from lcdb_amd import batch, corpus
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    ts = []
    for k in range(13):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        batch.decode(comp, out, st, s)
        e1.record(s)
        e1.synchronize()
        if k >= 3:
            ts.append(e0.elapsed_time(e1) * 1000.0)
    res = {"lib": os.path.basename(lib), "decode_us_p50": float(np.median(ts)),
           "status_ok": bool((st == 1).all())}
    if phases:
        v = out.len.cpu().numpy().astype(np.float64).reshape(-1, 32)   # 32 blocks per wave
        ph = v[:, :8]
        trips = v[:, 8]
        life = ph.sum(axis=1)
        med = np.median(ph, axis=0)
        res["waves"] = int(v.shape[0])
        res["trips_p50"] = float(np.median(trips))
        res["life_cycles_p50"] = float(np.median(life))
        res["life_cycles_max"] = float(life.max())
        res["phase_cycles_per_wave_p50"] = {n: float(x) for n, x in zip(NAMES, med)}
        res["phase_cycles_per_trip"] = {n: round(float(x) / float(np.median(trips)), 1)
                                        for n, x in zip(NAMES, med)}
        res["phase_share"] = {n: round(float(x) / float(med.sum()), 3) for n, x in zip(NAMES, med)}
    return res


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        print(json.dumps(child(sys.argv[2], sys.argv[3] == "1")))
        return
    libs = [(sys.argv[1], "1")] + ([(sys.argv[2], "0")] if len(sys.argv) > 2 else [])
    out = {}
    for lib, ph in libs:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib, ph],
                           capture_output=True, text=True, check=True)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        d = json.loads(line)
        out["probe" if ph == "1" else "product"] = d
    print(json.dumps(out))


if __name__ == "__main__":
    main()
