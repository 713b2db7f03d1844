#!/usr/bin/env python3
"""Trips per wave of the ring decoder on C2, from a probe build with
-DLGS_PROBE_TRIPCOUNT (the kernel writes its wave's trip count to out_len).
Divides a PMC pass's per-wave instruction counts into per-trip counts.

usage: python tools/ring_trips.py PROBE_SO
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import lcdb_amd.build as b
    b.LIB = os.path.abspath(sys.argv[1])
    import numpy as np
    import torch
    from lcdb_amd import batch, corpus
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    batch.decode(comp, out, st)
    torch.cuda.synchronize()
    trips = out.len.cpu().numpy().astype(np.int64).reshape(-1, 32)   # 32 blocks per wave
    per_wave = trips.max(axis=1)
    print(json.dumps({"waves": int(per_wave.size), "trips_mean": float(per_wave.mean()),
                      "trips_min": int(per_wave.min()), "trips_max": int(per_wave.max()),
                      "status_ok": bool((st == 1).all())}))


if __name__ == "__main__":
    main()
