#!/usr/bin/env python3
"""Phases of an encode wave's life on C2, from a probe build with
-DLGS_PROBE_ENC_TIMING (each wave stores two shader-clock intervals in the
last 16 bytes of its output slot): staging (per-block arrays, the block's
bytes into LDS) and the rest (table, parse, emission).

usage: python tools/enc_phases.py PROBE_SO
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
    for _ in range(3):
        batch.encode(raw, comp)
    torch.cuda.synchronize()
    buf = comp.buf.cpu().numpy()
    off = comp.off.cpu().numpy().astype(np.int64)
    bound = 32 + c.len.astype(np.int64) + c.len.astype(np.int64) // 6
    at = off + bound - 16
    words = np.stack([buf[at + k] for k in range(12)], axis=1).astype(np.uint32)
    w = words[:, 0::4] | (words[:, 1::4] << 8) | (words[:, 2::4] << 16) | (words[:, 3::4] << 24)
    ok = w[:, 2] == 0x7E57
    stage, rest = w[ok, 0].astype(np.float64), w[ok, 1].astype(np.float64)
    print(json.dumps({"waves": int(ok.sum()), "stage_cycles_mean": stage.mean(),
                      "stage_cycles_p50": float(np.median(stage)), "rest_cycles_mean": rest.mean(),
                      "rest_cycles_p50": float(np.median(rest)),
                      "stage_frac": float(stage.mean() / (stage.mean() + rest.mean()))}))


if __name__ == "__main__":
    main()
