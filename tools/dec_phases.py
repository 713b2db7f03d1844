#!/usr/bin/env python3
"""Phases of a wave-decoder wave's life (decode_kernel, the drop-in's and the
small batches' decoder), from a probe build with -DLGS_PROBE_DEC_TIMING: each
wave stores the shader-clock cycles of staging (per-block arrays, the stream
into LDS), the tag walk (decode_win) and the output flush, plus the 100 MHz
real-time ticks of the whole, in the last 16 bytes of its output capacity.

usage: python tools/dec_phases.py PROBE_SO [N_BLOCKS ...]
Prints one JSON line per batch size: medians, and the shader clock in MHz.
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
    sizes = [int(x) for x in sys.argv[2:]] or [1, 64]
    for n in sizes:
        c = corpus.fillseq(n)
        raw = batch.upload(c)
        comp = batch.encode_slots(raw)
        batch.encode(raw, comp)
        out = batch.decode_slots(c.len.astype(np.uint64) + 32)
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        rows = []
        for _ in range(50):
            batch.decode(comp, out, st)
            torch.cuda.synchronize()
            buf = out.buf.cpu().numpy()
            off = out.off.cpu().numpy().astype(np.int64)
            cap = out.cap.cpu().numpy().astype(np.int64)
            at = off + ((cap - 16) & ~3)
            words = np.stack([buf[at + k] for k in range(16)], axis=1).astype(np.uint64)
            w = words[:, 0::4] | (words[:, 1::4] << 8) | (words[:, 2::4] << 16) | (words[:, 3::4] << 24)
            rows.append(w)
        w = np.concatenate(rows).astype(np.float64)
        assert bool((st.cpu().numpy() == 1).all())
        stage, walk, flush, rt = (np.median(w[:, k]) for k in range(4))
        clk = (w[:, 0] + w[:, 1] + w[:, 2]) / (w[:, 3] / 100.0)        # cycles per us = MHz
        print(json.dumps({"blocks": n, "stage_cycles": stage, "walk_cycles": walk,
                          "flush_cycles": flush, "total_us_realtime": rt / 100.0,
                          "shader_MHz_p50": float(np.median(clk))}))


if __name__ == "__main__":
    main()
