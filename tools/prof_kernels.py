#!/usr/bin/env python3
"""Run the encode / decode kernels on a resident corpus, for rocprofv3.

usage: python tools/prof_kernels.py [--blocks N] [--iters K] [--which encode,decode] [--lib SO]
Every launch is preceded by a sync so per-dispatch counters are clean.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))



def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None, help="a probe build of the codec library")
    p.add_argument("--blocks", type=int, default=65536)
    p.add_argument("--block-size", type=int, default=4096)
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--which", default="encode,decode")
    a = p.parse_args()
    if a.lib:
        import lcdb_amd.build as b
        b.LIB = os.path.abspath(a.lib)
    import torch
    from lcdb_amd import batch, corpus
    which = a.which.split(",")
    c = corpus.fillseq(a.blocks, block_size=a.block_size)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    batch.encode(raw, comp)
    torch.cuda.synchronize()
    for _ in range(a.iters):
        if "encode" in which:
            batch.encode(raw, comp)
            torch.cuda.synchronize()
        if "decode" in which:
            batch.decode(comp, out, st)
            torch.cuda.synchronize()
    assert bool((st == 1).all()) or "decode" not in which
    print("ok", c.n, c.raw_bytes, int(comp.len.sum().item()))


if __name__ == "__main__":
    main()
