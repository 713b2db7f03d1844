#!/usr/bin/env python3
"""Decode time of the ring and the wave decoder against batch size, on
fillseq and random 4 KiB blocks: where the automatic choice should switch
(lgs_decode.hip kLaneMinBlocks).  HIP events, mean of 10 after 3 warm-ups;
every run's statuses and decoded bytes are checked.  One JSON line per point.

usage: python tools/sweep_decoders.py [--lib SO] [--sizes 8192,16384,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None)
    p.add_argument("--sizes", default="8192,16384,24576,32768,40960,49152,65536")
    a = p.parse_args()
    if a.lib:
        import lcdb_amd.build as b
        b.LIB = os.path.abspath(a.lib)
    import numpy as np
    import torch
    from lcdb_amd import _native, batch, corpus
    s = torch.cuda.current_stream()
    for kind in ("fillseq", "random"):
        for n in [int(x) for x in a.sizes.split(",")]:
            c = corpus.fillseq(n) if kind == "fillseq" else corpus.random_blocks(n, 4096,
                                                                                seed=0x5EED)
            raw = batch.upload(c)
            comp = batch.encode_slots(raw)
            batch.encode(raw, comp, s)
            out = batch.decode_slots(c.len)
            st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
            row = {"kind": kind, "blocks": n}
            for dec in ("ring", "wave"):
                _native.set_option("decoder", dec)
                ts = []
                for k in range(13):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    batch.decode(comp, out, st, s)
                    e1.record(s)
                    e1.synchronize()
                    if k >= 3:
                        ts.append(e0.elapsed_time(e1) * 1e3)
                ho = batch.to_host(out)
                ok = bool((st == 1).all()) and np.array_equal(
                    corpus.block_digests(ho.buf, ho.off, ho.len),
                    corpus.block_digests(c.buf, c.off, c.len))
                row[dec + "_us"] = float(np.mean(ts))
                row[dec + "_GiBps"] = c.raw_bytes / (row[dec + "_us"] * 1e-6) / 2**30
                row[dec + "_ok"] = ok
            _native.set_option("decoder", "auto")
            print(json.dumps(row), flush=True)
            del raw, comp, out, st
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
