#!/usr/bin/env python3
"""C2 encode and decode on CU-masked streams (hipExtStreamCreateWithCUMask,
bench.py's cu_partition_streams): each kernel alone on its share, then both
at once, for a few decode shares (CUs per XCD, every XCD alike).  Tells whether a partitioned kernel runs in
the time its share predicts (pipelined).

usage: python tools/cu_mask_probe.py [DEC_CUS_PER_XCD ...]      (default 11 10 12 16)
Prints one JSON line per share: HIP-event medians in microseconds.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import numpy as np
    import torch

    import bench
    from lcdb_amd import batch, corpus
    torch.cuda.set_device(0)
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    batch.encode(raw, comp)
    raw2 = batch.upload(c)
    comp2 = batch.encode_slots(raw2)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def timed(fn, streams, reps=7):
        ts = []
        for k in range(reps + 2):
            torch.cuda.synchronize()
            e0 = [torch.cuda.Event(enable_timing=True) for _ in streams]
            e1 = [torch.cuda.Event(enable_timing=True) for _ in streams]
            for s, e in zip(streams, e0):
                e.record(s)
            fn()
            for s, e in zip(streams, e1):
                e.record(s)
            torch.cuda.synchronize()
            if k >= 2:
                ts.append([a.elapsed_time(b) * 1e3 for a, b in zip(e0, e1)])
        return [float(np.median([t[i] for t in ts])) for i in range(len(streams))]

    full = torch.cuda.current_stream()
    base = {"encode_full_us": timed(lambda: batch.encode(raw2, comp2, full), [full])[0],
            "decode_full_us": timed(lambda: batch.decode(comp, out, st, full), [full])[0]}
    print(json.dumps(base), flush=True)
    for nd in [int(x) for x in sys.argv[1:]] or [11, 10, 12, 16]:
        s_enc, s_dec, split = bench.cu_partition_streams(0, nd)
        r = {"cus_encode_decode": split}
        r["encode_alone_us"] = timed(lambda: batch.encode(raw2, comp2, s_enc), [s_enc])[0]
        r["decode_alone_us"] = timed(lambda: batch.decode(comp, out, st, s_dec), [s_dec])[0]

        def both():
            batch.encode(raw2, comp2, s_enc)
            batch.decode(comp, out, st, s_dec)
        r["together_encode_us"], r["together_decode_us"] = timed(both, [s_enc, s_dec])
        r["status_ok"] = bool((st == 1).all())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
