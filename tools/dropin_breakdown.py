#!/usr/bin/env python3
"""Where a drop-in call's time goes: one 4 KiB fillseq block.

  kernel    the batch kernel on that one block, device-resident, HIP events
            (the block's serial chain on one wave of an idle GPU)
  floor     the same 16-byte copy kernel between two HIP events (what the
            event pair adds to a kernel time above)
  launch    an empty-work launch + stream synchronisation through the same
            library (lgs_hbm_copy_dev of 16 bytes, then torch.cuda.synchronize)
  dropin    ldb_snappy_encode / ldb_snappy_decode from the host (pageable
            buffers, the slot's mapped pinned memory, one synchronisation)

Prints one JSON line of medians in microseconds."""
from __future__ import annotations

import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import numpy as np
    import torch

    from lcdb_amd import _native, batch, corpus
    L = _native.lib()
    reps = int(os.environ.get("REPS", "400"))
    c = corpus.fillseq(8)
    one = corpus.Corpus(c.buf, c.off[:1].copy(), c.len[:1].copy())
    raw = batch.upload(one)
    comp = batch.encode_slots(raw)
    out = batch.decode_slots(one.len)
    st = torch.zeros(1, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    def ev_time(fn):
        ts = []
        for k in range(reps + 20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            if k >= 20:
                ts.append(e0.elapsed_time(e1) * 1e3)
        return float(np.median(ts))

    def wall(fn):
        ts = []
        for k in range(reps + 20):
            t0 = time.perf_counter()
            fn()
            if k >= 20:
                ts.append((time.perf_counter() - t0) * 1e6)
        return float(np.median(ts))

    res = {"block_bytes": int(one.len[0])}
    res["kernel_encode_us"] = ev_time(lambda: batch.encode(raw, comp, s))
    res["kernel_decode_us"] = ev_time(lambda: batch.decode(comp, out, st, s))
    a = torch.zeros(64, dtype=torch.uint8, device="cuda")
    b = torch.zeros(64, dtype=torch.uint8, device="cuda")

    def empty():
        L.lgs_hbm_copy_dev(C.c_void_p(b.data_ptr()), C.c_void_p(a.data_ptr()), 16, None)
        torch.cuda.synchronize()
    res["launch_sync_us"] = wall(empty)
    res["event_floor_us"] = ev_time(lambda: L.lgs_hbm_copy_dev(
        C.c_void_p(b.data_ptr()), C.c_void_p(a.data_ptr()), 16, C.c_void_p(s.cuda_stream)))
    blk = bytes(c.buf[c.off[0]:c.off[0] + c.len[0]])
    src = C.create_string_buffer(blk + b"\0" * 16, len(blk) + 16)
    dst = C.create_string_buffer(8192)
    n = L.ldb_snappy_encode(dst, src, len(blk))
    enc = C.create_string_buffer(dst.raw[:n] + b"\0" * 16, n + 16)
    o = C.create_string_buffer(8192)
    res["dropin_encode_us"] = wall(lambda: L.ldb_snappy_encode(dst, src, len(blk)))
    res["dropin_decode_us"] = wall(lambda: L.ldb_snappy_decode(o, enc, n))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
