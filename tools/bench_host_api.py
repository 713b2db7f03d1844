#!/usr/bin/env python3
"""Wall-clock rate of the C ABI's host-buffer entry points on BASELINE config 2
(pageable host memory in and out, as lcdb would call them; recorded in
DESIGN.md section 7, never bench.py's `value`):

* lgs_encode_batch_host / lgs_decode_batch_host (the batched codec), and
* lgs_table_write_host / lgs_table_read_host (the framed table paths).

Each call includes its staging into pinned memory, the transfers, the kernels
and the copy back.  Median of --reps after one warm-up call.  One JSON line.
usage: python tools/bench_host_api.py [--blocks 65536] [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--blocks", type=int, default=65536)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--lib", default=None, help="a probe build of the codec library")
    a = p.parse_args()
    if a.lib:
        import lcdb_amd.build as b
        b.LIB = os.path.abspath(a.lib)

    from lcdb_amd import _native, corpus  # noqa: E402
    from lcdb_amd._native import check

    L = _native.lib()
    c = corpus.fillseq(a.blocks)
    n = c.n
    raw = np.concatenate([c.buf, np.zeros(16, dtype=np.uint8)])
    roff = c.off.astype(np.uint64)
    rlen = c.len.astype(np.uint32)
    rb = c.raw_bytes
    bound = (32 + rlen.astype(np.uint64) + rlen.astype(np.uint64) // 6 + 15) & ~np.uint64(15)
    eoff = np.zeros(n, dtype=np.uint64)
    eoff[1:] = np.cumsum(bound[:-1])
    enc = np.empty(int(bound.sum()) + 16, dtype=np.uint8)
    elen = np.zeros(n, dtype=np.uint32)
    dec = np.empty(rb + 16 * n, dtype=np.uint8)
    dcap = (rlen + 15) & ~np.uint32(15)
    doff = np.zeros(n, dtype=np.uint64)
    doff[1:] = np.cumsum(dcap[:-1].astype(np.uint64))
    dlen = np.zeros(n, dtype=np.uint32)
    st = np.zeros(n, dtype=np.uint8)
    fcap = rb + 5 * n + 16
    fimg = np.empty(fcap, dtype=np.uint8)
    hoff = np.zeros(n, dtype=np.uint64)
    hsize = np.zeros(n, dtype=np.uint64)
    end = np.zeros(1, dtype=np.uint64)

    def timed(fn):
        fn()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    def encode():
        check(L.lgs_encode_batch_host(raw.ctypes.data, roff.ctypes.data, rlen.ctypes.data,
                                      enc.ctypes.data, eoff.ctypes.data, elen.ctypes.data, n),
              "lgs_encode_batch_host")

    def decode():
        check(L.lgs_decode_batch_host(enc.ctypes.data, eoff.ctypes.data, elen.ctypes.data,
                                      dec.ctypes.data, doff.ctypes.data, dcap.ctypes.data,
                                      dlen.ctypes.data, st.ctypes.data, n),
              "lgs_decode_batch_host")

    def twrite():
        check(L.lgs_table_write_host(raw.ctypes.data, roff.ctypes.data, rlen.ctypes.data, n, 1, 0,
                                     fimg.ctypes.data, fcap, hoff.ctypes.data, hsize.ctypes.data,
                                     end.ctypes.data),
              "lgs_table_write_host")

    def tread():
        check(L.lgs_table_read_host(fimg.ctypes.data, int(end[0]), hoff.ctypes.data,
                                    hsize.ctypes.data, n, 1, dec.ctypes.data, doff.ctypes.data,
                                    dcap.ctypes.data, dlen.ctypes.data, st.ctypes.data),
              "lgs_table_read_host")

    te = timed(encode)
    td = timed(decode)
    ok_codec = bool((st == 1).all()) and bool((dlen == rlen).all())
    tw = timed(twrite)
    tr = timed(tread)
    ok_table = bool((st == 1).all()) and bool((dlen == rlen).all())
    for i in range(n):                                        # every byte back
        o, m = int(doff[i]), int(rlen[i])
        if not np.array_equal(dec[o:o + m], c.buf[int(roff[i]):int(roff[i]) + m]):
            ok_table = False
            break
    g = 2 ** 30
    print(json.dumps({
        "workload": f"C2: {n} fillseq blocks, pageable host buffers",
        "raw_bytes": rb, "file_bytes": int(end[0]),
        "encode_host_GiBps": rb / te / g, "decode_host_GiBps": rb / td / g,
        "table_write_host_GiBps": rb / tw / g, "table_read_host_GiBps": rb / tr / g,
        "encode_ms": te * 1e3, "decode_ms": td * 1e3, "table_write_ms": tw * 1e3,
        "table_read_ms": tr * 1e3,
        "parity": "round trips exact" if ok_codec and ok_table else "FAILED"}))
    if not (ok_codec and ok_table):
        sys.exit(1)


if __name__ == "__main__":
    main()
