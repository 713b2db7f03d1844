#!/usr/bin/env python3
"""Per-call latency of the drop-in (ldb_snappy_encode / ldb_snappy_decode on
one 4 KiB fillseq block, as lcdb's table builder and block reader call them:
table_builder.c:182-188, format.c:237-251), and the wall time of lcdb's own
t-db suite linked against the drop-in and against lcdb's snappy.c.

Prints one JSON line: p50/p90/p99 microseconds per call (ctypes call
overhead included, ~1 us), single thread and 4 threads."""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def percentiles(ts):
    a = np.array(ts) * 1e6
    return {"p50": float(np.percentile(a, 50)), "p90": float(np.percentile(a, 90)),
            "p99": float(np.percentile(a, 99)), "mean": float(a.mean()), "calls": len(ts)}


def main():
    from lcdb_amd import _native, corpus
    L = _native.lib()
    c = corpus.fillseq(256)
    blocks = c.blocks()
    srcs = [C.create_string_buffer(b + b"\0" * 16, len(b) + 16) for b in blocks]
    dst = C.create_string_buffer(8192)
    encs = []
    for b, s in zip(blocks, srcs):
        n = L.ldb_snappy_encode(dst, s, len(b))
        encs.append(C.create_string_buffer(dst.raw[:n] + b"\0" * 16, n + 16))
    enc_len = [len(e.raw) - 16 for e in encs]
    out = C.create_string_buffer(8192)
    reps = int(os.environ.get("REPS", "2000"))
    for _ in range(50):                                   # warm-up
        L.ldb_snappy_encode(dst, srcs[0], len(blocks[0]))
        L.ldb_snappy_decode(out, encs[0], enc_len[0])
    te, td = [], []
    for k in range(reps):
        i = k % len(blocks)
        t0 = time.perf_counter()
        L.ldb_snappy_encode(dst, srcs[i], len(blocks[i]))
        t1 = time.perf_counter()
        ok = L.ldb_snappy_decode(out, encs[i], enc_len[i])
        t2 = time.perf_counter()
        assert ok == 1
        te.append(t1 - t0)
        td.append(t2 - t1)
    res = {"encode_4KiB_us": percentiles(te), "decode_4KiB_us": percentiles(td)}

    # 4 threads calling at once (lcdb: user reads + compaction writes).
    lat = [[] for _ in range(4)]

    def work(t):
        d = C.create_string_buffer(8192)
        o = C.create_string_buffer(8192)
        for k in range(reps // 4):
            i = (k * 4 + t) % len(blocks)
            t0 = time.perf_counter()
            L.ldb_snappy_encode(d, srcs[i], len(blocks[i]))
            L.ldb_snappy_decode(o, encs[i], enc_len[i])
            lat[t].append(time.perf_counter() - t0)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    res["roundtrip_4threads_us"] = percentiles([x for v in lat for x in v])
    res["roundtrip_4threads_calls_per_s"] = sum(len(v) for v in lat) / wall

    # lcdb's t-db, unchanged, linked both ways (oracle/lcdb.mk).
    bindir = os.path.join(ROOT, "oracle", "_ref", "lcdb")
    for kind in (() if os.environ.get("NO_TDB") else ("cpu", "gpu")):
        exe = os.path.join(bindir, f"t-db.{kind}")
        if not os.path.exists(exe):
            continue
        with tempfile.TemporaryDirectory() as tmp:
            t0 = time.perf_counter()
            r = subprocess.run([exe], cwd=tmp, env=dict(os.environ, TEST_TMPDIR=tmp),
                               capture_output=True, timeout=900)
            res[f"t-db.{kind}_s"] = round(time.perf_counter() - t0, 2)
            res[f"t-db.{kind}_rc"] = r.returncode
    res["dropin"] = _native.dropin_footprint()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
