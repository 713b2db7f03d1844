"""Device-resident throughput of the block-framing rows on
C2 (65 536 x 4 KiB db_bench fillseq blocks), one JSON line:

* write: lgs_table_write_dev = encode + 12.5 % rule + trailers + packing
  (table_builder.c:155-213 for every block), GiB/s of raw block bytes;
* read:  lgs_table_read_dev = truncation + checksum + type + decode
  (format.c:162-270 for every handle, verify_checksums on), GiB/s of
  decoded bytes;
* crc:   lgs_crc32c_batch_dev over the framed contents + type bytes (the
  trailer CRCs alone), GB/s of bytes read.

Times are HIP events on the launch stream, median of --iters runs; parity
of the round trip is re-checked.  usage: python tools/bench_table.py
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
    p.add_argument("--blocks", type=int, default=65536)
    p.add_argument("--block-size", type=int, default=4096)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--lib", default=None, help="a probe build of the codec library")
    a = p.parse_args()
    if a.lib:
        import lcdb_amd.build as b
        b.LIB = os.path.abspath(a.lib)

    import numpy as np
    import torch

    from lcdb_amd import batch, corpus, table

    torch.cuda.set_device(0)
    c = corpus.fillseq(a.blocks, block_size=a.block_size)
    raw = batch.upload(c)
    n = c.n
    raw_bytes = int(c.len.astype(np.int64).sum())
    max_len = int(c.len.max())

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

    out = {}
    res = {}

    def write():
        res["w"] = table.write_blocks(raw.buf, raw.off, raw.len, 1, 0, max_len, raw_bytes)

    t_w = timed(write)
    d_file, hoff, hsize, end = res["w"]
    file_len = int(end.cpu()[0])
    comp_bytes = int(hsize.sum().cpu())
    dec = batch.decode_slots(c.len)
    olen = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")

    def read():
        table.read_blocks(d_file, file_len, hoff, hsize, dec.buf, dec.off, dec.cap, dec.max_cap,
                          True, olen, st)

    t_r = timed(read)

    def read0():   # lcdb's default ReadOptions: no checksum verification
        table.read_blocks(d_file, file_len, hoff, hsize, dec.buf, dec.off, dec.cap, dec.max_cap,
                          False, olen, st)

    t_r0 = timed(read0)
    ok0 = bool((st == 1).all()) and torch.equal(olen, raw.len)
    read()
    torch.cuda.synchronize()
    ok = ok0 and bool((st == 1).all()) and torch.equal(olen, raw.len)
    ho = batch.to_host(dec)
    ho.len = olen.cpu().numpy().astype(np.uint32)
    ok = ok and all(ho.block(i) == c.block(i) for i in range(0, n, 251))

    types = torch.ones(n, dtype=torch.uint8, device="cuda")
    hsize32 = hsize.to(torch.int32)
    crc = torch.empty(n, dtype=torch.int32, device="cuda")

    def crcs():
        table.crc32c_batch(d_file, hoff, hsize32, types, True, crc)

    t_c = timed(crcs)
    out.update({
        "workload": f"C2 framing: {n} x {a.block_size} B fillseq blocks, device-resident",
        "blocks": n, "raw_bytes": raw_bytes, "file_bytes": file_len, "comp_bytes": comp_bytes,
        "write_ms": t_w * 1e3, "write_GiBps_raw": raw_bytes / t_w / 2**30,
        "read_ms": t_r * 1e3, "read_GiBps_raw": raw_bytes / t_r / 2**30,
        "read_noverify_ms": t_r0 * 1e3,
        "crc_ms": t_c * 1e3, "crc_GBps_read": (comp_bytes + n) / t_c / 1e9,
        "parity": "write->read round trip exact, all checksums verified" if ok else "FAILED",
    })
    print(json.dumps(out))
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
