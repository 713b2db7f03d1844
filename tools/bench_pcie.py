#!/usr/bin/env python3
"""PCIe-inclusive rate of the codec on BASELINE config 2 (recorded in DESIGN.md,
never bench.py's `value`).

Host side: the corpus in pinned host memory (as the .ldb reader/builder would
stage it).  One encode pass = H2D raw blocks + encode + D2H encoded slots;
one decode pass = H2D encoded slots + decode + D2H raw blocks; hipMemcpyAsync
on the codec's stream, timed with events, median over --steps.  Encoded slots
are bound-spaced (the D2H moves slot capacity, an upper bound on a compacted
transfer); the packed-compressed-bytes figure is reported beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lcdb_amd import batch, corpus, table  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--blocks", type=int, default=65536)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--chunks", type=int, default=8,
                   help="pipelined passes: blocks split into this many chunks over 3 streams")
    a = p.parse_args()
    c = corpus.fillseq(a.blocks)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    h_raw = torch.from_numpy(c.buf).pin_memory()
    h_comp = torch.empty(comp.buf.numel(), dtype=torch.uint8).pin_memory()
    h_out = torch.empty(out.buf.numel(), dtype=torch.uint8).pin_memory()
    s = torch.cuda.current_stream()
    batch.encode(raw, comp)
    torch.cuda.synchronize()
    comp_bytes = int(comp.len.sum().item())

    def timed(fn):
        ts = []
        for _ in range(a.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        return float(np.median(ts))

    def enc_pass():
        raw.buf.copy_(h_raw, non_blocking=True)
        batch.encode(raw, comp)
        h_comp.copy_(comp.buf, non_blocking=True)

    def dec_pass():
        comp.buf.copy_(h_comp, non_blocking=True)
        batch.decode(comp, out, st)
        h_out.copy_(out.buf, non_blocking=True)

    def h2d_raw():
        raw.buf.copy_(h_raw, non_blocking=True)

    te, td, th = timed(enc_pass), timed(dec_pass), timed(h2d_raw)
    assert bool((st == 1).all())

    # Pipelined passes: the blocks in chunks, each chunk's H2D, kernel and D2H
    # on one of three streams in turn, so one chunk's upload, another's
    # kernel and a third's download overlap (the copy engines run both
    # directions at once).  Same bytes moved as the serial passes.
    streams = [torch.cuda.Stream() for _ in range(3)]
    bounds = np.linspace(0, c.n, a.chunks + 1).astype(np.int64)
    r_off, r_len = c.off.astype(np.int64), c.len.astype(np.int64)
    k_off = comp.off.cpu().numpy().astype(np.int64)
    k_cap = comp.cap.cpu().numpy().astype(np.int64)
    o_off = out.off.cpu().numpy().astype(np.int64)
    o_cap = out.cap.cpu().numpy().astype(np.int64)
    chunks = []
    for j in range(a.chunks):
        b0, b1 = int(bounds[j]), int(bounds[j + 1])
        if b1 <= b0:
            continue
        sl = slice(b0, b1)
        view = lambda x: batch.Slots(x.buf, x.off[sl], x.len[sl], x.cap[sl], x.max_cap)  # noqa: E731
        chunks.append((view(raw), view(comp), view(out), st[sl],
                       (int(r_off[b0]), int(r_off[b1 - 1] + r_len[b1 - 1])),
                       (int(k_off[b0]), int(k_off[b1 - 1] + k_cap[b1 - 1])),
                       (int(o_off[b0]), int(o_off[b1 - 1] + o_cap[b1 - 1]))))

    def piped(one):
        e = torch.cuda.Event()
        e.record(s)
        for k, ch in enumerate(chunks):
            t = streams[k % len(streams)]
            t.wait_event(e)
            with torch.cuda.stream(t):
                one(ch, t)
        for t in streams:
            s.wait_stream(t)

    def enc_one(ch, t):
        rv, kv, _, _, (r0, r1), (k0, k1), _ = ch
        raw.buf[r0:r1].copy_(h_raw[r0:r1], non_blocking=True)
        batch.encode(rv, kv, stream=t)
        h_comp[k0:k1].copy_(comp.buf[k0:k1], non_blocking=True)

    def dec_one(ch, t):
        _, kv, ov, sv, _, (k0, k1), (o0, o1) = ch
        comp.buf[k0:k1].copy_(h_comp[k0:k1], non_blocking=True)
        batch.decode(kv, ov, sv, stream=t)
        h_out[o0:o1].copy_(out.buf[o0:o1], non_blocking=True)

    st.zero_()
    tpe = timed(lambda: piped(enc_one))
    tpd = timed(lambda: piped(dec_one))
    torch.cuda.synchronize()
    assert bool((st == 1).all())
    # The pipelined passes' bytes: the host-side output equals the device's.
    assert torch.equal(h_out[:out.buf.numel() - 64], out.buf[:-64].cpu())

    # The table paths as lcdb would call them: the
    # data-block region of a table written from host blocks (H2D raw, encode,
    # 12.5 % rule, trailers, packing, D2H of exactly the region), and that
    # region read back (H2D region, checksums, decode, D2H blocks).
    max_len, raw_total = int(c.len.max()), int(c.len.sum())
    d_file, hoff, hsize, end = table.write_blocks(raw.buf, raw.off, raw.len, 1, 0, max_len,
                                                  raw_total)
    torch.cuda.synchronize()
    region = int(end.item())
    h_file = torch.empty(d_file.numel(), dtype=torch.uint8).pin_memory()

    def tw_pass():
        raw.buf.copy_(h_raw, non_blocking=True)
        f, _, _, e = table.write_blocks(raw.buf, raw.off, raw.len, 1, 0, max_len, raw_total)
        n = int(e.item())                     # the host needs the region's size
        h_file[:n].copy_(f[:n], non_blocking=True)

    olen = torch.zeros(c.n, dtype=torch.int32, device="cuda")

    def tr_pass():
        d_file[:region].copy_(h_file[:region], non_blocking=True)
        table.read_blocks(d_file, region, hoff, hsize, out.buf, out.off, out.cap, out.max_cap,
                          True, olen, st)
        h_out.copy_(out.buf, non_blocking=True)

    ttw = timed(tw_pass)
    ttr = timed(tr_pass)
    assert bool((st == 1).all()) and torch.equal(olen, raw.len)
    rb = c.raw_bytes
    print(json.dumps({
        "blocks": c.n, "raw_bytes": rb, "comp_bytes_packed": comp_bytes,
        "comp_slot_bytes": comp.buf.numel(), "h2d_raw_GBps": h_raw.numel() / th / 1e9,
        "encode_pcie_GiBps": rb / te / 2**30, "decode_pcie_GiBps": rb / td / 2**30,
        "roundtrip_pcie_GiBps": rb / (te + td) / 2**30,
        "encode_pass_ms": te * 1e3, "decode_pass_ms": td * 1e3,
        "pipelined_chunks": len(chunks), "pipelined_streams": len(streams),
        "encode_pcie_pipelined_GiBps": rb / tpe / 2**30,
        "decode_pcie_pipelined_GiBps": rb / tpd / 2**30,
        "roundtrip_pcie_pipelined_GiBps": rb / (tpe + tpd) / 2**30,
        "table_region_bytes": region,
        "table_write_pcie_GiBps": rb / ttw / 2**30, "table_read_pcie_GiBps": rb / ttr / 2**30,
        "table_write_pass_ms": ttw * 1e3, "table_read_pass_ms": ttr * 1e3}))


if __name__ == "__main__":
    main()
