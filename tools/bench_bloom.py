"""Device-resident throughput of the bloom filter row: one
filter per 4 KiB fillseq data block (36 "%016d" user keys, 10 bits per key,
the shape lcdb's filter block has with bloom_bits = 10), 65 536 filters.
Builds them (lgs_bloom_build_dev), then probes every key against its own
filter and against the next one (lgs_bloom_match_dev); then the filter block
of one table holding those blocks (lgs_filter_block_build_dev: layout, offset
scan, filters) and every key probed through it (lgs_filter_block_match_dev).  HIP-event timed,
median of --iters; one JSON line.  usage: python tools/bench_bloom.py
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
    p.add_argument("--filters", type=int, default=65536)
    p.add_argument("--keys-per-filter", type=int, default=36)
    p.add_argument("--bits-per-key", type=int, default=10)
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args()

    import numpy as np
    import torch

    from lcdb_amd import bloom

    torch.cuda.set_device(0)
    nf, per, bpk = a.filters, a.keys_per_filter, a.bits_per_key
    nk = nf * per
    keys = np.frombuffer(b"".join(b"%016d" % k for k in range(nk)) + b"\0" * 16, dtype=np.uint8)
    d_keys = torch.from_numpy(keys.copy()).cuda()
    d_koff = torch.arange(nk, dtype=torch.int64, device="cuda") * 16
    d_klen = torch.full((nk,), 16, dtype=torch.int32, device="cuda")
    d_first = torch.arange(nf + 1, dtype=torch.int32, device="cuda") * per
    size = bloom.filter_size(per, bpk)
    d_foff = torch.arange(nf, dtype=torch.int64, device="cuda") * size
    d_flen = torch.full((nf,), size, dtype=torch.int32, device="cuda")
    d_out = torch.zeros(nf * size + 16, dtype=torch.uint8, device="cuda")
    d_qf = torch.arange(nk, dtype=torch.int32, device="cuda") // per
    d_qn = (d_qf + 1) % nf
    d_m = torch.zeros(nk, dtype=torch.uint8, device="cuda")

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

    t_b = timed(lambda: bloom.build(d_keys, d_koff, d_klen, d_first, bpk, d_out, d_foff))
    t_m = timed(lambda: bloom.match(d_out, d_foff, d_flen, d_qf, d_keys, d_koff, d_klen, d_m))
    members_ok = bool((d_m == 1).all())
    t_n = timed(lambda: bloom.match(d_out, d_foff, d_flen, d_qn, d_keys, d_koff, d_klen, d_m))
    fp = float(d_m.float().mean())
    key_bytes = nk * 16

    # The filter block of one table holding these nf data blocks (one per
    # ~2.3 KB of file offsets, lcdb's fillseq block size once framed).
    sizes = np.random.default_rng(3).integers(2200, 2500, size=nf).astype(np.int64)
    boff = np.zeros(nf, dtype=np.int64)
    boff[1:] = np.cumsum(sizes[:-1])
    end = int(boff[-1] + sizes[-1])
    d_boff = torch.from_numpy(boff).cuda()
    d_fb = torch.zeros(bloom.filter_block_bound(nk, nf, end, bpk), dtype=torch.uint8,
                       device="cuda")
    d_fsize = torch.zeros(1, dtype=torch.int64, device="cuda")
    d_scr = torch.empty(bloom.filter_block_scratch(end), dtype=torch.uint8, device="cuda")
    t_fb = timed(lambda: bloom.filter_block_build(d_keys, d_koff, d_klen, d_first, d_boff, end,
                                                  bpk, d_fb, d_fsize, d_scr))
    fbn = int(d_fsize.item())
    d_qoff = torch.repeat_interleave(d_boff, per)
    t_fm = timed(lambda: bloom.filter_block_match(d_fb, fbn, d_qoff, d_keys, d_koff, d_klen, d_m))
    members_ok = members_ok and bool((d_m == 1).all())
    print(json.dumps({
        "workload": f"{nf} filters x {per} 16-B keys, {bpk} bits/key ({size} B per filter)",
        "build_ms": t_b * 1e3, "build_Mkeys_per_s": nk / t_b / 1e6,
        "build_GBps": (key_bytes + nf * size) / t_b / 1e9,
        "match_member_ms": t_m * 1e3, "match_Mqueries_per_s": nk / t_m / 1e6,
        "match_nonmember_ms": t_n * 1e3, "false_positive_rate": fp,
        "filter_block_build_ms": t_fb * 1e3, "filter_block_bytes": fbn,
        "filter_block_match_ms": t_fm * 1e3,
        "parity": "every member matches" if members_ok else "FAILED",
    }))
    if not members_ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
