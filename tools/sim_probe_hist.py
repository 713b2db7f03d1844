#!/usr/bin/env python3
"""Probes per search of lcdb's greedy parse on C2-shaped blocks (the encoder's
batch width).  Restates encode_block's search (snappy.c:133-153)
and its post-copy re-probe (:172-186) in pure Python and counts, per search,
the probes it takes until a match (or the end of the block), and how often
the re-probe after a copy matches (lane B of a batch: no search at all).

The GPU encoder fires 62 search probes per batch (lanes 2-63) plus the two
re-probe lanes; a search that matches at probe k leaves 62 - k lanes that
swapped the table and must put back what they received.  This counts what
a narrower first batch would leave undone.

usage: python tools/sim_probe_hist.py [BLOCKS]
"""
from __future__ import annotations

import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lcdb_amd import corpus  # noqa: E402

K_HASH = 0x1e35a7bd


def ld32(b: bytes, i: int) -> int:
    return int.from_bytes(b[i:i + 4], "little")


def ld64(b: bytes, i: int) -> int:
    return int.from_bytes(b[i:i + 8], "little")


def parse(x: bytes, hist: collections.Counter, post: collections.Counter) -> None:
    n = len(x)
    if n < 17:                                     # snappy.c:379: a literal
        return
    limit = n - 15
    size, shift = 256, 32 - 8
    while size < 2048 and size < n:                # snappy.c:122-125 (lcdb: 2048 cap)
        size *= 2
        shift -= 1
    h = lambda v: ((v * K_HASH) & 0xffffffff) >> shift   # noqa: E731
    table = [0] * size
    pos = 1                                        # snappy.c:111
    nxt = h(ld32(x, pos))
    while True:
        skip, npos, k = 32, pos, 0
        while True:
            pos = npos
            npos = pos + (skip >> 5)
            skip += skip >> 5
            if npos > limit:
                hist["end"] += 1
                hist[("end_at", min(k, 200))] += 1
                return
            cand = table[nxt]
            table[nxt] = pos
            nxt = h(ld32(x, npos))
            k += 1
            if ld32(x, pos) == ld32(x, cand):
                break
        hist[min(k, 200)] += 1
        while True:
            base = pos
            pos += 4
            chk = cand + 4
            while pos < n and x[chk] == x[pos]:
                chk += 1
                pos += 1
            if pos >= limit:
                return
            v = ld64(x, pos - 1)
            table[h(v & 0xffffffff)] = pos - 1
            cur = h((v >> 8) & 0xffffffff)
            cand = table[cur]
            table[cur] = pos
            if (v >> 8) != ld32(x, cand):          # snappy.c:182, lcdb's 64-bit compare
                post["miss"] += 1
                nxt = h((v >> 16) & 0xffffffff)
                pos += 1
                break
            post["hit"] += 1


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    c = corpus.fillseq(n)
    hist: collections.Counter = collections.Counter()
    post: collections.Counter = collections.Counter()
    for b in c.blocks():
        parse(b, hist, post)
    searches = sum(v for k, v in hist.items() if isinstance(k, int))
    cum, out = 0, {}
    for k in range(1, 63):
        cum += hist.get(k, 0)
        if k in (1, 2, 3, 4, 6, 8, 10, 12, 14, 16, 20, 24, 30, 40, 50, 62):
            out[k] = round(cum / searches, 4)
    print(json.dumps({"blocks": n, "searches": searches, "searches_per_block": searches / n,
                      "ends_per_block": hist["end"] / n,
                      "rematch_hits_per_block": post["hit"] / n,
                      "rematch_misses_per_block": post["miss"] / n,
                      "frac_matched_within_k_probes": out,
                      "mean_probes_matched": sum(k * v for k, v in hist.items()
                                                 if isinstance(k, int)) / searches}))


if __name__ == "__main__":
    main()
