#!/usr/bin/env python3
"""How far back lcdb's encoder finds its candidates: the window question
behind the 64 KiB-class encoder's LDS ring.

Replays the greedy parse of src/util/snappy.c:104-195 (table of
min(2048, pow2 >= n) u16 entries, skip heuristic, post-copy re-probe) on
db_bench fillseq blocks and counts, for a window of W bytes behind the
probe, the probes whose candidate lies outside it and the search rounds
that contain such a probe.  (A sizing tool: the parse is a plain Python
restatement, not the oracle, and it is not used by any test.)

usage: python tools/sim_candidate_age.py [--block-size 65536] [--blocks 3] [--windows 28000,16000]
Prints one line per block and window: probes, far probes, rounds with a far probe.
"""
from __future__ import annotations

import argparse
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _h(x: int, shift: int) -> int:
    return ((x * 0x1E35A7BD) & 0xFFFFFFFF) >> shift


def _ld32(b: bytes, i: int) -> int:
    return struct.unpack_from("<I", b, i)[0]


def simulate(x: bytes, window: int) -> tuple[int, int, int]:
    n = len(x)
    limit = n - 15
    size, shift = 256, 24
    while size < 2048 and size < n:
        size *= 2
        shift -= 1
    tab = [0] * size
    pos = 1
    nxt = _h(_ld32(x, pos), shift)
    probes = far = far_rounds = 0
    while True:
        skip, npos, seen = 32, pos, False
        while True:                                   # snappy.c:135-154
            pos = npos
            npos = pos + (skip >> 5)
            skip += skip >> 5
            if npos > limit:
                return probes, far, far_rounds
            cand = tab[nxt]
            tab[nxt] = pos
            nxt = _h(_ld32(x, npos), shift)
            probes += 1
            if pos - cand > window:
                far += 1
                seen = True
            if _ld32(x, pos) == _ld32(x, cand):
                break
        far_rounds += seen
        while True:                                   # snappy.c:158-186
            pos += 4
            chk = cand + 4
            while pos < n and x[chk] == x[pos]:
                chk += 1
                pos += 1
            if pos >= limit:
                return probes, far, far_rounds
            xx = int.from_bytes(x[pos - 1:pos + 7].ljust(8, b"\0"), "little")
            tab[_h(xx & 0xFFFFFFFF, shift)] = pos - 1
            cur = _h((xx >> 8) & 0xFFFFFFFF, shift)
            cand = tab[cur]
            tab[cur] = pos
            if (xx >> 8) != _ld32(x, cand):           # lcdb's 64-bit compare (:182)
                nxt = _h((xx >> 16) & 0xFFFFFFFF, shift)
                pos += 1
                break


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--block-size", type=int, default=65536)
    p.add_argument("--blocks", type=int, default=3)
    p.add_argument("--windows", default="28000,24000,16000")
    a = p.parse_args()
    from lcdb_amd import corpus
    c = corpus.fillseq(a.blocks, block_size=a.block_size, key0=a.block_size)
    for k in range(c.n):
        b = c.block(k)[:65536]
        for w in (int(v) for v in a.windows.split(",")):
            print(f"block {k} ({len(b)} B) window {w}: probes, far probes, rounds with one "
                  f"= {simulate(b, w)}", flush=True)


if __name__ == "__main__":
    main()
