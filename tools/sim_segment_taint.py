#!/usr/bin/env python3
"""Segment-parallel decode of one big block, simulated.

Split a block's output into S segments decoded by S waves at once.  A copy
whose source lies before its segment's start cannot be served until the
earlier segments are done: it is deferred, and so is every later copy of the
segment whose source overlaps a deferred byte (taint).  Deferred ops run
after the segments, in order.  Prints the tainted fraction of ops and bytes
per segment, and the dependency depth of the deferred ops (the rounds a
fix-up pass needs even with unlimited parallelism per round).

usage: python tools/sim_segment_taint.py [BLOCK_SIZE] [S]
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ops_of(z: bytes):
    """(kind, len, dist) of every tag of a snappy stream (snappy.c:201-341)."""
    p, want, s = 0, 0, 0
    while True:
        b = z[p]
        p += 1
        want |= (b & 0x7F) << s
        s += 7
        if b < 0x80:
            break
    ops = []
    while p < len(z):
        t = z[p]
        k = t & 3
        if k == 0:
            m = t >> 2
            hl = 1
            if m >= 60:
                e = m - 59
                m = int.from_bytes(z[p + 1:p + 1 + e], "little")
                hl += e
            ops.append((0, m + 1, 0))
            p += hl + m + 1
        else:
            if k == 1:
                ln, d, hl = 4 + ((t >> 2) & 7), ((t & 0xE0) << 3) | z[p + 1], 2
            elif k == 2:
                ln, d, hl = 1 + (t >> 2), int.from_bytes(z[p + 1:p + 3], "little"), 3
            else:
                ln, d, hl = 1 + (t >> 2), int.from_bytes(z[p + 1:p + 5], "little"), 5
            ops.append((k, ln, d))
            p += hl
    return want, ops


def main() -> None:
    import numpy as np

    import oracle
    from lcdb_amd import corpus
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    c = corpus.fillseq(4, bs)
    z = oracle.best().encode(bytes(c.buf[c.off[1]:c.off[1] + c.len[1]]))
    want, ops = ops_of(z)
    seg = (want + S - 1) // S
    level = np.zeros(want, dtype=np.int32)   # fix-up round of each output byte (0 = served)
    made = 0
    tainted_ops = [0] * S
    tainted_bytes = [0] * S
    ops_per = [0] * S
    for kind, ln, d in ops:
        s = min(made // seg, S - 1)
        ops_per[s] += 1
        lo = s * seg
        if kind == 0:
            lv = 0
        else:
            src = made - d
            if src < lo:                       # reaches into an earlier segment
                lv = 1 + int(level[src:src + ln].max()) if src + ln > lo else 1
                lv = max(lv, 1)
            else:
                mx = int(level[src:src + min(ln, d)].max())
                lv = mx + 1 if mx > 0 else 0
        if lv:
            tainted_ops[s] += 1
            tainted_bytes[s] += ln
        level[made:made + ln] = lv
        made += ln
    print(f"block {bs} B, {len(ops)} ops, S={S} segments of {seg} B")
    for s in range(S):
        print(f"  segment {s}: {ops_per[s]} ops, deferred {tainted_ops[s]} "
              f"({100 * tainted_ops[s] / max(ops_per[s], 1):.0f} %), "
              f"{tainted_bytes[s]} B")
    print(f"  fix-up depth (rounds with unlimited parallelism): {int(level.max())}")


if __name__ == "__main__":
    main()
