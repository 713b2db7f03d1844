#!/usr/bin/env python3
"""Speculative segment walks for finding a Snappy stream's tag starts in
parallel (the workgroup decoder), measured on real blocks.

The stream (after the length header) is cut into segments of SEG bytes, one
per lane.  Each lane walks tags from its segment's first byte as if a tag
started there, recording the positions it visits inside the segment, until
it leaves the segment.  A tag step is a function of the position only, so a
walk that visits the segment's true entry (the first real tag start at or
after the segment's first byte) is the real walk from there on.  Prints per
corpus and SEG: the segments holding real tag starts, the fraction whose
speculative walk misses the true entry (those must be walked again), and
the mean / max steps per lane.

usage: python tools/sim_spec_segments.py [BLOCKS]
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def step(z: bytes, p: int) -> int:
    """The position after the tag at p (speculative: any byte may start one)."""
    t = z[p]
    k, m = t & 3, t >> 2
    if k == 0:
        if m >= 60:
            e = m - 59
            return p + 1 + e + int.from_bytes(z[p + 1:p + 1 + e].ljust(e, b"\0"), "little") + 1
        return p + 1 + m + 1
    return p + (2, 3, 5)[k - 1]


def main() -> None:
    import numpy as np

    import oracle
    from lcdb_amd import corpus
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    cod = oracle.best()
    sets = {"fillseq4K": corpus.fillseq(nb), "fillseq64K": corpus.fillseq(max(2, nb // 8), 65536),
            "random4K": corpus.random_blocks(nb, 4096)}
    for name, c in sets.items():
        for seg in (8, 16, 32, 64):
            on = miss = 0
            steps = []
            for i in range(c.n):
                z = cod.encode(c.block(i))
                p = 0
                while z[p] & 0x80:
                    p += 1
                h = p + 1
                S = len(z)
                chain = set()
                q = h
                while q < S:
                    chain.add(q)
                    q = step(z, q)
                for s0 in range(h, S, seg):
                    s1 = min(s0 + seg, S)
                    entry = next((x for x in range(s0, s1) if x in chain), None)
                    q, vis, n = s0, set(), 0
                    while q < s1:
                        vis.add(q)
                        q = step(z, q)
                        n += 1
                    steps.append(n)
                    if entry is None or s0 == h:
                        continue
                    on += 1
                    miss += entry not in vis
            print(f"{name:11s} SEG={seg:3d}  on-chain segments {on:6d}  missed {miss / max(on, 1):6.1%}"
                  f"  steps/lane mean {np.mean(steps):5.2f} max {max(steps)}", flush=True)


if __name__ == "__main__":
    main()
