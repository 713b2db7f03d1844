#!/usr/bin/env python3
"""How parallel is one fillseq block's decode?  

Simulates SURVEY 7's "decoder parallelism (b)" on real C2 blocks (encoded by
the reference codec through oracle/): the block's tags are split into S
segments of equal stream bytes, one per lane, each lane decoding its own
segment's ops in order; in each lockstep iteration a lane executes its next
op if every byte that op reads is already written (exact per-byte
readiness), 16 bytes of a move per iteration.  Prints the iterations a
block needs: its serial chain through copies of copies.

usage: python tools/sim_intrablock_decode.py [blocks]
"""
from __future__ import annotations

import bisect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def parse(z: bytes):
    """(stream pos, kind, len, dist or literal pos, out pos) per tag."""
    p, want, sh = 0, 0, 0
    while True:
        b = z[p]
        p += 1
        want |= (b & 0x7F) << sh
        sh += 7
        if b < 128:
            break
    ops, o = [], 0
    while p < len(z):
        t = z[p]
        k, sp = t & 3, p
        if k == 0:
            m = t >> 2
            p += 1
            if m >= 60:
                e = m - 59
                m = int.from_bytes(z[p:p + e], "little")
                p += e
            ops.append((sp, 0, m + 1, p, o))
            p += m + 1
            o += m + 1
        else:
            if k == 1:
                ln, d, p = 4 + ((t >> 2) & 7), ((t & 0xE0) << 3) | z[p + 1], p + 2
            elif k == 2:
                ln, d, p = 1 + (t >> 2), z[p + 1] | (z[p + 2] << 8), p + 3
            else:
                ln, d, p = 1 + (t >> 2), int.from_bytes(z[p + 1:p + 5], "little"), p + 5
            ops.append((sp, k, ln, d, o))
            o += ln
    assert o == want
    return ops


def iterations(ops, slen: int, segs: int, chunk: int = 16) -> int:
    bounds = [slen * k // segs for k in range(segs)]
    seg = [[] for _ in range(segs)]
    k = 0
    for op in ops:
        while k + 1 < segs and op[0] >= bounds[k + 1]:
            k += 1
        seg[k].append(op)
    live = [j for j in range(segs) if seg[j]]
    starts = [seg[j][0][4] for j in live]
    idx = {j: 0 for j in live}
    cur = {j: seg[j][0][4] for j in live}
    rem = {j: 0 for j in live}

    def written(a: int, b: int, snap) -> bool:
        while a < b:
            t = bisect.bisect_right(starts, a) - 1
            j = live[t]
            if snap[j] <= a:
                return False
            nxt = starts[t + 1] if t + 1 < len(starts) else 1 << 30
            if snap[j] < min(b, nxt):
                return False
            a = nxt if b > nxt else b
        return True

    it = 0
    while any(idx[j] < len(seg[j]) for j in live):
        it += 1
        snap = dict(cur)
        for j in live:
            if idx[j] >= len(seg[j]):
                continue
            if rem[j] > 0:
                rem[j] -= 1
                if rem[j] == 0:
                    op = seg[j][idx[j]]
                    idx[j] += 1
                    cur[j] = op[4] + op[2]
                continue
            sp, kind, ln, d, o = seg[j][idx[j]]
            ready = kind == 0 or (o - d < o and written(o - d, o - d + min(ln, d), snap))
            if ready:
                ch = (ln + chunk - 1) // chunk
                if ch <= 1:
                    idx[j] += 1
                    cur[j] = o + ln
                else:
                    rem[j] = ch - 1
    return it


def main() -> None:
    import oracle
    from lcdb_amd import corpus
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    c = corpus.fillseq(n)
    ref = oracle.best()
    streams = [ref.encode(b) for b in c.blocks()]
    tags = [len(parse(z)) for z in streams]
    print(f"{n} fillseq blocks, {np.mean(tags):.1f} tags per block")
    for segs in (8, 16, 32, 64):
        its = [iterations(parse(z), len(z), segs) for z in streams]
        print(f"  {segs:2d} segments: {np.mean(its):6.1f} iterations per block "
              f"(p90 {np.percentile(its, 90):.0f}, max {max(its)})")


if __name__ == "__main__":
    main()
