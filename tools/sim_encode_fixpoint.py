#!/usr/bin/env python3
"""How far is lcdb's greedy parse from a data-parallel formulation?

snappy.c:133-187 reads, at every probe p, the last position q < p written
into the hash table with hash(q) == hash(p) (or 0, the table's initial
value).  Written positions = every literal-search probe, plus at-1 and at
after each copy.  Given the written set S, every probe's candidate is a
data-parallel function of S (a segmented "last equal key before p"), and
the parse itself then only needs, per search batch, the first probe whose
candidate matches -- one dependent step instead of the encoder's four LDS
round trips.  But S is the parse's own output.  This iterates

    S_{k+1} = written set of the parse run with candidates from S_k

from a guess S_0 and counts the iterations until S_{k+1} == S_k (the serial
parse's S is the unique fixed point: the parse up to position p depends only
on S below p, so each iteration extends the agreeing prefix).  It also checks
that the fixed point reproduces the reference's bytes.

usage: python tools/sim_encode_fixpoint.py [BLOCKS]   
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from lcdb_amd import corpus  # noqa: E402


def le32(b, i):
    return int.from_bytes(b[i:i + 4], "little")


def parse(x: bytes, cand, shift: int):
    """snappy.c:104-187 with ref = cand(p, hash); returns (ops, written)."""
    n = len(x)
    last = n - 15
    h = lambda v: ((v * 0x1E35A7BD) & 0xFFFFFFFF) >> shift
    written, ops = [], []
    at, lit = 1, 0
    while True:
        skip, ahead = 32, at
        found = False
        while True:
            at = ahead
            ahead = at + (skip >> 5)
            skip += skip >> 5
            if ahead > last:
                break
            ref = cand(at, h(le32(x, at)))
            written.append(at)
            if le32(x, at) == le32(x, ref):
                found = True
                break
        if not found:
            break
        while True:
            start, r = at, ref + 4
            at += 4
            while at < n and x[r] == x[at]:
                r += 1
                at += 1
            ops.append((lit, start, at, start - ref))
            lit = at
            if at >= last:
                return ops, written
            written.append(at - 1)
            w = int.from_bytes(x[at - 1:at + 7], "little")
            ref = cand(at, h(w >> 8 & 0xFFFFFFFF))
            written.append(at)
            if (w >> 8) != le32(x, ref):
                at += 1
                break
    return ops, written


def cand_from(S, x, shift):
    """Candidate function of a written set: last q < p in S with equal hash."""
    h = lambda q: ((le32(x, q) * 0x1E35A7BD) & 0xFFFFFFFF) >> shift
    by = {}
    for q in sorted(S):
        by.setdefault(h(q), []).append(q)
    import bisect

    def cand(p, hp):
        lst = by.get(hp)
        if not lst:
            return 0
        i = bisect.bisect_left(lst, p)
        return lst[i - 1] if i else 0
    return cand


def emit(x: bytes, ops) -> bytes:
    """snappy.c:53-102 for the op list (literal then copy), plus the tail."""
    out = bytearray()

    def literal(a, b):
        m = b - a - 1
        if m < 60:
            out.append(m << 2)
        elif m < 256:
            out.extend([60 << 2, m])
        else:
            out.extend([61 << 2, m & 0xFF, m >> 8])
        out.extend(x[a:b])

    def copy(dist, ln):
        while ln >= 68:
            out.extend([(63 << 2) | 2, dist & 0xFF, dist >> 8])
            ln -= 64
        if ln > 64:
            out.extend([(59 << 2) | 2, dist & 0xFF, dist >> 8])
            ln -= 60
        if ln < 12 and dist < 2048:
            out.extend([((dist >> 8) << 5) | ((ln - 4) << 2) | 1, dist & 0xFF])
        else:
            out.extend([((ln - 1) << 2) | 2, dist & 0xFF, dist >> 8])
    lit = 0
    for (l0, start, end, dist) in ops:
        if start > l0:
            literal(l0, start)
        copy(dist, end - start)
        lit = end
    if lit < len(x):
        literal(lit, len(x))
    return bytes(out)


def iterate(x: bytes, S0):
    n = len(x)
    tsize, shift = 256, 24
    while tsize < 2048 and tsize < n:
        tsize, shift = tsize * 2, shift - 1
    S = set(S0)
    for k in range(1, 200):
        ops, written = parse(x, cand_from(S, x, shift), shift)
        W = set(written)
        if W == S:
            return k, ops
        S = W
    return None, ops


def main() -> None:
    nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    ref = oracle.best()
    blocks = corpus.fillseq(nblk).blocks()
    hist = {}
    for guess in ("all", "empty"):
        its = []
        for b in blocks:
            x = bytes(b)
            S0 = range(1, len(x) - 15) if guess == "all" else []
            k, ops = iterate(x, S0)
            its.append(k if k is not None else 999)
        its.sort()
        hist[guess] = its
        print(f"S0={guess}: iterations to the fixed point over {nblk} blocks: "
              f"median {its[len(its) // 2]}, p90 {its[int(len(its) * 0.9)]}, max {its[-1]}")
    # the fixed point is the serial parse: its bytes are the reference's
    same = 0
    for b in blocks:
        x = bytes(b)
        _, ops = iterate(x, range(1, len(x) - 15))
        v = len(x)
        hdr = bytearray()
        while v >= 0x80:
            hdr.append((v & 0x7F) | 0x80)
            v >>= 7
        hdr.append(v)
        same += bytes(hdr) + emit(x, ops) == ref.encode(x)
    print(f"fixed point == reference bytes on {same} of {nblk} blocks")


if __name__ == "__main__":
    main()
