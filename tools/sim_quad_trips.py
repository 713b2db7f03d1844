#!/usr/bin/env python3
"""Trips per block of a G-lanes-per-block decoder (the quad decoder, G = 4),
simulated on fillseq blocks encoded by the reference: a trip takes the
block's next ops up to G tags, a budget of output bytes, the input landed so
far (refills of 64 B, ring of `ring_in` B) and at most one far copy (beyond
the 240-byte near window) as its last op; rounds = how many write rounds the
trip's ops need (a copy reading this trip's output waits a round unless it
copies the previous op's literal, which is read from the input ring).

usage: python tools/sim_quad_trips.py [BLOCKS]   
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from lcdb_amd import corpus  # noqa: E402


def ops_of(s: bytes):
    """(kind, out_pos, len, dist | literal_data_pos, tag_pos) per tag."""
    i = 0
    while s[i] & 0x80:
        i += 1
    i += 1
    made, out = 0, []
    while i < len(s):
        t, k, p0 = s[i], s[i] & 3, i
        if k == 0:
            m = t >> 2
            if m < 60:
                ln, i = m + 1, i + 1
            else:
                e = m - 59
                ln, i = int.from_bytes(s[i + 1:i + 1 + e], "little") + 1, i + 1 + e
            out.append(("L", made, ln, i, p0))
            i += ln
        else:
            if k == 1:
                ln, d, i = 4 + ((t >> 2) & 7), ((t & 0xE0) << 3) | s[i + 1], i + 2
            elif k == 2:
                ln, d, i = (t >> 2) + 1, s[i + 1] | (s[i + 2] << 8), i + 3
            else:
                ln, d, i = (t >> 2) + 1, int.from_bytes(s[i + 1:i + 5], "little"), i + 5
            out.append(("C", made, ln, d, p0))
        made += ln
    return out


def sim(streams, G=4, budget=128, near=240, ring_in=128, refills=2):
    trips = rounds = nblk = 0
    for s in streams:
        ops = ops_of(s)
        nblk += 1
        k, landed, inflight = 0, min(len(s), ring_in), 0
        while k < len(ops):
            trips += 1
            landed, inflight = min(len(s), landed + inflight), 0
            made0, taken, mx, prev_lit = ops[k][1], 0, 1, None
            rnd = []
            while taken < G and k < len(ops):
                o = ops[k]
                need = (o[3] + min(o[2], 64)) if o[0] == "L" else o[4] + 3
                if need > landed or (taken and o[1] + min(o[2], 64) - made0 > budget):
                    break
                r = 1
                if o[0] == "C":
                    d, src = o[3], o[1] - o[3]
                    if d > near + (o[1] - made0):          # far: the trip's last op
                        taken, k = taken + 1, k + 1
                        break
                    if src + o[2] > made0:                 # reads this trip's output
                        remap = prev_lit and prev_lit[1] <= src and src + o[2] <= prev_lit[1] + prev_lit[2]
                        if not remap:
                            r = 1 + max([x for x in rnd] or [0])
                rnd.append(r)
                mx = max(mx, r)
                prev_lit = o if o[0] == "L" else None
                taken, k = taken + 1, k + 1
                if o[2] > 64:
                    break
            rounds += mx
            cons = ops[k][4] if k < len(ops) else len(s)
            inflight = min(refills * 64, max(0, cons + ring_in - landed) // 64 * 64)
    return trips / nblk, rounds / trips


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    ref = oracle.best()
    streams = [ref.encode(b) for b in corpus.fillseq(n).blocks()]
    print("ring-like (1 lane, 2 ops a trip): ~%.0f trips/block" % (179.1 / 2 * 1.23))
    for G in (2, 4, 8):
        t, r = sim(streams, G=G)
        print(f"G={G}: {t:.1f} trips/block, {r:.2f} write rounds/trip")


if __name__ == "__main__":
    main()
