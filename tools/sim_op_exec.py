#!/usr/bin/env python3
"""Op-list statistics for the two-pass decoder:
pass 1 walks each block's tags into op records, pass 2 executes a block's
ops 64 at a time in one wave -- all literals at once, then the copies.  A
copy can run in the batch's parallel round when its source cannot hold
bytes written by an earlier copy of the same batch; this counts how many
copies that leaves for the in-order round under two tests:

  conservative: source starts at or after the end of the batch's previous
                copy, or ends at or before the batch's first copy;
  exact:        source meets no earlier copy's output in the batch
                (levels = rounds if each round runs every ready copy).

usage: python tools/sim_op_exec.py [BLOCKS]
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import oracle  # noqa: E402
from lcdb_amd import corpus  # noqa: E402
from sim_quad_trips import ops_of  # noqa: E402


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    ref = oracle.best()
    streams = [ref.encode(b) for b in corpus.fillseq(n).blocks()]
    nops = ncopy = dep_c = dep_x = overlap = 0
    max_ops = 0
    levels = 0
    batches = 0
    for s in streams:
        ops = ops_of(s)
        max_ops = max(max_ops, len(ops))
        nops += len(ops)
        for b0 in range(0, len(ops), 64):
            batch = ops[b0:b0 + 64]
            batches += 1
            copies = [o for o in batch if o[0] == "C"]
            if not copies:
                continue
            first = copies[0][1]
            prev_end = 0
            done = []            # (dst, end, level) of earlier copies in the batch
            maxlvl = 0
            for o in batch:
                if o[0] != "C":
                    continue
                ncopy += 1
                d, ln, dist = o[1], o[2], o[3]
                s0, s1 = d - dist, d - dist + ln
                if dist < ln:
                    overlap += 1
                indep = dist >= ln and (s0 >= prev_end or s1 <= first)
                dep_c += not indep
                hit = [lv for (a, e, lv) in done if a < s1 and e > s0]
                dep_x += bool(hit) or dist < ln
                lvl = 1 + max(hit) if hit else 0
                maxlvl = max(maxlvl, lvl)
                done.append((d, d + ln, lvl))
                prev_end = d + ln
            levels += maxlvl + 1
    print(f"{n} fillseq blocks: {nops / n:.1f} ops/block (max {max_ops}), "
          f"{ncopy / n:.1f} copies/block, {overlap / n:.2f} overlapping")
    print(f"in-order copies per block: conservative {dep_c / n:.1f}, exact {dep_x / n:.1f}")
    print(f"rounds per 64-op batch with exact levels: {levels / batches:.2f}")


if __name__ == "__main__":
    main()
