#!/usr/bin/env python3
"""SURVEY §7(b)'s pointer-jumping decoder, costed on real C2 blocks
(VERDICT r2 #1 asked for it to be tested as written).

The scheme, per block:
  1. every compressed byte position parses the tag that would start there
     (speculative: its step to the next tag);
  2. tag starts = the positions reachable from the header by following the
     steps: pointer jumping (nxt <- nxt[nxt]) until every chain has jumped
     past the stream: ceil(log2(tags)) rounds over all positions;
  3. output offsets of the tags: a scan;
  4. each output byte's source: a literal byte (final) or output byte
     pos - dist (to be resolved); pointer jumping (src <- src[src]) until
     every byte points at a literal: rounds = ceil(log2(longest chain));
  5. one gather of every output byte from the stream.
Prints, averaged over sampled blocks, the rounds and the lane operations
(one lane op = one element handled in one round), and the wave
instructions per block and per C2 launch per SIMD that they imply at the
assumed instructions per element per round given below.

usage: python tools/sim_pointer_jump.py [BLOCKS]
"""
from __future__ import annotations

import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

# VALU instructions per element and round (a lean estimate: address, the
# LDS gather, a select, loop overhead amortised); parse 10 per position.
K_PARSE, K_JUMP, K_SCAN, K_SRC, K_GATHER = 10, 4, 3, 6, 3


def main() -> None:
    import numpy as np

    import oracle
    from lcdb_amd import corpus
    from sim_segment_taint import ops_of
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    c = corpus.fillseq(nb)
    cod = oracle.best()
    rows = []
    for i in range(nb):
        z = cod.encode(c.block(i))
        want, ops = ops_of(z)
        # chain depth: hops from an output byte to a literal byte
        depth = np.zeros(want, dtype=np.int32)
        made = 0
        for kind, ln, d in ops:
            if kind == 0:
                depth[made:made + ln] = 0
            else:
                for k in range(ln):
                    depth[made + k] = depth[made + k - d] + 1
            made += ln
        tags = len(ops)
        r_tag = math.ceil(math.log2(max(tags, 2)))
        r_src = math.ceil(math.log2(max(int(depth.max()) + 1, 2)))
        lane_ops = (len(z) * K_PARSE + r_tag * len(z) * K_JUMP
                    + math.ceil(math.log2(len(z))) * len(z) * K_SCAN
                    + want * K_SRC + r_src * want * K_JUMP + want * K_GATHER)
        rows.append((len(z), want, tags, int(depth.max()), r_tag, r_src, lane_ops))
    a = np.array(rows, dtype=np.float64).mean(axis=0)
    wave_instr = a[6] / 64
    per_simd = wave_instr * 65536 / 1024
    print(f"{nb} C2 blocks: compressed {a[0]:.0f} B, raw {a[1]:.0f} B, {a[2]:.0f} tags, "
          f"longest copy chain {a[3]:.1f} hops")
    print(f"  rounds: tag starts {a[4]:.1f}, byte sources {a[5]:.1f}")
    print(f"  lane ops per block {a[6]:.0f} = {wave_instr:.0f} wave instructions "
          f"(the ring: ~1.9 K per block)")
    print(f"  C2 per SIMD: {per_simd / 1e3:.0f} K wave instructions = "
          f"{per_simd * 2 / 2.4e3:.0f} us of VALU issue at 2 cycles each, 2.4 GHz "
          f"(the ring's whole launch: 281 us)")


if __name__ == "__main__":
    main()
