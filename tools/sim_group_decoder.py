#!/usr/bin/env python3
"""The workgroup decoder's window algorithm (lcdb_amd/csrc/lgs_decode_group.hip),
restated sequentially in Python, run against every golden decode vector and
seeded corruptions of real blocks (a logic check before GPU time: windows,
pointer-doubling marks, cuts, solo literals, source resolution, rejects).
It also prints the rounds each step takes (marking and resolve rounds per
window) on fillseq 4 KiB / 64 KiB blocks.

usage: python tools/sim_group_decoder.py [--stats]
"""
from __future__ import annotations

import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

IN_WIN, OUT_WIN, NT = 4096, 8192, 1024
KSW = IN_WIN + 96
C = OUT_WIN // NT
TERM = None


def parse_tag(z: bytes, p: int, S: int, want: int, made: int):
    """lgs_decode_common.h parse_tag: (kind, len, hl, dist, next, bad)."""
    b = z[p:p + 5].ljust(5, b"\0")
    tag = b[0]
    kind, m0 = tag & 3, tag >> 2
    left = S - p
    b1 = int.from_bytes(b[1:5], "little")
    lit = kind == 0
    extra = m0 - 59 if m0 >= 60 else 0
    emask = 0xFFFFFFFF if extra >= 4 else (1 << (8 * extra)) - 1
    m = (b1 & emask) if extra else m0
    clen = 4 + (m0 & 7) if kind == 1 else m0 + 1
    cdist = (((tag & 0xE0) << 3) | (b1 & 0xFF)) if kind == 1 else ((b1 & 0xFFFF) if kind == 2 else b1)
    ln = m + 1 if lit else clen
    hl = 1 + extra if lit else (5 if kind == 3 else kind + 1)
    dist = 0 if lit else cdist
    u = lambda x: x & 0xFFFFFFFF
    bad = (hl > left) or (ln > u(want - made)) or (
        ((m >= 0x7FFFFFFF) or (hl + ln > left)) if lit else (u(cdist - 1) >= made))
    return kind, ln, hl, dist, p + hl + (ln if lit else 0), bad


def decode(z: bytes, cap: int = 66048, stats=None):
    S = len(z)
    want, hlen = 0, 0
    for k in range(min(5, S)):
        b = z[k]
        want = (want | ((b & 0x7F) << (7 * k))) & 0xFFFFFFFF
        if b < 0x80:
            hlen = k + 1
            break
    if hlen == 0 or want > 0x7FFFFFFF:
        return 0, None
    if want > cap:
        return 2, None
    img = bytearray(want + 64)
    ws, wo = hlen, 0
    while ws < S:
        wn = min(IN_WIN, S - ws)
        sw = z[ws:ws + KSW]
        # parse
        J = [TERM] * IN_WIN
        for r in range(wn):
            _, _, _, _, nxt, bad = parse_tag(z, ws + r, S, 0xFFFFFFFF, 0x7FFFFFFF)
            if not bad and nxt - ws < wn:
                J[r] = nxt - ws
        M = [False] * IN_WIN
        M[0] = True
        rounds = 0
        while J[0] is not TERM:
            J2 = [TERM] * IN_WIN
            for r in range(IN_WIN):
                a = J[r]
                if a is not TERM:
                    if M[r]:
                        M[a] = True
                    J2[r] = J[a]
            J = J2
            rounds += 1
        # ops
        ops, mb, bad_any, nxt_last, cut = [], 0, False, S, None
        for r in range(wn):
            if not M[r]:
                continue
            kind, ln, hl, dist, nxt, bad = parse_tag(z, ws + r, S, want, wo + mb)
            lit = kind == 0
            ln = 0 if bad else ln
            ops.append((mb, (ws + r + hl) if lit else dist, r, lit, ln))
            if bad:
                bad_any = True
            elif nxt - ws >= wn:
                nxt_last = nxt
            if mb <= OUT_WIN < mb + ln:
                cut = len(ops) - 1
            mb += ln
        lw = mb
        if bad_any:
            return 0, None
        solo = lw > OUT_WIN and cut == 0
        if lw <= OUT_WIN:
            wl, nws, nops = lw, nxt_last, len(ops)
        elif not solo:
            wl, nws, nops = ops[cut][0], ws + ops[cut][2], cut
        else:
            wl = ops[1][0] if len(ops) > 1 else lw
            nws = ws + ops[1][2] if len(ops) > 1 else nxt_last
            nops = 1
        if not solo:
            R = [0] * wl
            for k in range(nops):
                oo, sv, _, lit, ln = ops[k]
                for j in range(ln):
                    o = oo + j
                    if o >= wl:
                        break
                    if lit:
                        q = sv + j
                        img[wo + o] = sw[q - ws] if q - ws < KSW else z[q]
                        R[o] = wo + o
                    else:
                        R[o] = wo + o - sv
            rr = 0
            changed = True
            while changed:
                changed = False
                R2 = list(R)   # (the kernel updates in place: fewer rounds, same fixed point)
                for o in range(wl):
                    r0 = R[o]
                    if r0 >= wo and r0 != wo + o:
                        r1 = R[r0 - wo]
                        if r1 != r0:
                            R2[o] = r1
                            changed = True
                R = R2
                rr += 1
            for o in range(wl):
                if R[o] != wo + o:
                    img[wo + o] = img[R[o]]
            if stats is not None:
                stats.append((rounds, rr, len(ops), wl))
        else:
            lp = ops[0][1]
            for o in range(wl):
                q = lp + o
                img[wo + o] = sw[q - ws] if q - ws < KSW else z[q]
        wo += wl
        ws = nws
    if wo != want:
        return 0, None
    return 1, bytes(img[:want])


def main() -> None:
    import golden_io
    import oracle
    ref = oracle.best()
    vecs = [v for v in golden_io.read() if v.kind == 1]
    bad = 0
    for v in vecs:
        st, outb = decode(v.a)
        exp_st = 1 if v.ok else 0
        # oversize headers: the kernel's class cap makes them status 2
        if st == 2:
            continue
        if st != exp_st or (st == 1 and outb != v.b):
            bad += 1
            print("MISMATCH", v.name, st, exp_st)
    print(f"golden decode vectors: {len(vecs)}, mismatches {bad}")
    from lcdb_amd import corpus
    rng = random.Random(7)
    n = 0
    for c in (corpus.fillseq(24), corpus.fillseq(3, 65536), corpus.random_blocks(4, 4096)):
        for i in range(c.n):
            raw = c.block(i)
            z = ref.encode(raw)
            st, outb = decode(z)
            assert st == 1 and outb == raw, ("clean", i)
            for _ in range(40):
                zz = bytearray(z)
                for _ in range(rng.randint(1, 3)):
                    zz[rng.randrange(len(zz))] = rng.randrange(256)
                if rng.random() < 0.3:
                    zz = zz[:rng.randrange(1, len(zz))]
                zz = bytes(zz)
                exp = ref.decode(zz)
                exp_ok = exp is not None
                st, outb = decode(zz)
                if st == 2:
                    continue
                n += 1
                if st != (1 if exp_ok else 0) or (st == 1 and outb != exp):
                    bad += 1
                    print("CORRUPT MISMATCH", i, st, exp_ok)
    print(f"seeded corruptions: {n}, mismatches {bad}")
    if "--stats" in sys.argv:
        for name, c in (("fillseq4K", corpus.fillseq(8)), ("fillseq64K", corpus.fillseq(2, 65536))):
            stats = []
            for i in range(c.n):
                decode(ref.encode(c.block(i)), stats=stats)
            print(name, "windows", len(stats), "(mark rounds, resolve rounds, ops, out):",
                  stats[:12])
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
