#!/usr/bin/env python3
"""Where a decoder build writes wrong bytes on C2 (diagnosis, not a test).

usage: LGS_DECODE_KERNEL=quad python tools/quad_diag.py LIB [MAX_BLOCKS]
Decodes C2 with LIB, then for each block whose output differs from the raw
block maps every wrong byte to the op of the stream that produced it (a
literal, a copy from the 240-byte near window, or a far copy) and tests what
the wrong value equals: the stream byte one input-ring lap (128) earlier, the
output byte one output-ring lap (256) earlier, or zero.  Prints one JSON line
of totals and up to MAX_BLOCKS per-block lines.
"""
from __future__ import annotations

import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ops_of(stream: bytes):
    """(kind, out_pos, length, dist, stream_pos_of_first_byte) per op."""
    p, want, sh = 0, 0, 0
    while True:
        b = stream[p]
        want |= (b & 0x7F) << sh
        p += 1
        sh += 7
        if b < 0x80:
            break
    out, ops = 0, []
    while p < len(stream):
        t = stream[p]
        k, m = t & 3, t >> 2
        if k == 0:
            if m >= 60:
                e = m - 59
                ln = int.from_bytes(stream[p + 1:p + 1 + e], "little") + 1
                hl = 1 + e
            else:
                ln, hl = m + 1, 1
            ops.append(("lit", out, ln, 0, p + hl))
            p += hl + ln
        elif k == 1:
            ln, d = 4 + ((m) & 7), ((t & 0xE0) << 3) | stream[p + 1]
            ops.append(("copy", out, ln, d, p))
            p += 2
        elif k == 2:
            ln, d = m + 1, int.from_bytes(stream[p + 1:p + 3], "little")
            ops.append(("copy", out, ln, d, p))
            p += 3
        else:
            ln, d = m + 1, int.from_bytes(stream[p + 1:p + 5], "little")
            ops.append(("copy", out, ln, d, p))
            p += 5
        out += ln
    return ops


def main() -> None:
    lib = sys.argv[1]
    maxb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sys.path.insert(0, ROOT)
    import lcdb_amd.build as b
    b.LIB = os.path.abspath(lib)
    import numpy as np
    import torch
    from lcdb_amd import batch, corpus
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    out = batch.decode_slots(c.len)
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    batch.encode(raw, comp, s)
    batch.decode(comp, out, st, s)
    torch.cuda.synchronize()
    hc, ho = batch.to_host(comp), batch.to_host(out)
    sts = st.cpu().numpy()
    tot = collections.Counter()
    lines = []
    bad_blocks = 0
    for i in range(c.n):
        o0, n = int(c.off[i]), int(c.len[i])
        ref = c.buf[o0:o0 + n]
        got = ho.buf[int(ho.off[i]):int(ho.off[i]) + n]
        if np.array_equal(ref, got):
            continue
        bad_blocks += 1
        stream = bytes(hc.buf[int(hc.off[i]):int(hc.off[i]) + int(hc.len[i])])
        ops = ops_of(stream)
        starts = np.array([op[1] for op in ops])
        wrong = np.nonzero(ref != got)[0]
        per = collections.Counter()
        first = None
        for w in wrong:
            j = int(np.searchsorted(starts, w, side="right") - 1)
            kind, at, ln, d, sp = ops[j]
            cls = kind if kind == "lit" else ("near" if d <= 240 else "far")
            per[cls] += 1
            tot[cls] += 1
            v = int(got[w])
            if kind == "lit":
                q = sp + (w - at)
                if q >= 128 and v == stream[q - 128]:
                    tot["lit=stream-128"] += 1
                if q >= 64 and v == stream[q - 64]:
                    tot["lit=stream-64"] += 1
            if w >= 256 and v == int(ref[w - 256]):
                tot["=out-256"] += 1
            if v == 0:
                tot["=0"] += 1
            if first is None:
                first = {"byte": int(w), "op": j, "kind": kind, "at": at, "len": ln, "dist": d,
                         "stream_pos": sp, "got": v, "want": int(ref[w])}
        tot["wrong_bytes"] += len(wrong)
        if len(lines) < maxb and first is not None:
            # what the first wrong op's bytes equal: output at another
            # distance, or stream bytes somewhere
            at, ln = first["at"], first["len"]
            gotb = bytes(got[at:at + ln])
            first["got_bytes"] = gotb.hex()
            first["want_bytes"] = bytes(ref[at:at + ln]).hex()
            first["as_output_dist"] = [d for d in range(1, at + 1)
                                       if bytes(ref[at - d:at - d + ln]) == gotb][:8]
            first["as_stream_pos"] = [x for x in range(len(stream) - ln)
                                      if stream[x:x + ln] == gotb][:8]
            first["as_got_output_dist"] = [d for d in range(1, at + 1)
                                           if bytes(got[at - d:at - d + ln]) == gotb][:8]
        if len(lines) < maxb:
            lines.append({"block": i, "status": int(sts[i]), "wrong": int(len(wrong)),
                          "by_op_class": dict(per), "first": first,
                          "ops": len(ops), "stream_len": len(stream)})
    print(json.dumps({"lib": os.path.basename(lib), "bad_blocks": bad_blocks,
                      "status_ok": int((sts == 1).sum()), **dict(tot)}), flush=True)
    for ln in lines:
        print(json.dumps(ln), flush=True)


if __name__ == "__main__":
    main()
