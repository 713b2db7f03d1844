#!/usr/bin/env python3
"""A/B timing of probe builds of the codec library on C2 (timing only).

usage: python tools/probe_ab.py LIB[@DECODER] [LIB[@DECODER] ...]
Each LIB (a .so built from the same sources with a probe macro, e.g.
-DLGS_PROBE_ALIGNED_RING) runs in its own process: C2 encode and decode,
3 warm-up + 20 timed launches each, HIP events on the launch stream.
Probe builds may produce wrong bytes by design; only the statuses are
checked (a probe must not change the control flow).  With PROBE_CHECK=1
each library's C2 output is also checked against the pinned reference
digest and the raw blocks (for candidate builds, not probes).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib: str) -> None:
    sys.path.insert(0, ROOT)
    import lcdb_amd.build as b
    b.LIB = os.path.abspath(lib)
    import numpy as np
    import torch
    from lcdb_amd import batch, corpus
    c = corpus.fillseq(65536)
    k = int(os.environ.get("PROBE_SHIFT", "0"))
    if k:   # every block k bytes off its 16-byte alignment
        buf = np.zeros(len(c.buf) + k, dtype=np.uint8)
        buf[k:] = c.buf
        c = corpus.Corpus(buf, c.off + np.uint64(k), c.len)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)
    out = batch.decode_slots(c.len)
    kd = int(os.environ.get("PROBE_DSHIFT", "0"))
    kc = int(os.environ.get("PROBE_CSHIFT", str(kd)))   # compressed streams only
    ko = int(os.environ.get("PROBE_OSHIFT", str(kd)))   # decoder outputs only
    if kc:  # compressed streams kc bytes off their 16-byte alignment
        comp.off += kc
    if ko:  # decoder outputs ko bytes off
        out = batch.decode_slots(c.len + 16)
        out.off += ko
    st = torch.zeros(c.n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    res = {"lib": os.path.basename(lib) + (("@" + os.environ["LGS_DECODE_KERNEL"])
                                           if os.environ.get("LGS_DECODE_KERNEL") else "")}
    for name, fn in (("encode", lambda: batch.encode(raw, comp, s)),
                     ("decode", lambda: batch.decode(comp, out, st, s))):
        ts = []
        for k in range(23):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            if k >= 3:
                ts.append(e0.elapsed_time(e1) * 1e3)
        res[name + "_us"] = float(np.mean(ts))
        res[name + "_GiBps"] = c.raw_bytes / (res[name + "_us"] * 1e-6) / 2**30
    res["status_ok"] = bool((st == 1).all())
    if os.environ.get("PROBE_CHECK"):
        # a candidate (not a probe): its bytes must be the reference's
        dg = json.load(open(os.path.join(ROOT, "tests", "golden", "digests.json")))
        hc, ho = batch.to_host(comp), batch.to_host(out)
        res["encode_exact"] = corpus.digest_of_digests(
            corpus.block_digests(hc.buf, hc.off, hc.len)) == dg["C2_fillseq_65536x4KiB"]["comp_dd"]
        res["decode_exact"] = bool(np.array_equal(corpus.block_digests(ho.buf, ho.off, ho.len),
                                                  corpus.block_digests(c.buf, c.off, c.len)))
    print(json.dumps(res), flush=True)


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    for spec in sys.argv[1:]:
        # LIB or LIB@DECODER (LGS_DECODE_KERNEL for that child: ring, quad, wave)
        lib, _, dk = spec.partition("@")
        env = dict(os.environ, **({"LGS_DECODE_KERNEL": dk} if dk else {}))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib],
                           capture_output=True, text=True, timeout=300, env=env)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        print(line[-1] if line else f"{lib}: rc={r.returncode} {r.stderr[-800:]}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
