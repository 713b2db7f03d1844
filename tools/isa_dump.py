#!/usr/bin/env python3
"""Device ISA of one kernel of a codec source, for instruction counting.

usage: python tools/isa_dump.py SOURCE.hip KERNEL_SUBSTRING [OUT.s] [-- extra hipcc args]

Compiles SOURCE for gfx950 (device only, -O3, the build's flags), writes the
named kernel's assembly to OUT.s (default /tmp/<kernel>.s) and prints its
basic blocks with their instruction counts by class (VALU, SALU, LDS,
VMEM, branch, wait), loops marked.  Used to count the hot loop of a kernel
before and after a change.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(ins: str) -> str:
    op = ins.split()[0]
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main() -> None:
    args = sys.argv[1:]
    extra: list[str] = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    src, kname = args[0], args[1]
    out = args[2] if len(args) > 2 else None
    asm = "/tmp/_isa_dump.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17",
                    "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S", src,
                    "-o", asm, *extra], check=True)
    lines = open(asm).read().split("\n")
    starts = [i for i, ln in enumerate(lines)
              if re.match(r"^_Z\w+:", ln) and kname in ln]
    if not starts:
        sys.exit(f"no kernel matching {kname}")
    st = starts[0]
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[st:en]
    out = out or f"/tmp/{kname}.s"
    open(out, "w").write("\n".join(body) + "\n")
    blk, counts, total = lines[st].rstrip(":"), {}, 0

    def flush() -> None:
        if counts:
            n = sum(counts.values())
            print(f"{blk:60s} {n:4d}  " + " ".join(f"{k}={v}" for k, v in sorted(counts.items())))

    for ln in body[1:]:
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):", ln.strip()) or re.match(r"^\.LBB\w+:", ln):
            flush()
            blk, counts = ln.strip()[:60], {}
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".")) or ln.startswith(("\t.", "\t;")):
            continue
        if not ln.startswith("\t"):
            continue
        c = classify(t)
        counts[c] = counts.get(c, 0) + 1
        total += 1
    flush()
    print(f"total {total} instructions -> {out}")


if __name__ == "__main__":
    main()
