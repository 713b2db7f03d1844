#!/usr/bin/env python3
"""Summarise tools/profile.sh output: per-kernel average duration (trace) and
PMC counters per dispatch, with per-wave ratios and HBM bytes.

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE
reports half the bytes of wide coalesced streaming reads on gfx950; the
corrected read estimate doubles it (`fetch_x2`).  Usage:
    python tools/pmc_summary.py gpurun_out/prof_TAG [--json out.json]
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys


def main() -> None:
    d = sys.argv[1]
    out = {}
    stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
    if stats:
        for r in csv.DictReader(open(stats[0])):
            if "lgs::" in r["Name"]:
                k = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                out.setdefault(k, {})["avg_us"] = float(r["AverageNs"]) / 1e3
                out[k]["calls"] = int(r["Calls"])
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            if "lgs::" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            for c, v in cs.items():
                out.setdefault(k, {})[c] = sum(v) / len(v)
    for k, m in out.items():
        w = m.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH",
                      "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                      "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
                if c in m:
                    m[c + "/wave"] = m[c] / w
        if "FETCH_SIZE" in m:
            m["hbm_read_bytes_x2"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = m["hbm_read_bytes_x2"] + m["hbm_write_bytes"]
    for k, m in out.items():
        print(k)
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:.6g}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
