#!/usr/bin/env python3
"""Write profiles/traffic_latest.json from a tools/profile.sh directory.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both KiB x 1024), the
gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE tallies 128-B
requests at 64 B for wide coalesced streaming reads (our staging loads are
16 B/lane coalesced), WRITE_SIZE is exact.  FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes.  Entries for kernels absent from this profile
are kept from the previous file.

usage: python tools/traffic_json.py gpurun_out/prof_TAG [TAG]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "traffic_latest.json")


def main() -> None:
    d = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d.rstrip("/"))
    tmp = os.path.join(d, "pmc_summary.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), d,
                    "--json", tmp], check=True, stdout=subprocess.DEVNULL)
    summ = json.load(open(tmp))
    try:
        cur = json.load(open(OUT))
    except (OSError, ValueError):
        cur = {"blocks": 65536, "kernels": {}}
    for name, m in summ.items():
        if "hbm_bytes_per_launch" not in m:
            continue
        kind = "encode" if "encode_kernel" in name else "decode" if "decode" in name else None
        if kind is None:
            continue
        cur["kernels"][kind] = {
            "kernel": name, "hbm_bytes_per_launch": m["hbm_bytes_per_launch"],
            "fetch_size_kib": m["FETCH_SIZE"], "write_size_kib": m["WRITE_SIZE"],
            "avg_us_profiled": m.get("avg_us"), "profile": tag,
            "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950, MI355X_MICROARCH.md HBM)",
        }
    cur["blocks"] = 65536
    sys.path.insert(0, ROOT)
    from lcdb_amd.build import kernel_sources_sha
    cur["sources_sha"] = kernel_sources_sha()   # bench.py drops traffic on a mismatch
    json.dump(cur, open(OUT, "w"), indent=1, sort_keys=True)
    print(json.dumps(cur, indent=1))


if __name__ == "__main__":
    main()
