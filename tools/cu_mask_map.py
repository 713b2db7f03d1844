#!/usr/bin/env python3
"""How many CUs a hipExtStreamCreateWithCUMask mask really gives: the C2
encode kernel (65 536 one-wave workgroups) timed alone on streams whose mask
sets K CUs, contiguous bits [0, K) or spread (every 256/K-th bit).  Its time
scales as 1 / (CUs it runs on).  usage: python tools/cu_mask_map.py"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import numpy as np
    import torch
    from lcdb_amd import batch, corpus
    torch.cuda.set_device(0)
    hip = C.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    words = (ncu + 31) // 32
    c = corpus.fillseq(65536)
    raw = batch.upload(c)
    comp = batch.encode_slots(raw)

    def stream(bits):
        m = [0] * words
        for i in bits:
            m[i // 32] |= 1 << (i % 32)
        s = C.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(words), (C.c_uint32 * words)(*m)) == 0
        return torch.cuda.ExternalStream(s.value, device=torch.device("cuda", 0))

    def t_enc(s):
        ts = []
        for k in range(6):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            batch.encode(raw, comp, s)
            e1.record(s)
            torch.cuda.synchronize()
            if k >= 1:
                ts.append(e0.elapsed_time(e1) * 1e3)
        return float(np.median(ts))

    full = t_enc(torch.cuda.current_stream())
    res = {"ncu": ncu, "full_us": full}
    for K in (32, 64, 128, 192):
        for name, bits in (("contig", range(K)), ("spread", [i for i in range(ncu) if (i * K) % ncu < K])):
            bits = list(bits)
            t = t_enc(stream(bits))
            res[f"{name}_{K}"] = {"set": len(bits), "us": round(t, 1), "effective_cus": round(ncu * full / t, 1)}
    for name, bits in (("xcd_interleave_0mod8", [i for i in range(ncu) if i % 8 == 0]),
                       ("low_half_each_word", [i for i in range(ncu) if i % 32 < 16])):
        t = t_enc(stream(bits))
        res[name] = {"set": len(bits), "us": round(t, 1), "effective_cus": round(ncu * full / t, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
