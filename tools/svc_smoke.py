#!/usr/bin/env python3
"""A few drop-in calls through the resident service (debug aid): prints the
results and the first error, stderr unbuffered."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from lcdb_amd import corpus, snappy  # noqa: E402

ref = oracle.best()
c = corpus.fillseq(16)
t0 = time.perf_counter()
e = snappy.encode(c.block(0))
print("first encode", len(e), e == ref.encode(c.block(0)), round((time.perf_counter() - t0) * 1e3, 3), "ms", flush=True)
d = snappy.decode(e)
print("first decode", d == c.block(0), flush=True)
ok = 0
for b in c.blocks():
    e = snappy.encode(b)
    ok += e == ref.encode(b) and snappy.decode(e) == b
print("ok", ok, "of", c.n, flush=True)
