"""The drop-in service (lgs_launch.h, lgs_service.h): resident waves that
serve ldb_snappy_encode / ldb_snappy_decode calls of one <= 4 608-byte block
from mailboxes in the slots' mapped memory, instead of a kernel launch and a
stream synchronisation per call.

* Its results are the reference's (golden vectors, corruptions) and equal
  the launch path's (lgs_set_option("service", "0")) call by call.
* Its waves leave after LGS_SERVICE_IDLE_US without a request, and the next
  call brings the kernel back; a device-wide synchronisation after a call
  returns once they have left.
* Concurrent callers (one slot each) are served at once
  (test_gpu_parity.py::test_dropin_concurrent_threads covers the same with
  the service on, the default).
"""
from __future__ import annotations

import os
import random
import subprocess
import sys
import textwrap

import pytest

import oracle
from lcdb_amd import _native, corpus

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _small_cases():
    rng = random.Random(5)
    ref = oracle.best()
    blocks = list(corpus.fillseq(40).blocks())
    blocks += [bytes(rng.randrange(256) for _ in range(n)) for n in (0, 1, 16, 17, 100, 4096, 4608)]
    blocks += [bytes([rng.randrange(3)]) * n for n in (5, 60, 61, 4000)]
    streams = [ref.encode(b) for b in blocks]
    bad = []
    for s in streams[:20]:
        for _ in range(10):
            b = bytearray(s)
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            bad.append(bytes(b))
    return ref, blocks, streams, bad


def test_service_equals_reference_and_launch_path(gpu, vectors, force):
    ref, blocks, streams, bad = _small_cases()
    small = [v for v in vectors if v.kind == 0 and len(v.a) <= 4608]
    got = {}
    for mode in ("1", "0", "1"):
        force("service", mode)
        enc = [gpu.encode(b) for b in blocks] + [gpu.encode(v.a) for v in small]
        dec = [gpu.decode(s) for s in streams] + [gpu.decode(s) for s in bad]
        got.setdefault(mode, []).append((enc, dec))
    want_enc = streams + [v.b for v in small]
    want_dec = blocks + [ref.decode(s) for s in bad]
    for mode, runs in got.items():
        for enc, dec in runs:
            assert enc == want_enc, mode
            assert dec == want_dec, mode


_CHILD = textwrap.dedent("""
    import sys, time
    sys.path.insert(0, {root!r})
    import oracle
    from lcdb_amd import corpus, snappy
    import torch
    ref = oracle.best()
    c = corpus.fillseq(8)
    for b in c.blocks():
        assert snappy.encode(b) == ref.encode(b)
    # the waves leave after 300 us idle; calls after that relaunch them
    for k in range(5):
        time.sleep(0.004)
        b = c.block(k)
        e = snappy.encode(b)
        assert e == ref.encode(b) and snappy.decode(e) == b
    # a device-wide synchronisation right after a call returns once the
    # waves have left (idle), not never
    snappy.encode(c.block(0))
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert dt < 2.0, dt
    print("ok", round(dt * 1e3, 3))
""")


def test_service_idle_exit_and_relaunch(gpu):
    env = dict(os.environ, LGS_SERVICE_IDLE_US="300", LGS_DROPIN_SERVICE="1")
    r = subprocess.run([sys.executable, "-c", _CHILD.format(root=ROOT)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().startswith("ok"), r.stdout
