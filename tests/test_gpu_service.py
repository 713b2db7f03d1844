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


def test_service_same_slot_back_to_back(gpu, vectors):
    """Same-length, different-content streams back to back through one slot
    (GPUTEST_r05: craft/overlap1/d10 right after craft/overlap/d10 came back
    corrupt when round 5 staged inputs in host-written device
    memory).  A single thread leases the same slot every call; every result
    is checked against the oracle."""
    ref = oracle.best()
    by_name = {v.name: v for v in vectors if v.kind == 1}
    pair = [by_name["craft/overlap/d10"].a, by_name["craft/overlap1/d10"].a]
    # Valid streams of one length that differ only in their last literal
    # byte, and their corruptions of equal length.
    rng = random.Random(11)
    base = bytearray(rng.randrange(256) for _ in range(3000))
    twins = []
    for k in range(8):
        b = bytes(base[:-1]) + bytes([k])
        twins.append(ref.encode(b))
    assert len({len(t) for t in twins}) == 1 and len(set(twins)) == 8
    # Every golden decode vector, grouped by length, so neighbours share one.
    groups: dict[int, list[bytes]] = {}
    for v in vectors:
        if v.kind == 1 and len(v.a) <= 4096:
            groups.setdefault(len(v.a), []).append(v.a)
    seq = []
    for _ in range(200):
        seq += pair
    for _ in range(20):
        seq += twins
    for g in groups.values():
        if len(g) > 1:
            seq += g * 3
    want = {s: ref.decode(s) for s in set(seq)}
    bad = [(i, s) for i, s in enumerate(seq) if gpu.decode(s) != want[s]]
    assert not bad, f"{len(bad)} of {len(seq)} wrong, first at {bad[0][0]}: {bad[0][1]!r}"
    # Encode through the same slot: inputs of one length, different bytes.
    blocks = [bytes(base[:-1]) + bytes([k]) for k in range(8)] * 25
    assert [gpu.encode(b) for b in blocks] == [ref.encode(b) for b in blocks]


_CHILD_TWO_SLOTS = textwrap.dedent("""
    import sys, threading, time
    sys.path.insert(0, {root!r})
    import oracle
    from lcdb_amd import corpus, snappy
    import torch
    ref = oracle.best()
    c = corpus.fillseq(16)
    blocks = list(c.blocks())
    streams = [ref.encode(b) for b in blocks]
    stop = threading.Event()
    errors = []
    def busy():
        k = 0
        while not stop.is_set():
            i = k % len(blocks)
            if snappy.decode(streams[i]) != blocks[i]:
                errors.append(("busy", i))
            k += 1
    t = threading.Thread(target=busy)
    t.start()
    time.sleep(0.05)
    worst = 0.0
    for k in range(60):
        time.sleep(0.0003 + 0.0001 * (k % 9))     # around the 300 us idle mark
        i = k % len(blocks)
        t0 = time.perf_counter()
        e = snappy.encode(blocks[i])
        ok = e == streams[i] and snappy.decode(e) == blocks[i]
        worst = max(worst, time.perf_counter() - t0)
        if not ok:
            errors.append(("idle", i))
    stop.set()
    t.join()
    assert not errors, errors[:5]
    print("ok", round(worst * 1e3, 3))
""")


def test_service_busy_slot_does_not_strand_another(gpu):
    """one slot kept busy across the idle boundary, another
    slot calling now and then around the 300 us idle mark.  The waves leave
    together (lgs_service.h), so the second slot's calls are answered at
    once rather than after the busy slot's traffic stops."""
    env = dict(os.environ, LGS_SERVICE_IDLE_US="300", LGS_DROPIN_SERVICE="1")
    r = subprocess.run([sys.executable, "-c", _CHILD_TWO_SLOTS.format(root=ROOT)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout.strip()
    assert out.startswith("ok"), out
    assert float(out.split()[1]) < 500.0, out          # ms for the slowest round trip


_CHILD_QUIESCE = textwrap.dedent("""
    import sys, threading, time
    sys.path.insert(0, {root!r})
    import oracle
    from lcdb_amd import _native, corpus, snappy
    import torch
    ref = oracle.best()
    blocks = list(corpus.fillseq(8).blocks())
    streams = [ref.encode(b) for b in blocks]
    stop = threading.Event()
    errors = []
    def busy():
        k = 0
        while not stop.is_set():
            i = k % len(blocks)
            if snappy.decode(streams[i]) != blocks[i]:
                errors.append(i)
            k += 1
    ts = [threading.Thread(target=busy) for _ in range(2)]
    for t in ts:
        t.start()
    time.sleep(0.1)
    worst = 0.0
    for _ in range(5):
        t0 = time.perf_counter()
        _native.check(_native.lib().lgs_service_quiesce(), "quiesce")
        torch.cuda.synchronize()
        worst = max(worst, time.perf_counter() - t0)
        time.sleep(0.01)                      # calls keep coming, launch path
        _native.check(_native.lib().lgs_service_resume(), "resume")
        time.sleep(0.01)
    stop.set()
    for t in ts:
        t.join()
    assert not errors, errors[:5]
    print("ok", round(worst * 1e3, 3))
""")


def test_service_quiesce_under_traffic(gpu):
    """lgs_service_quiesce / _resume: with two threads calling without pause
    (the service never idles), a device-wide synchronisation after quiesce
    returns promptly, and every call -- before, during (launch path, or a
    request withdrawn from the stopped waves) and after -- is still right."""
    env = dict(os.environ, LGS_DROPIN_SERVICE="1")
    r = subprocess.run([sys.executable, "-c", _CHILD_QUIESCE.format(root=ROOT)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = r.stdout.strip()
    assert out.startswith("ok"), out
    assert float(out.split()[1]) < 1000.0, out
