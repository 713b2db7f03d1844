"""The drop-in's error and memory contract (SURVEY §8(b) "Errors"; callers
src/table/format.c:237-251 and table_builder.c:182-188).

* A stream whose size header its length cannot satisfy is rejected on the
  host -- the reference's 0, no allocation, no device work (lgs_api.cpp
  host_verdict).  The CPU test drives ONLY such streams through
  ldb_snappy_decode in a child process (any stream reaching the device path
  without a GPU would abort that child, not pytest).
* On the GPU: hdr-5max-style headers and 1 000 seeded corruptions come back
  as the reference's result while the drop-in's staging stays within its
  stated cap (lgs_dropin_footprint); a forced 1 MiB slot (LGS_DROPIN_MB=1)
  still encodes a 4 MiB input byte-identically and decodes it through the
  over-slot path.
"""
from __future__ import annotations

import os
import random
import subprocess
import sys

import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def _host_rejectable(s: bytes):
    """The reference result when the header alone decides it (else None)."""
    want, sh, i = 0, 0, 0
    while True:
        if i >= len(s) or i >= 5:
            return 0
        b = s[i]
        want |= (b & 0x7F) << sh
        i += 1
        if b < 0x80:
            break
        sh += 7
    if want > 0x7FFFFFFF:
        return 0
    m = len(s) - i
    if want == 0:
        return 1 if m == 0 else 0
    if 3 * want > 64 * m or m > 6 * want:
        return 0
    return None


def _streams(seed: int, n: int):
    rng = random.Random(seed)
    out = [b"", b"\x80", b"\xff\xff\xff\xff\x7f", _varint(0x7FFFFFFF), _varint(0x7FFFFFFF) + b"\x00",
           _varint(0), _varint(0) + b"\x00", _varint(1 << 20) + bytes(10), _varint(64) + b"\xfe\x01\x00",
           _varint(65) + b"\xfe\x01\x00", _varint(3) + bytes(19), _varint(3) + bytes(18),
           b"\x80\x00", b"\x80\x80\x00" + b"\x00"]
    for _ in range(n):
        want = rng.choice([rng.randrange(0, 64), rng.randrange(0, 1 << 16), rng.randrange(0, 1 << 31)])
        m = rng.choice([0, 1, 2, 3, rng.randrange(0, 200), rng.randrange(0, 5000)])
        out.append(_varint(want) + bytes(rng.randrange(256) for _ in range(m)))
    return out


def test_host_rejects_need_no_device():
    ref = oracle.best()
    cases = [s for s in _streams(11, 3000) if _host_rejectable(s) is not None]
    assert len(cases) > 1000
    for s in cases:
        assert (ref.decode(s) is not None) == bool(_host_rejectable(s)), s[:16]
    # The drop-in itself, in a child process (no GPU here: these must not
    # touch the device at all).
    prog = r'''
import sys, ctypes as C
sys.path.insert(0, %r)
from lcdb_amd import _native
L = _native.lib()
data = sys.stdin.buffer.read()
res = []
at = 0
while at < len(data):
    n = int.from_bytes(data[at:at + 4], "little"); at += 4
    s = data[at:at + n]; at += n
    buf = C.create_string_buffer(s + b"\0" * 16, len(s) + 16)
    out = C.create_string_buffer(64)
    res.append(str(L.ldb_snappy_decode(out, buf, len(s))))
print(",".join(res))
''' % ROOT
    blob = b"".join(len(s).to_bytes(4, "little") + s for s in cases)
    r = subprocess.run([sys.executable, "-c", prog], input=blob, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = [int(x) for x in r.stdout.decode().strip().split(",")]
    assert got == [int(bool(_host_rejectable(s))) for s in cases]


@pytest.mark.gpu
def test_dropin_corrupt_streams_bounded(gpu, vectors):
    from lcdb_amd import _native, corpus
    ref = oracle.best()
    rng = random.Random(5)
    good = [ref.encode(b) for b in corpus.fillseq(40).blocks()]
    streams = _streams(12, 300)
    streams += [v.a for v in vectors if v.kind == 1 and v.name.startswith("craft/hdr")]
    for _ in range(1000):                       # seeded corruptions of real blocks
        s = bytearray(rng.choice(good))
        for _ in range(rng.randrange(1, 4)):
            if not s:
                break
            op = rng.randrange(3)
            if op == 0:
                k = rng.randrange(len(s))
                s[k] ^= 1 << rng.randrange(8)
            elif op == 1:
                del s[rng.randrange(len(s)):]
            else:
                k = rng.randrange(len(s))
                s[k:k] = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 9)))
        streams.append(bytes(s))
    for s in streams:
        assert gpu.decode(s) == ref.decode(s), s[:12]
    fp = _native.dropin_footprint()
    assert fp["slot_bytes"] == 4 << 20
    assert 1 <= fp["slots"] <= 8
    assert fp["pinned"] <= fp["slots"] * fp["slot_bytes"]
    assert fp["device"] <= fp["slots"] * fp["slot_bytes"]


@pytest.mark.gpu
def test_dropin_small_slot_large_blocks(gpu, tmp_path):
    # LGS_DROPIN_MB=1: a 4 MiB input is encoded in 1 MiB-slot passes of whole
    # 64 KiB chunks (byte-identical to the reference), and decoded through
    # the over-slot path (device memory for that call only).
    prog = r'''
import sys, hashlib
sys.path.insert(0, %r)
import numpy as np
import oracle
from lcdb_amd import corpus, snappy, _native
c = corpus.fillseq(600)
data = b"".join(c.blocks())[:4 << 20]
data = data + bytes(range(256)) * 37 + b"tail"
ref = oracle.best()
enc = snappy.encode(data)
assert enc == ref.encode(data), "encode differs"
assert snappy.decode(enc) == data, "decode differs"
bad = bytearray(enc); bad[len(bad) // 2] ^= 0x40
assert snappy.decode(bytes(bad)) == ref.decode(bytes(bad))
fp = _native.dropin_footprint()
assert fp["slot_bytes"] == 1 << 20, fp
assert fp["pinned"] <= fp["slots"] * fp["slot_bytes"], fp
print("ok", len(data), len(enc), fp)
''' % ROOT
    env = dict(os.environ, LGS_DROPIN_MB="1")
    r = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (r.stdout, r.stderr[-3000:])


@pytest.mark.gpu
def test_dropin_alloc_failure_is_not_corruption(gpu):
    # a block larger than a drop-in slot takes device memory for
    # the call; a failed allocation must never come back as 0 (lcdb turns
    # that into LDB_CORRUPTION, format.c:247-251).  A few failures are
    # retried and the block decodes; a device that stays out of memory ends
    # the call loudly (LGS_DIE_EXIT makes that an exit code, not SIGABRT).
    prog = r'''
import sys
sys.path.insert(0, %r)
import oracle
from lcdb_amd import corpus, snappy, _native
data = b"".join(corpus.fillseq(400).blocks())[:(3 << 20) + 77]
enc = oracle.best().encode(data)
_native.set_option("inject_alloc_failures", sys.argv[1])
out = snappy.decode(enc)
print("decoded", out == data)
''' % ROOT
    env = dict(os.environ, LGS_DROPIN_MB="1", LGS_DIE_EXIT="70")
    r = subprocess.run([sys.executable, "-c", prog, "3"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "decoded True", (r.stdout, r.stderr[-2000:])
    r = subprocess.run([sys.executable, "-c", prog, "1000"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 70, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "decoded" not in r.stdout
    assert "hipMalloc" in r.stderr and "ldb_snappy_decode failed" in r.stderr, r.stderr[-2000:]
