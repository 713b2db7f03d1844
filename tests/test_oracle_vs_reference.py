"""Seeded differential fuzz: restatement vs the reference compiled from
lcdb's own snappy.c (oracle/_ref).  Skipped where the reference build is
absent; the golden vectors still pin the restatement there."""
from __future__ import annotations

import random

import pytest

import oracle

ref = oracle.reference()
pytestmark = pytest.mark.skipif(ref is None, reason="oracle/_ref/libref_snappy.so not built")


def _rand_input(rng: random.Random) -> bytes:
    n = rng.choice([rng.randrange(0, 64), rng.randrange(64, 5000), rng.randrange(60000, 140000)])
    kind = rng.randrange(4)
    if kind == 0:
        return bytes(rng.randrange(256) for _ in range(n))
    if kind == 1:
        alpha = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 6)))
        return bytes(rng.choice(alpha) for _ in range(n))
    if kind == 2:
        unit = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 40)))
        return (unit * (n // max(1, len(unit)) + 1))[:n]
    b = bytearray(n)
    for _ in range(n // 16):
        b[rng.randrange(n)] = rng.randrange(256)
    return bytes(b)


def test_encode_matches_reference():
    orc = oracle.restatement()
    rng = random.Random(1234)
    for _ in range(120):
        data = _rand_input(rng)
        assert orc.encode(data) == ref.encode(data)


def test_decode_accept_reject_matches_reference():
    orc = oracle.restatement()
    rng = random.Random(99)
    for _ in range(1500):
        base = ref.encode(_rand_input(rng)[:3000])
        b = bytearray(base)
        op = rng.randrange(3)
        if op == 0 and b:
            for _ in range(rng.randrange(1, 4)):
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
        elif op == 1:
            b = b[:rng.randrange(len(b) + 1)]
        else:
            b = bytearray(rng.randrange(256) for _ in range(rng.randrange(0, 64)))
        assert orc.decode(bytes(b)) == ref.decode(bytes(b))
        assert orc.decode_size(bytes(b)) == ref.decode_size(bytes(b))
