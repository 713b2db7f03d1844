"""Bloom filter oracle (oracle/bloom_oracle.c), pinned (CPU only) to the
known answers of the reference's test/t-hash.c and to lcdb's own bloom.c +
hash.c (oracle/harness/bloom_ref.c, linked against lcdb's sources)."""
from __future__ import annotations

import random

import pytest

import oracle

RFC3720 = bytes([
    0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00,
    0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18, 0x28, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00])

# test/t-hash.c:33-38
HASH_KNOWN = [
    (b"", 0xbc9f1d34, 0xbc9f1d34),
    (bytes([0x62]), 0xbc9f1d34, 0xef1345c4),
    (bytes([0xc3, 0x97]), 0xbc9f1d34, 0x5b663814),
    (bytes([0xe2, 0x99, 0xa5]), 0xbc9f1d34, 0x323c078f),
    (bytes([0xe1, 0x80, 0xb9, 0x32]), 0xbc9f1d34, 0xed21633a),
    (RFC3720, 0x12345678, 0xf333dabb),
]


def _impls():
    out = [oracle.bloom_restatement()]
    ref = oracle.bloom_reference()
    if ref is not None:
        out.append(ref)
    return out


@pytest.mark.parametrize("data,seed,want", HASH_KNOWN)
def test_hash_known_answers(data, seed, want):
    for b in _impls():
        assert b.hash(data, seed) == want, b.name


def key_groups(seed: int):
    """Key sets of every shape the filter path meets (test infrastructure)."""
    rng = random.Random(seed)
    groups = [[], [b""], [b"a"], [b"hello", b"world"]]
    groups.append([b"%016d" % k for k in range(36)])               # a fillseq block's keys
    groups.append([rng.randbytes(rng.randrange(0, 60)) for _ in range(rng.randrange(1, 300))])
    groups.append([b"%08d" % k for k in range(7000)])              # > 8 KiB of bits at 10/key
    for _ in range(20):
        groups.append([rng.randbytes(rng.randrange(0, 40)) for _ in range(rng.randrange(0, 80))])
    return groups


BPK = [0, 1, 5, 10, 16, 44, 50]


def test_bloom_build_and_match_vs_reference():
    ref = oracle.bloom_reference()
    if ref is None:
        pytest.skip("oracle/_ref/lcdb/libref_bloom.so not built")
    orc = oracle.bloom_restatement()
    rng = random.Random(7)
    for bpk in BPK:
        for g in key_groups(bpk):
            f_ref, f_orc = ref.build(g, bpk), orc.build(g, bpk)
            assert f_ref == f_orc, (bpk, len(g))
            probes = g[:50] + [rng.randbytes(rng.randrange(0, 30)) for _ in range(50)]
            for k in probes:
                assert ref.match(f_ref, k) == orc.match(f_orc, k)
    # Edge filters: too short, and k > 30 ("reserved", bloom.c:137-141).
    for filt in (b"", b"\x01", b"\x00\x00\x1f", b"\xff" * 8 + b"\x06", b"\x00" * 8 + b"\x06"):
        for k in (b"", b"x", b"hello"):
            assert ref.match(filt, k) == orc.match(filt, k)


def test_members_always_match():
    # t-bloom.c:44-64: no false negatives.
    orc = oracle.bloom_restatement()
    for g in key_groups(3):
        f = orc.build(g, 10)
        assert all(orc.match(f, k) for k in g)
