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


# ---- the filter block (filter_block.c) ----

def random_table_layout(rng: random.Random, internal: bool):
    """Data blocks of random keys at increasing file offsets, the shapes the
    filter block meets: empty tables, blocks under and over 2 KiB, a first
    block not at offset 0, key-less blocks (never written by lcdb, but the
    builder's arithmetic is defined for them)."""
    nb = rng.randrange(0, 12)
    lo = 8 if internal else 0
    blocks = [[rng.randbytes(rng.randrange(lo, 30)) for _ in range(
        rng.randrange(0 if rng.random() < 0.1 else 1, 40))] for _ in range(nb)]
    off, pos = [], rng.choice([0, 0, 0, 3000])
    for _ in blocks:
        off.append(pos)
        pos += rng.choice([rng.randrange(10, 300), rng.randrange(100, 9000)])
    return blocks, off, pos


def test_filter_block_vs_reference():
    ref = oracle.bloom_reference()
    if ref is None:
        pytest.skip("oracle/_ref/lcdb/libref_bloom.so not built")
    orc = oracle.bloom_restatement()
    rng = random.Random(21)
    for _ in range(150):
        internal = rng.random() < 0.5
        blocks, off, end = random_table_layout(rng, internal)
        bpk = rng.choice([1, 10, 16])
        fb = orc.filter_block(blocks, off, end, bpk, internal)
        assert fb == ref.filter_block(blocks, off, end, bpk, internal), (off, end)
        keys = [k for b in blocks for k in b] or [b"x" * 9]
        for _ in range(20):
            bo = rng.randrange(0, end + 5000)
            key = rng.choice(keys) if rng.random() < 0.5 else rng.randbytes(rng.randrange(8, 20))
            assert orc.filter_matches(fb, bo, key, internal) == ref.filter_matches(fb, bo, key,
                                                                                   internal)


def malformed_filter_blocks(rng: random.Random, count: int):
    """Too-short blocks, offset arrays past the end, inverted ranges."""
    out = []
    for _ in range(count):
        b = bytearray(rng.randbytes(rng.randrange(0, 40)))
        if len(b) >= 5 and rng.random() < 0.7:
            b[-5:-1] = rng.randrange(0, len(b)).to_bytes(4, "little")
            b[-1] = rng.choice([11, 0, 63, 200])
        out.append(bytes(b))
    return out


def test_filter_matches_malformed_vs_reference():
    ref = oracle.bloom_reference()
    if ref is None:
        pytest.skip("oracle/_ref/lcdb/libref_bloom.so not built")
    orc = oracle.bloom_restatement()
    rng = random.Random(5)
    for blk in malformed_filter_blocks(rng, 1500):
        bo, key = rng.randrange(0, 1 << 16), rng.randbytes(rng.randrange(8, 12))
        for internal in (False, True):
            assert orc.filter_matches(blk, bo, key, internal) == \
                ref.filter_matches(blk, bo, key, internal), (blk, bo)


def lcdb_table_with_filter(tmp_path, entries=5000, block_size=4096):
    """An .ldb written by lcdb's own builder with the DB's filter policy
    (bloom, 10 bits/key), its data blocks' keys and offsets, and its filter
    block as stored in the file."""
    from table_io import block_entries, build_table, dump_blocks, filter_handle
    path = build_table(tmp_path, entries, block_size, bloom_bits=10)
    d = dump_blocks(path, str(tmp_path / "dump"), True)
    nd = d.n - 2                                   # data blocks, then metaindex, index
    fh = filter_handle(d.contents[-2])
    assert fh is not None
    raw = open(path, "rb").read()
    blocks = [[k for k, _ in block_entries(c)] for c in d.contents[:nd]]
    off = [int(x) for x in d.off[:nd]]
    data_end = int(d.off[nd - 1] + d.size[nd - 1] + 5)
    assert fh[0] == data_end                      # the filter block follows the data
    return blocks, off, data_end, raw[fh[0]:fh[0] + fh[1]]


def test_filter_block_of_lcdb_table(tmp_path):
    """The restatement reproduces the filter block lcdb's table builder wrote
    (internal keys, user-key filters), and it answers every key present."""
    blocks, off, end, stored = lcdb_table_with_filter(tmp_path)
    orc = oracle.bloom_restatement()
    assert orc.filter_block(blocks, off, end, 10, True) == stored
    for b, keys in enumerate(blocks):
        for k in keys[::7]:
            assert orc.filter_matches(stored, off[b], k, True)
