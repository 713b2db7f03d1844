"""GPU parity of the bloom filter row (§8(f) 4) through the C ABI: filters
built by lgs_bloom_build_* are byte-identical to lcdb's own ldb_bloom_build,
and lgs_bloom_match_* answers exactly as ldb_bloom_match (the reference
behind oracle/harness/bloom_ref.c; the restatement where that is absent)."""
from __future__ import annotations

import random

import numpy as np
import pytest

import oracle
from test_bloom_oracle import BPK, key_groups

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bl(gpu):
    from lcdb_amd import bloom
    return bloom


def _checker():
    return oracle.bloom_reference() or oracle.bloom_restatement()


@pytest.mark.parametrize("bpk", BPK)
def test_build_host_vs_reference(bl, bpk):
    ref = _checker()
    groups = key_groups(100 + bpk)
    got = bl.build_host(groups, bpk)
    for g, f in zip(groups, got):
        assert f == (ref.build(g, bpk) if g else b""), (bpk, len(g))
        assert len(f) == bl.filter_size(len(g), bpk)


def test_match_host_vs_reference(bl):
    ref = _checker()
    rng = random.Random(11)
    groups = key_groups(5)
    filters = bl.build_host(groups, 10)
    edge = [b"", b"\x01", b"\x00\x00\x1f", b"\xff" * 8 + b"\x06", b"\x00" * 8 + b"\x06"]
    filters = filters + edge
    queries = []
    for f, g in enumerate(groups):
        queries += [(f, k) for k in g[:64]]
        queries += [(f, rng.randbytes(rng.randrange(0, 40))) for _ in range(64)]
    for j in range(len(edge)):
        queries += [(len(groups) + j, k) for k in (b"", b"x", b"hello")]
    got = bl.match_host(filters, queries)
    want = np.array([ref.match(filters[f], k) for f, k in queries], dtype=np.uint8)
    assert np.array_equal(got, want)
    # No false negatives (t-bloom.c:44-64).
    for i, (f, k) in enumerate(queries):
        if f < len(groups) and k in set(groups[f]):
            assert got[i] == 1


def test_device_build_and_match_fillseq_scale(bl):
    """65 536 filters of 36 "%016d" keys (one per fillseq data block) built and
    probed on the device; a sample checked against the reference, every
    member matches, the false-positive rate is the reference's."""
    import torch
    ref = _checker()
    nf, per = 65536, 36
    keys = b"".join(b"%016d" % k for k in range(nf * per))
    d_keys = torch.frombuffer(bytearray(keys + b"\0" * 16), dtype=torch.uint8).cuda()
    d_koff = torch.arange(nf * per, dtype=torch.int64).cuda() * 16
    d_klen = torch.full((nf * per,), 16, dtype=torch.int32).cuda()
    d_first = (torch.arange(nf + 1, dtype=torch.int32) * per).cuda()
    size = bl.filter_size(per, 10)
    d_foff = torch.arange(nf, dtype=torch.int64).cuda() * size
    d_out = torch.zeros(nf * size + 16, dtype=torch.uint8).cuda()
    bl.build(d_keys, d_koff, d_klen, d_first, 10, d_out, d_foff)
    torch.cuda.synchronize()
    host = d_out.cpu().numpy().tobytes()
    for f in list(range(0, nf, 4099)) + [nf - 1]:
        g = [b"%016d" % k for k in range(f * per, (f + 1) * per)]
        assert host[f * size:(f + 1) * size] == ref.build(g, 10), f
    # members: every key against its own filter; non-members: keys of the
    # next filter's range against this filter.
    d_flen = torch.full((nf,), size, dtype=torch.int32).cuda()
    d_qf = (torch.arange(nf * per, dtype=torch.int32) // per).cuda()
    d_m = torch.zeros(nf * per, dtype=torch.uint8).cuda()
    bl.match(d_out, d_foff, d_flen, d_qf, d_keys, d_koff, d_klen, d_m)
    torch.cuda.synchronize()
    assert bool((d_m == 1).all())
    d_qn = ((torch.arange(nf * per, dtype=torch.int32) // per + 1) % nf).cuda()
    bl.match(d_out, d_foff, d_flen, d_qn, d_keys, d_koff, d_klen, d_m)
    torch.cuda.synchronize()
    fp = d_m.cpu().numpy()
    sample = range(0, nf * per, 9973)
    want = [ref.match(host[((q // per + 1) % nf) * size:((q // per + 1) % nf + 1) * size],
                      b"%016d" % q) for q in sample]
    assert [bool(fp[q]) for q in sample] == want
    assert fp.mean() < 0.02                                  # t-bloom.c:136


# ---- the filter block (filter_block.c) through lgs_filter_block_* ----

def test_filter_block_host_vs_reference(bl):
    from test_bloom_oracle import random_table_layout
    ref = _checker()
    rng = random.Random(31)
    for _ in range(60):
        internal = rng.random() < 0.5
        blocks, off, end = random_table_layout(rng, internal)
        bpk = rng.choice([1, 10, 16])
        want = ref.filter_block(blocks, off, end, bpk, internal)
        assert bl.filter_block_host(blocks, off, end, bpk, internal) == want, (off, end)


def test_filter_block_match_host_vs_reference(bl):
    from test_bloom_oracle import malformed_filter_blocks, random_table_layout
    ref = _checker()
    rng = random.Random(32)
    cases = []
    for _ in range(20):
        blocks, off, end = random_table_layout(rng, True)
        cases.append((ref.filter_block(blocks, off, end, 10, True),
                      [k for b in blocks for k in b] or [b"y" * 9], end))
    cases += [(b, [b"k" * 9], 1 << 16) for b in malformed_filter_blocks(rng, 200)]
    for blk, keys, end in cases:
        queries = [(rng.randrange(0, end + 5000),
                    rng.choice(keys) if rng.random() < 0.5 else rng.randbytes(rng.randrange(8, 20)))
                   for _ in range(16)]
        got = bl.filter_block_match_host(blk, queries, True)
        want = [ref.filter_matches(blk, o, k, True) for o, k in queries]
        assert [bool(x) for x in got] == want, blk


def test_filter_block_of_lcdb_table(bl, tmp_path):
    """Byte-identical to the filter block lcdb's table builder wrote, and
    every key present in the table matches its block's filter."""
    from test_bloom_oracle import lcdb_table_with_filter
    blocks, off, end, stored = lcdb_table_with_filter(tmp_path, entries=20000)
    assert bl.filter_block_host(blocks, off, end, 10, True) == stored
    queries = [(off[b], k) for b, keys in enumerate(blocks) for k in keys]
    assert bool(bl.filter_block_match_host(stored, queries, True).all())


def test_filter_block_device_fillseq_scale(bl):
    """A filter block over 65 536 data blocks of 36 internal fillseq keys
    (~150 MB of data offsets) on the device; checked against the C
    restatement (pinned above), then every key probed."""
    import torch
    ref = oracle.bloom_restatement()
    nb, per = 65536, 36
    rng = np.random.default_rng(3)
    sizes = rng.integers(2200, 2500, size=nb).astype(np.uint64)   # framed fillseq blocks
    off = np.zeros(nb, dtype=np.uint64)
    off[1:] = np.cumsum(sizes[:-1])
    end = int(off[-1] + sizes[-1])
    user = [b"%016d" % k for k in range(nb * per)]
    keys = [u + (k + 1).to_bytes(7, "little") + b"\x01" for k, u in enumerate(user)]
    blocks = [keys[b * per:(b + 1) * per] for b in range(nb)]
    want = ref.filter_block(blocks, off.tolist(), end, 10, True)
    buf = np.frombuffer(b"".join(keys) + b"\0" * 16, dtype=np.uint8)
    d_keys = torch.from_numpy(buf.copy()).cuda()
    d_koff = torch.arange(nb * per, dtype=torch.int64).cuda() * 24
    d_klen = torch.full((nb * per,), 24, dtype=torch.int32).cuda()
    d_first = (torch.arange(nb + 1, dtype=torch.int32) * per).cuda()
    d_boff = torch.from_numpy(off.astype(np.int64)).cuda()
    cap = bl.filter_block_bound(nb * per, nb, end, 10)
    d_out = torch.zeros(cap, dtype=torch.uint8).cuda()
    d_size = torch.zeros(1, dtype=torch.int64).cuda()
    d_scr = torch.empty(bl.filter_block_scratch(end), dtype=torch.uint8).cuda()
    bl.filter_block_build(d_keys, d_koff, d_klen, d_first, d_boff, end, 10, d_out, d_size, d_scr,
                          internal_keys=True)
    torch.cuda.synchronize()
    n = int(d_size.item())
    assert n == len(want)
    assert d_out[:n].cpu().numpy().tobytes() == want
    d_qoff = torch.repeat_interleave(d_boff, per)
    d_m = torch.zeros(nb * per, dtype=torch.uint8).cuda()
    bl.filter_block_match(d_out, n, d_qoff, d_keys, d_koff, d_klen, d_m, internal_keys=True)
    torch.cuda.synchronize()
    assert bool((d_m == 1).all())
