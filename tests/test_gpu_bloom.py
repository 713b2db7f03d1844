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
