"""The oracle (CPU restatement, oracle/snappy_oracle.c) pinned against the
reference: its own known answers (test/t-snappy.c) and the golden vectors the
compiled reference produced (tests/golden/make_golden.py)."""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import oracle
from lcdb_amd import corpus


@pytest.fixture(scope="module")
def orc():
    return oracle.restatement()


def test_ramp_known_answer(orc, digests):
    # t-snappy.c:24-53: 1 MiB of i & 0xff encodes to exactly 53203 bytes.
    data = bytes(i & 0xFF for i in range(1 << 20))
    enc = orc.encode(data)
    assert len(enc) == 53203
    assert hashlib.sha256(enc).hexdigest() == digests["ramp_1MiB"]["comp_sha256"]
    assert orc.decode_size(enc) == len(data)
    assert orc.decode(enc) == data


def test_golden_vectors(orc, vectors):
    n_enc = n_dec = n_rej = 0
    for v in vectors:
        if v.kind == 0:
            assert orc.encode(v.a) == v.b, v.name
            assert orc.decode(v.b) == v.a, v.name
            n_enc += 1
        else:
            out = orc.decode(v.a)
            assert (out is not None) == bool(v.ok), v.name
            if v.ok:
                assert out == v.b, v.name
            n_dec += 1
            n_rej += 0 if v.ok else 1
    assert n_enc > 250 and n_dec > 400 and n_rej > 100, (n_enc, n_dec, n_rej)


def test_twain_roundtrip_and_golang_stream(orc, vectors):
    # t-snappy.c:56-99
    by = {v.name: v for v in vectors}
    tw = by["twain/encode"]
    assert len(tw.a) == 14168 and len(tw.b) < len(tw.a)
    assert orc.decode(tw.b) == tw.a
    go = by["twain/golang-rawsnappy"]
    assert go.ok and orc.decode(go.a) == tw.a


def test_encode_size_bound(orc):
    # snappy.c:347-362
    assert orc.encode_size(0) == 32
    assert orc.encode_size(4096) == 32 + 4096 + 4096 // 6
    assert orc.encode_size(0x7FFFFFFF) is None
    assert orc.encode_size(1 << 40) is None


def test_corpus_digest_c1(orc, digests):
    d = digests["C1_fillseq_1024x4KiB"]
    c = corpus.fillseq(1024)
    assert c.sha256() == d["raw_sha256"]
    out, ooff, olen = orc.encode_batch(c.buf, c.off, c.len, threads=4)
    h = hashlib.sha256()
    for o, k in zip(ooff, olen):
        h.update(memoryview(out[int(o):int(o) + int(k)]))
    assert h.hexdigest() == d["comp_sha256"]
    assert int(olen.sum(dtype=np.uint64)) == d["comp_bytes"]


@pytest.mark.slow
def test_corpus_digest_c3_mixed(orc, digests):
    d = digests["C3_mixed"]
    c = corpus.mixed()
    assert c.sha256() == d["raw_sha256"]
    out, ooff, olen = orc.encode_batch(c.buf, c.off, c.len, threads=4)
    h = hashlib.sha256()
    for o, k in zip(ooff, olen):
        h.update(memoryview(out[int(o):int(o) + int(k)]))
    assert h.hexdigest() == d["comp_sha256"]


@pytest.mark.slow
def test_corpus_digest_c3_mixed_x32(orc, digests):
    # The C3 mix at the scale bench.py times (43 008 blocks, 403 MB): the
    # restatement reproduces the reference's per-block digests, which bench.py
    # diffs the GPU's compressed blocks against.
    d = digests["C3_mixed_x32"]
    c = corpus.mixed(32)
    assert c.n == d["blocks"] and c.raw_bytes == d["raw_bytes"]
    out, ooff, olen = orc.encode_batch(c.buf, c.off, c.len, threads=8)
    assert int(olen.sum(dtype=np.uint64)) == d["comp_bytes"]
    assert corpus.digest_of_digests(corpus.block_digests(out, ooff, olen)) == d["comp_dd"]
