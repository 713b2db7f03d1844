"""Block framing oracle (oracle/table_oracle.c), pinned (CPU only):

* CRC32C against the known answers of the reference's test/t-crc32c.c and
  against lcdb's own crc32c.c compiled unmodified (oracle/_ref);
* the data-block write restatement against .ldb files written by lcdb's own
  table builder (src/builder.c -> table_builder.c);
* the block read restatement against lcdb's own ldb_read_block (format.c),
  on intact, corrupted and truncated inputs (oracle/harness/dump_blocks.c).
"""
from __future__ import annotations

import random

import numpy as np
import pytest

import oracle
import table_io
from table_io import LDB_OK

RFC3720 = bytes([
    0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00,
    0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18, 0x28, 0x00, 0x00, 0x00,
    0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00])

# test/t-crc32c.c:39-54, 108 (RFC 3720 B.4 and the 1 MiB + 17 test).
KNOWN = [
    (bytes(32), 0x8a9136aa),
    (b"\xff" * 32, 0x62a8ab43),
    (bytes(range(32)), 0x46dd794e),
    (bytes(range(31, -1, -1)), 0x113fdb5c),
    (RFC3720, 0xd9963a56),
    (b"\xaa" * ((1 << 20) + 17), 0xb0d7025a),
]


@pytest.mark.parametrize("data,want", KNOWN, ids=[f"known{i}" for i in range(len(KNOWN))])
def test_crc32c_known_answers(data, want):
    assert oracle.crc32c(data) == want
    ref = oracle.reference_crc32c()
    if ref is not None:
        buf = np.frombuffer(data + b"\0", dtype=np.uint8)
        assert ref.ldb_crc32c_extend(0, buf.ctypes.data, len(data)) == want


def test_crc32c_extend_and_mask():
    # t-crc32c.c:114-135
    assert oracle.crc32c(b"a") != oracle.crc32c(b"foo")
    assert oracle.crc32c(b"hello world") == oracle.crc32c(b"world", oracle.crc32c(b"hello "))
    c = oracle.crc32c(b"foo")
    assert c != oracle.crc32c_mask(c)
    assert c != oracle.crc32c_mask(oracle.crc32c_mask(c))
    assert c == oracle.crc32c_unmask(oracle.crc32c_mask(c))
    assert c == oracle.crc32c_unmask(oracle.crc32c_unmask(oracle.crc32c_mask(oracle.crc32c_mask(c))))


def test_crc32c_vs_reference_random():
    ref = oracle.reference_crc32c()
    if ref is None:
        pytest.skip("oracle/_ref/libref_crc32c.so not built")
    rng = random.Random(0xc5c)
    for _ in range(300):
        n = rng.choice([rng.randrange(0, 40), rng.randrange(40, 9000), rng.randrange(60000, 70000)])
        data = rng.randbytes(n)
        init = rng.choice([0, rng.getrandbits(32)])
        buf = np.frombuffer(data + b"\0", dtype=np.uint8)
        assert oracle.crc32c(data, init) == ref.ldb_crc32c_extend(init, buf.ctypes.data, n)


@pytest.fixture(scope="module")
def tables(tmp_path_factory):
    """Reference-built .ldb files: (path, file bytes, dump with checksums)."""
    tmp = tmp_path_factory.mktemp("ldb")
    out = {}
    for entries, bs in [(6000, 4096), (1500, 256), (9000, 65536)]:
        path = table_io.build_table(tmp, entries, bs)
        d = table_io.dump_blocks(path, str(tmp / f"dump_{bs}.bin"), verify=True)
        out[bs] = (path, open(path, "rb").read(), d)
    return out


def _check_reads(file: bytes, d, verify: bool):
    for i in range(d.n):
        cap = max(len(d.contents[i]), 1 << 17)
        st, got = oracle.table_read_block(file, int(d.off[i]), int(d.size[i]), verify, cap)
        assert table_io.same_outcome(st, d.rc[i]), (i, st, d.rc[i])
        if d.rc[i] == LDB_OK:
            assert got == d.contents[i], i


@pytest.mark.parametrize("bs", [4096, 256, 65536])
def test_read_block_matches_reference(tables, bs):
    path, file, d = tables[bs]
    assert all(rc == LDB_OK for rc in d.rc)
    _check_reads(file, d, verify=True)


@pytest.mark.parametrize("bs", [4096, 256, 65536])
def test_write_blocks_reproduces_reference_file(tables, bs):
    # Re-frame the reference's decoded data blocks: the bytes and handles of
    # the whole data region must come out identical to lcdb's own writer.
    path, file, d = tables[bs]
    ndata = d.n - 2                                    # minus metaindex, index
    region, hoff, hsize, end = oracle.table_write_blocks(d.contents[:ndata], 1, 0)
    assert end == d.metaindex[0]
    assert region == file[:end]
    assert np.array_equal(hoff, d.off[:ndata]) and np.array_equal(hsize, d.size[:ndata])


@pytest.mark.parametrize("verify", [True, False])
def test_read_block_corrupted_matches_reference(tables, tmp_path, verify):
    path, file, d = tables[4096]
    data_end = d.metaindex[0]
    for seed in range(3):
        bad = table_io.corrupt(file, 0, data_end, 40, seed)
        p = tmp_path / f"bad{seed}.ldb"
        p.write_bytes(bad)
        # The handles of the intact file, read from the corrupted one.
        handles = np.stack([d.off, d.size], axis=1)
        dd = table_io.dump_blocks(str(p), str(tmp_path / f"d{seed}.bin"), verify, handles)
        assert any(rc != LDB_OK for rc in dd.rc) or not verify
        _check_reads(bad, dd, verify)


def test_read_block_bad_handles_match_reference(tables, tmp_path):
    path, file, d = tables[256]
    n = len(file)
    handles = [(0, n), (n - 4, 0), (n - 5, 0), (n, 0), (n + 10, 3), (int(d.off[1]), int(d.size[1]) + 1),
               (int(d.off[2]) + 1, int(d.size[2])), (1, 2), (0, 0), (2**64 - 100, 50),
               (5, 2**64 - 3)]
    dd = table_io.dump_blocks(path, str(tmp_path / "h.bin"), True, handles)
    _check_reads(file, dd, True)
