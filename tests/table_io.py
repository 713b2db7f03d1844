"""Test helpers for the block-framing rows (§8(f) 1-3): build .ldb files and
read their blocks with the REFERENCE's own table code (oracle/harness,
compiled by oracle/lcdb.mk), and parse what it returns."""
from __future__ import annotations

import os
import struct
import subprocess
from dataclasses import dataclass

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "lcdb")

LDB_OK, LDB_CORRUPTION, LDB_IOERR = 0, 30002, 30005     # include/lcdb.h:47-52

# Product / oracle status -> the reference's return code (format.c:162-270).
ST_TO_RC = {1: LDB_OK, 0: LDB_CORRUPTION, 4: LDB_CORRUPTION, 5: LDB_CORRUPTION, 3: LDB_IOERR}


def same_outcome(st: int, rc: int) -> bool:
    """Product/oracle status `st` vs the reference's ldb_read_block return.
    A read outside the file is LDB_IOERR through pread ("truncated block
    read", format.c:195-198) but the env's own errno (EINVAL) for offsets it
    refuses outright (env_unix_impl.h:1086-1097): both are the I/O class."""
    if st == 3:
        return rc == LDB_IOERR or 0 < rc < 30000
    return ST_TO_RC[st] == rc


def binary(name: str) -> str:
    p = os.path.join(BIN, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (make -C oracle -f lcdb.mk, needs /root/reference)")
    return p


def build_table(tmp, entries: int, block_size: int, kind: str = "cpu", bloom_bits: int = 0) -> str:
    """An .ldb of db_bench fillseq entries written by lcdb's own builder
    (with its filter block when bloom_bits > 0)."""
    d = os.path.join(str(tmp), f"db_{kind}_{entries}_{block_size}_{bloom_bits}")
    args = [binary(f"build_table.{kind}"), d, str(entries), str(block_size)]
    if bloom_bits:
        args.append(str(bloom_bits))
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "rc=0" in r.stdout, r.stdout + r.stderr
    return os.path.join(d, "000001.ldb")


@dataclass
class Dump:
    file_size: int
    metaindex: tuple[int, int]
    index: tuple[int, int]
    off: np.ndarray          # uint64
    size: np.ndarray         # uint64
    rc: list[int]
    contents: list[bytes]    # b"" unless rc == LDB_OK

    @property
    def n(self) -> int:
        return len(self.rc)


def dump_blocks(path: str, out: str, verify: bool, handles=None) -> Dump:
    """ldb_read_block (format.c:162-270) on every block, by the reference."""
    args = [binary("dump_blocks.cpu"), path, out, "1" if verify else "0"]
    if handles is not None:
        hp = out + ".handles"
        np.asarray(handles, dtype=np.uint64).reshape(-1, 2).tofile(hp)
        args.append(hp)
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stderr)
    b = open(out, "rb").read()
    fsz, mo, ms, io_, is_ = struct.unpack_from("<5Q", b, 0)
    (count,) = struct.unpack_from("<I", b, 40)
    at = 44
    off, size, rc, contents = [], [], [], []
    for _ in range(count):
        o, s, c, ln = struct.unpack_from("<QQiI", b, at)
        at += 24
        off.append(o)
        size.append(s)
        rc.append(c)
        contents.append(b[at:at + ln])
        at += ln
    return Dump(fsz, (mo, ms), (io_, is_), np.array(off, dtype=np.uint64),
                np.array(size, dtype=np.uint64), rc, contents)


def corrupt(data: bytes, lo: int, hi: int, count: int, seed: int) -> bytes:
    """Flip `count` seeded bytes of data[lo:hi)."""
    rng = np.random.default_rng(seed)
    b = bytearray(data)
    for p in rng.integers(lo, hi, size=count):
        b[int(p)] ^= int(rng.integers(1, 256))
    return bytes(b)


def _varint(b: bytes, at: int, limit: int, bits: int):
    """coding.h varint32/64 read: (value, next) or None."""
    v, sh = 0, 0
    while at < limit and sh <= bits - 1:
        c = b[at]
        at += 1
        v |= (c & 0x7F) << sh
        if c < 0x80:
            return v, at
        sh += 7
    return None


def block_entries(contents: bytes) -> list[tuple[bytes, bytes]]:
    """A block's (key, value) entries in order, as lcdb's block iterator
    walks them from the first restart (block.c:49-130, 255-297).  Test
    helper: asserts on malformed blocks."""
    n = len(contents)
    assert n >= 4
    nr = struct.unpack_from("<I", contents, n - 4)[0]
    assert nr <= (n - 4) // 4
    limit = n - (1 + nr) * 4
    out, key, at = [], b"", 0
    while at < limit:
        if limit - at >= 3 and max(contents[at:at + 3]) < 128:
            shared, non_shared, vlen = contents[at], contents[at + 1], contents[at + 2]
            at += 3
        else:
            shared, at = _varint(contents, at, limit, 32)
            non_shared, at = _varint(contents, at, limit, 32)
            vlen, at = _varint(contents, at, limit, 32)
        assert shared <= len(key) and at + non_shared + vlen <= limit
        key = key[:shared] + contents[at:at + non_shared]
        at += non_shared
        out.append((key, contents[at:at + vlen]))
        at += vlen
    return out


def filter_handle(metaindex: bytes, name: bytes = b"filter.leveldb.BuiltinBloomFilter2"):
    """(offset, size) of the filter block named in a metaindex block
    (table.c:78-120), or None."""
    for k, v in block_entries(metaindex):
        if k == name:
            off, at = _varint(v, 0, len(v), 64)
            size, _ = _varint(v, at, len(v), 64)
            return off, size
    return None


def entry_offsets(contents: bytes) -> list[int]:
    """Start offset of every entry of a well-formed block, in order."""
    n = len(contents)
    nr = struct.unpack_from("<I", contents, n - 4)[0]
    limit = n - (1 + nr) * 4
    out, at = [], 0
    while at < limit:
        out.append(at)
        shared, at2 = _varint(contents, at, limit, 32)
        non_shared, at2 = _varint(contents, at2, limit, 32)
        vlen, at2 = _varint(contents, at2, limit, 32)
        at = at2 + non_shared + vlen
    return out


def with_raw_index(file: bytes, index_off: int, metaindex, contents: bytes) -> bytes:
    """The table file with its index block replaced by `contents`, stored raw
    (type 0, masked CRC32C trailer, table_builder.c:123-153) at the old
    index offset, and a footer pointing at it (format.c:92-106)."""
    import oracle

    def v(x):
        out = bytearray()
        while x >= 128:
            out.append((x & 127) | 128)
            x >>= 7
        out.append(x)
        return bytes(out)
    crc = oracle.crc32c_mask(oracle.crc32c(b"\x00", oracle.crc32c(contents)))
    block = contents + b"\x00" + crc.to_bytes(4, "little")
    handles = v(metaindex[0]) + v(metaindex[1]) + v(index_off) + v(len(contents))
    footer = handles + b"\x00" * (40 - len(handles)) + (0xdb4775248b80fb57).to_bytes(8, "little")
    return file[:index_off] + block + footer
