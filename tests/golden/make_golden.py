#!/usr/bin/env python3
"""Generate tests/golden/{vectors.bin,digests.json} from the REFERENCE codec.

Run in the build container, where /root/reference exists and
oracle/_ref/libref_snappy.so has been compiled from the reference's own
src/util/snappy.c (oracle/Makefile).  Every expected output below is what
lcdb's encoder/decoder itself produced; nothing is computed by our code.

Inputs:
  * the reference's test data (test/data/snappy_data.h: the Mark Twain text
    and golang's .rawsnappy of it, t-snappy.c:82-99), parsed from the header;
  * db_bench-shaped fillseq blocks and splitmix64 random blocks from
    lcdb_amd.corpus (the synthetic workload of BASELINE.json);
  * hand-made edge cases (tiny inputs, all-zero, 64 KiB chunk boundaries,
    every literal/copy tag form, COPY4, overlapping copies) and seeded
    corruptions of valid streams (bit flips, truncations, garbage), each
    with the reference's accept/reject bit.
Large corpora are pinned by SHA-256 digests (digests.json), not bytes.

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from golden_io import DIGESTS, VECTORS, Vector, write  # noqa: E402
from lcdb_amd import corpus  # noqa: E402

REF_DATA = "/root/reference/test/data/snappy_data.h"


def parse_c_array(text: str, name: str) -> bytes:
    m = re.search(r"%s\[\]\s*=\s*\{(.*?)\};" % re.escape(name), text, re.S)
    return bytes(int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{2})", m.group(1)))


def varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def main() -> None:
    ref = oracle.reference()
    if ref is None:
        sys.exit("oracle/_ref/libref_snappy.so missing: run `make -C oracle` here first")
    rng = random.Random(0x6C636462)
    vecs: list[Vector] = []

    def enc(name: str, raw: bytes) -> bytes:
        comp = ref.encode(raw)
        assert ref.decode(comp) == raw, name
        vecs.append(Vector(0, name, raw, 1, comp))
        return comp

    def dec(name: str, stream: bytes) -> None:
        out = ref.decode(stream)
        vecs.append(Vector(1, name, stream, 1 if out is not None else 0, out or b""))

    # -- reference test data (t-snappy.c) --
    text = open(REF_DATA).read()
    twain = parse_c_array(text, "snappy_test_input")
    golang = parse_c_array(text, "snappy_test_output")
    assert len(twain) == 14168 and len(golang) == 9871
    enc("twain/encode", twain)
    dec("twain/golang-rawsnappy", golang)

    # -- fillseq blocks (4 KiB, plus a later region of the key space) --
    c = corpus.fillseq(48)
    for i in range(c.n):
        enc(f"fillseq4k/{i}", c.block(i))
    c = corpus.fillseq(8, key0=5_000_000, ring0=700_000)
    for i in range(c.n):
        enc(f"fillseq4k-far/{i}", c.block(i))
    for bs in (256, 1024, 16384, 65536):
        c = corpus.fillseq(2, block_size=bs, key0=1000)
        for i in range(c.n):
            enc(f"fillseq{bs}/{i}", c.block(i))

    # -- random blocks (incompressible) --
    for i, size in enumerate((4096, 4096, 4096, 16384, 65536)):
        enc(f"random/{size}/{i}", corpus.random_blocks(1, size, seed=0x5EED + i).block(0))

    # -- tiny inputs, every length around MIN_BLOCK_SIZE (snappy.c:27,377) --
    for n in range(0, 41):
        enc(f"tiny/zero/{n}", bytes(n))
        enc(f"tiny/rand/{n}", bytes(rng.randrange(256) for _ in range(n)))
        enc(f"tiny/ramp/{n}", bytes(i & 0xFF for i in range(n)))
        enc(f"tiny/ab/{n}", (b"ab" * 40)[:n])

    # -- all-zero and near-zero blocks (exercise the 64-bit re-match compare,
    #    snappy.c:182: it succeeds only when the 3 bytes after the 4 match) --
    for n in (17, 18, 100, 4096, 65535, 65536, 65537, 70000):
        enc(f"zeros/{n}", bytes(n))
    for k in range(6):
        b = bytearray(4096)
        for j in range(0, 4096, rng.choice([5, 7, 8, 9, 13, 64])):
            b[j] = rng.randrange(1, 256)
        enc(f"sparse/{k}", bytes(b))
    for k in range(6):
        unit = bytes(rng.randrange(256) for _ in range(rng.choice([1, 2, 3, 4, 5, 6, 7, 8, 11])))
        pad = bytes(rng.choice([0, 0, 0, 1]) for _ in range(rng.choice([0, 1, 2, 3, 4])))
        enc(f"period/{k}", ((unit + pad) * 2000)[:4000 + k * 37])

    # -- text-like and mixed data --
    words = twain.split()[:3000]
    for k in range(4):
        s = b" ".join(rng.choice(words) for _ in range(900 + 300 * k))
        enc(f"words/{k}", s)

    # -- 64 KiB chunk boundaries and multi-chunk inputs (snappy.c:370-381) --
    big = corpus.fillseq(40, block_size=4096, key0=77)
    blob = b"".join(big.blocks())
    for n in (65535, 65536, 65537, 65536 + 16, 65536 + 17, 131072, 131072 + 5, 150001):
        enc(f"multichunk/{n}", blob[:n])
    enc("multichunk/twain-x6", twain * 6)

    # -- hand-made decode streams: every tag form and reject condition --
    def lit(data: bytes) -> bytes:
        m = len(data) - 1
        if m < 60:
            return bytes([m << 2]) + data
        if m < 256:
            return bytes([60 << 2, m]) + data
        if m < 65536:
            return bytes([61 << 2, m & 255, m >> 8]) + data
        return bytes([62 << 2, m & 255, (m >> 8) & 255, m >> 16]) + data

    def c1(dist, ln):
        return bytes([((dist >> 8) << 5) | ((ln - 4) << 2) | 1, dist & 255])

    def c2(dist, ln):
        return bytes([((ln - 1) << 2) | 2, dist & 255, dist >> 8])

    def c4(dist, ln):
        return bytes([((ln - 1) << 2) | 3]) + dist.to_bytes(4, "little")

    hello = b"hello, snappy world"
    cases = {
        "empty": b"",
        "hdr-only-zero": b"\x00",
        "hdr-zero-extra": b"\x00\x00",
        "hdr-5cont": b"\x80\x80\x80\x80\x80",
        "hdr-5max": b"\xff\xff\xff\xff\x07",
        "hdr-5big": b"\xff\xff\xff\xff\x0f",
        "hdr-trunc": b"\x80",
        "lit-ok": varint(len(hello)) + lit(hello),
        "lit-short": varint(len(hello) + 1) + lit(hello),
        "lit-long": varint(len(hello) - 1) + lit(hello),
        "lit-trunc": varint(len(hello)) + lit(hello)[:-1],
        "lit60": varint(100) + lit(bytes(range(100))),
        "lit61": varint(300) + lit(bytes(i & 255 for i in range(300))),
        "lit62": varint(70000) + lit(bytes(i * 7 & 255 for i in range(70000))),
        "lit60-trunc-hdr": varint(100) + bytes([60 << 2]),
        "lit61-trunc-hdr": varint(100) + bytes([61 << 2, 5]),
        "lit62-trunc-hdr": varint(100) + bytes([62 << 2, 5, 0]),
        "lit63-trunc-hdr": varint(100) + bytes([63 << 2, 5, 0, 0]),
        "lit63-huge": varint(100) + bytes([63 << 2, 0xFF, 0xFF, 0xFF, 0x7F]) + b"x" * 8,
        "lit63-max": varint(100) + bytes([63 << 2, 0xFE, 0xFF, 0xFF, 0x7F]) + b"x" * 8,
        "lit63-small": varint(3) + bytes([63 << 2, 2, 0, 0, 0]) + b"abc",
        "c1-ok": varint(12) + lit(b"abcd") + c1(4, 8),
        "c1-dist0": varint(12) + lit(b"abcd") + c1(0, 8),
        "c1-far": varint(12) + lit(b"abcd") + c1(5, 8),
        "c1-trunc": varint(12) + lit(b"abcd") + c1(4, 8)[:1],
        "c1-over": varint(10) + lit(b"abcd") + c1(4, 8),
        "c2-ok": varint(68) + lit(b"abcd") + c2(4, 64),
        "c2-len1": varint(5) + lit(b"abcd") + c2(2, 1),
        "c2-trunc": varint(68) + lit(b"abcd") + c2(4, 64)[:2],
        "c2-dist0": varint(68) + lit(b"abcd") + c2(0, 64),
        "c4-ok": varint(40) + lit(b"0123456789") + c4(10, 30),
        "c4-far": varint(40) + lit(b"0123456789") + c4(11, 30),
        "c4-neg": varint(40) + lit(b"0123456789") + c4(0x80000000, 30),
        "c4-trunc": varint(40) + lit(b"0123456789") + c4(10, 30)[:4],
        "c4-len64": varint(74) + lit(b"0123456789") + c4(3, 64),
        "tag-then-nothing": varint(4) + lit(b"abcd") + b"\x01",
        "underfill": varint(9) + lit(b"abcd") + c1(4, 4),
        "zero-want-lit": b"\x00" + lit(b"a"),
    }
    for d in range(1, 12):
        cases[f"overlap/d{d}"] = varint(d + 64) + lit(bytes(range(65, 65 + d))) + c2(d, 64)
        cases[f"overlap1/d{d}"] = varint(d + 11) + lit(bytes(range(97, 97 + d))) + c1(d, 11)
    chain = lit(b"xyz")
    for _ in range(60):
        chain += c1(3, 7)
    cases["rle-chain"] = varint(3 + 60 * 7) + chain
    for name, s in cases.items():
        dec(f"craft/{name}", s)

    # -- seeded corruptions of valid streams --
    bases = [ref.encode(corpus.fillseq(1).block(0)[:n]) for n in (64, 200, 700, 2000)]
    bases.append(ref.encode(twain[:1500]))
    for bi, base in enumerate(bases):
        for t in range(40):
            b = bytearray(base)
            for _ in range(rng.choice([1, 1, 2, 3])):
                p = rng.randrange(len(b))
                b[p] ^= 1 << rng.randrange(8)
            dec(f"flip/{bi}/{t}", bytes(b))
        for t in range(15):
            dec(f"trunc/{bi}/{t}", base[:rng.randrange(len(base))])
        for t in range(10):
            b = bytearray(base)
            p = rng.randrange(1, len(b))
            b[p:p] = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 4)))
            dec(f"insert/{bi}/{t}", bytes(b))
    for t in range(60):
        n = rng.randrange(0, 300)
        body = bytes(rng.randrange(256) for _ in range(n))
        dec(f"garbage/{t}", varint(rng.randrange(0, 600)) + body)

    write(VECTORS, vecs)

    make_digests(ref)
    print(f"{len(vecs)} vectors, {os.path.getsize(VECTORS)} bytes")


C5_ENTRIES = 32768000      # db_bench fillseq entries -> a 2.0 GiB .ldb


def c5_table() -> dict:
    """BASELINE config 5: the .ldb lcdb's own src/builder.c writes for
    C5_ENTRIES fillseq entries with lcdb's own snappy.c (build_table.cpu,
    oracle/lcdb.mk), pinned by size and SHA-256; plus its index block, which
    at this size is tens of MiB (the multi-chunk drop-in encode, snappy.c:
    370-374, and an over-slot decode on re-open, builder.c:99)."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "oracle", "_ref", "lcdb", "build_table.cpu")
    with tempfile.TemporaryDirectory() as tmp:
        r = subprocess.run([exe, os.path.join(tmp, "db"), str(C5_ENTRIES), "4096"],
                           capture_output=True, text=True, check=True)
        assert "rc=0" in r.stdout, r.stdout
        path = os.path.join(tmp, "db", "000001.ldb")
        h = hashlib.sha256()
        with open(path, "rb") as f:
            for piece in iter(lambda: f.read(1 << 24), b""):
                h.update(piece)
            size = f.tell()
            f.seek(size - 48)
            foot = f.read(48)
    vals, i = [], 0
    for _ in range(4):                       # footer: metaindex + index handles
        v = sh = 0
        while True:
            c = foot[i]
            i += 1
            v |= (c & 0x7F) << sh
            sh += 7
            if c < 0x80:
                break
        vals.append(v)
    return {"entries": C5_ENTRIES, "block_size": 4096, "file_size": size,
            "sha256": h.hexdigest(), "index_block_offset": vals[2],
            "index_block_stored_bytes": vals[3]}


def digest(ref, c: corpus.Corpus, threads: int = 8, concat: bool = True) -> dict:
    """The reference's compressed output of corpus c, as digests."""
    out, ooff, olen = ref.encode_batch(c.buf, c.off, c.len, threads=threads)
    d = {"blocks": c.n, "raw_bytes": c.raw_bytes,
         "comp_bytes": int(olen.sum(dtype=np.uint64)),
         "raw_dd": corpus.digest_of_digests(corpus.block_digests(c.buf, c.off, c.len)),
         "comp_dd": corpus.digest_of_digests(corpus.block_digests(out, ooff, olen))}
    if concat:
        h = hashlib.sha256()
        for o, k in zip(ooff, olen):
            h.update(memoryview(out[int(o):int(o) + int(k)]))
        d.update(raw_sha256=c.sha256(), comp_sha256=h.hexdigest())
    return d


def make_digests(ref) -> None:
    """Digests of the BASELINE.json corpora (reference outputs).

    ``*_sha256``: SHA-256 of the concatenated blocks; ``*_dd``: SHA-256 of the
    concatenated per-block SHA-256s (lcdb_amd.corpus.digest_of_digests), which
    round-robin shards reassemble without moving blocks (bench.py at N > 1).
    C4 (1 048 576 blocks, BASELINE.json configs[3]) is pinned by its _dd
    digests only.  C3_mixed_x32 is the mix at the scale bench.py times."""

    ramp = ref.encode(bytes(i & 255 for i in range(1 << 20)))
    digs = {
        "C1_fillseq_1024x4KiB": digest(ref, corpus.fillseq(1024)),
        "C2_fillseq_65536x4KiB": digest(ref, corpus.fillseq(65536)),
        "C3_mixed": digest(ref, corpus.mixed()),
        "C3_mixed_x32": digest(ref, corpus.mixed(32)),
        "C4_fillseq_1048576x4KiB": digest(ref, corpus.fillseq(1048576), concat=False),
        "ramp_1MiB": {"raw_bytes": 1 << 20, "comp_bytes": len(ramp),
                      "comp_sha256": hashlib.sha256(ramp).hexdigest()},
        "C5_table_2GiB": c5_table(),
        "_generator": "tests/golden/make_golden.py with oracle/_ref/libref_snappy.so "
                      "(lcdb src/util/snappy.c compiled unmodified)",
    }
    with open(DIGESTS, "w") as f:
        json.dump(digs, f, indent=2, sort_keys=True)
    print("digests: " + ", ".join(k for k in digs if not k.startswith("_")))

if __name__ == "__main__":
    if "--digests-only" in sys.argv:
        import oracle
        make_digests(oracle.reference())
    elif "--add-c3x32" in sys.argv:
        # merge one digest into the pinned file without re-running the rest
        import oracle
        with open(DIGESTS) as f:
            digs = json.load(f)
        digs["C3_mixed_x32"] = digest(oracle.reference(), corpus.mixed(32))
        with open(DIGESTS, "w") as f:
            json.dump(digs, f, indent=2, sort_keys=True)
    else:
        main()
