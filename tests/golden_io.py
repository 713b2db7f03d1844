"""Reader/writer for tests/golden/vectors.bin (fixture container).

Format (little-endian):
    magic  b"LGSGOLD1"
    u32    record count
    per record:
        u8   kind        0 = encode vector (a = raw input, b = expected stream)
                         1 = decode vector (a = stream, ok = expected result,
                             b = expected output when ok)
        u16  name length, name (utf-8)
        u32  len(a), a
        u8   ok
        u32  len(b), b
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

MAGIC = b"LGSGOLD1"
GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
VECTORS = os.path.join(GOLDEN_DIR, "vectors.bin")
DIGESTS = os.path.join(GOLDEN_DIR, "digests.json")


@dataclass
class Vector:
    kind: int
    name: str
    a: bytes
    ok: int
    b: bytes


def write(path: str, vecs: list[Vector]) -> None:
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<I", len(vecs)))
        for v in vecs:
            nm = v.name.encode()
            f.write(struct.pack("<BH", v.kind, len(nm)))
            f.write(nm)
            f.write(struct.pack("<I", len(v.a)))
            f.write(v.a)
            f.write(struct.pack("<BI", v.ok, len(v.b)))
            f.write(v.b)


def read(path: str = VECTORS) -> list[Vector]:
    with open(path, "rb") as f:
        data = f.read()
    assert data[:8] == MAGIC, "bad golden file"
    (n,) = struct.unpack_from("<I", data, 8)
    at = 12
    out = []
    for _ in range(n):
        kind, nl = struct.unpack_from("<BH", data, at)
        at += 3
        name = data[at:at + nl].decode()
        at += nl
        (la,) = struct.unpack_from("<I", data, at)
        at += 4
        a = data[at:at + la]
        at += la
        ok, lb = struct.unpack_from("<BI", data, at)
        at += 5
        b = data[at:at + lb]
        at += lb
        out.append(Vector(kind, name, a, ok, b))
    return out
