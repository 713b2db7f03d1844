"""Synthetic block corpora shaped like lcdb's db_bench workloads.

Wraps ``libcorpus.so`` (lcdb_amd/csrc/corpus.c).  The generator restates
db_bench's fillseq data (bench/db_bench.c:206-257, 975-1030) packed by the
block builder (src/table/block_builder.c:76-151, flush rule
table_builder.c:251-254) -- see the C file's header for the details.

Corpora are numpy arrays: ``buf`` (uint8), ``off`` (uint64), ``len`` (uint32).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
from dataclasses import dataclass

import numpy as np

from .build import CORPUS_LIB

_lib = None


def _corpus_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(CORPUS_LIB):
            raise ImportError(f"{CORPUS_LIB} missing (run the build)")
        _lib = C.CDLL(CORPUS_LIB)
        _lib.corpus_fillseq.restype = C.c_uint64
        _lib.corpus_fillseq.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                        C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_uint32]
        _lib.corpus_fillseq_shard.restype = C.c_uint64
        _lib.corpus_fillseq_shard.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                              C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                              C.c_uint32, C.c_uint32, C.c_uint32]
        _lib.corpus_random.restype = None
        _lib.corpus_random.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        _lib.corpus_ring.restype = C.c_void_p
        _lib.corpus_ring.argtypes = [C.POINTER(C.c_uint64)]
    return _lib


@dataclass
class Corpus:
    buf: np.ndarray   # uint8
    off: np.ndarray   # uint64
    len: np.ndarray   # uint32

    @property
    def n(self) -> int:
        return int(self.len.shape[0])

    def block(self, i: int) -> bytes:
        o = int(self.off[i])
        return self.buf[o:o + int(self.len[i])].tobytes()

    def blocks(self) -> list[bytes]:
        return [self.block(i) for i in range(self.n)]

    @property
    def raw_bytes(self) -> int:
        return int(self.len.sum(dtype=np.uint64))

    def sha256(self) -> str:
        """Digest of the concatenated block payloads (layout-independent)."""
        h = hashlib.sha256()
        for i in range(self.n):
            o = int(self.off[i])
            h.update(memoryview(self.buf[o:o + int(self.len[i])]))
        return h.hexdigest()


def fillseq(n: int, block_size: int = 4096, align: int = 16, key0: int = 0,
            ring0: int = 0, stride: int = 1, phase: int = 0) -> Corpus:
    """n data blocks of db_bench fillseq entries (16-B keys, 100-B values).

    With ``stride`` > 1, the round-robin shard ``phase`` of the stream: the
    blocks g of the unsharded stream with g % stride == phase."""
    per = block_size + block_size // 4 + 512
    cap = n * (per + align) + 64
    buf = np.zeros(cap, dtype=np.uint8)
    off = np.zeros(n, dtype=np.uint64)
    ln = np.zeros(n, dtype=np.uint32)
    used = _corpus_lib().corpus_fillseq_shard(buf.ctypes.data, cap, off.ctypes.data,
                                              ln.ctypes.data, n, block_size, align, key0, ring0,
                                              stride, phase)
    if n and used == 0:
        raise RuntimeError("corpus_fillseq failed")
    return Corpus(buf[:int(used) + 16], off, ln)


def random_blocks(n: int, size: int, seed: int = 0x5EED, align: int = 16) -> Corpus:
    """n blocks of `size` uniform random bytes (splitmix64 stream)."""
    stride = (size + align - 1) // align * align
    buf = np.zeros(n * stride + 16, dtype=np.uint8)
    data = np.empty(n * size, dtype=np.uint8)
    if n * size:
        _corpus_lib().corpus_random(data.ctypes.data, n * size, seed)
    for i in range(n):
        buf[i * stride:i * stride + size] = data[i * size:(i + 1) * size]
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    return Corpus(buf, off, np.full(n, size, dtype=np.uint32))


def concat(*parts: Corpus, align: int = 16) -> Corpus:
    """Concatenate corpora (block order preserved, offsets re-aligned)."""
    lens = np.concatenate([p.len for p in parts]) if parts else np.zeros(0, np.uint32)
    stride = (lens.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    off = np.zeros(len(lens), dtype=np.uint64)
    if len(lens):
        off[1:] = np.cumsum(stride[:-1])
    buf = np.zeros(int(stride.sum()) + 16, dtype=np.uint8)
    i = 0
    for p in parts:
        for j in range(p.n):
            o = int(p.off[j]); k = int(p.len[j])
            buf[int(off[i]):int(off[i]) + k] = p.buf[o:o + k]
            i += 1
    return Corpus(buf, off, lens.astype(np.uint32))


def mixed(scale: int = 1) -> Corpus:
    """Config C3: 4/16/64 KiB classes, half fillseq, half random (seed 0x5eed).

    ``scale`` multiplies the block counts (512 / 128 / 32 per half at 1)."""
    parts = []
    for bs, n in ((4096, 512), (16384, 128), (65536, 32)):
        parts.append(fillseq(n * scale, block_size=bs, key0=bs))
        parts.append(random_blocks(n * scale, bs, seed=0x5EED + bs))
    return concat(*parts)


def value_ring() -> bytes:
    n = C.c_uint64(0)
    p = _corpus_lib().corpus_ring(C.byref(n))
    return C.string_at(p, n.value)


def block_digests(buf: np.ndarray, off: np.ndarray, ln: np.ndarray) -> np.ndarray:
    """SHA-256 of every block, as an (n, 32) uint8 array (layout-independent)."""
    n = int(ln.shape[0])
    out = bytearray(32 * n)
    mv = memoryview(buf)
    sha = hashlib.sha256
    for i, (o, k) in enumerate(zip(off.tolist(), ln.tolist())):
        out[32 * i:32 * i + 32] = sha(mv[o:o + k]).digest()
    return np.frombuffer(bytes(out), dtype=np.uint8).reshape(n, 32)


def digest_of_digests(per_block: np.ndarray) -> str:
    """SHA-256 over the per-block SHA-256s in block order: the corpus digest
    that round-robin shards reassemble without moving the blocks
    (tests/golden/digests.json "*_dd" fields)."""
    return hashlib.sha256(np.ascontiguousarray(per_block).tobytes()).hexdigest()
