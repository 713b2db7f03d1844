"""lcdb's bloom filter on the GPU.

Python face of the batched C ABI (``include/lcdb_gpu_snappy.h``):

* ``build_host(groups, bits_per_key)``: one filter per key group, each byte
  for byte what ``ldb_bloom_build`` appends (src/util/bloom.c:102-119);
* ``match_host(filters, queries)``: ``ldb_bloom_match`` per (filter, key)
  (bloom.c:121-165);
* ``build`` / ``match`` on device tensors (int64 offsets, int32 lengths);
* ``filter_block_host(blocks, block_off, data_end)``: a table's filter block
  as lcdb's table builder writes it (src/table/filter_block.c:79-150), and
  ``filter_block_match_host(block, queries)``: ``ldb_filter_matches``
  (filter_block.c:170-225); ``filter_block_build`` / ``filter_block_match``
  on device tensors.

Everything runs through ``liblcdb_gpu_snappy.so``; there is no CPU fallback.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import _native
from ._native import check
from .snappy import _stream_ptr

_L = _native.lib()

__all__ = ["filter_size", "build_host", "match_host", "build", "match", "filter_block_bound",
           "filter_block_scratch", "filter_block_host", "filter_block_match_host",
           "filter_block_build", "filter_block_match"]


def filter_size(nkeys: int, bits_per_key: int = 10) -> int:
    """Bytes of the filter for nkeys keys (0 for an empty filter)."""
    return int(_L.lgs_bloom_filter_size(nkeys, bits_per_key))


def _pack(items: Sequence[bytes]):
    lens = np.array([len(b) for b in items], dtype=np.uint32)
    offs = np.zeros(len(items), dtype=np.uint64)
    if len(items):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(items) + b"\0" * 16, dtype=np.uint8)
    return buf, offs, lens


def build_host(groups: Sequence[Sequence[bytes]], bits_per_key: int = 10) -> list[bytes]:
    """One filter per group of keys (an empty group gives b"")."""
    keys = [k for g in groups for k in g]
    first = np.zeros(len(groups) + 1, dtype=np.uint32)
    first[1:] = np.cumsum([len(g) for g in groups], dtype=np.uint64)
    buf, offs, lens = _pack(keys)
    sizes = [filter_size(len(g), bits_per_key) for g in groups]
    ooff = np.zeros(len(groups), dtype=np.uint64)
    if len(groups):
        ooff[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    out = np.zeros(int(sum(sizes)) + 1, dtype=np.uint8)
    check(_L.lgs_bloom_build_host(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                  first.ctypes.data, len(groups), bits_per_key, out.ctypes.data,
                                  ooff.ctypes.data),
          "lgs_bloom_build_host")
    return [out[int(o):int(o) + s].tobytes() for o, s in zip(ooff, sizes)]


def match_host(filters: Sequence[bytes], queries: Sequence[tuple[int, bytes]]) -> np.ndarray:
    """uint8 array: 1 where the key may be in its filter."""
    fbuf, foff, flen = _pack(filters)
    kbuf, koff, klen = _pack([k for _, k in queries])
    qf = np.array([f for f, _ in queries], dtype=np.uint32)
    m = np.zeros(len(queries), dtype=np.uint8)
    check(_L.lgs_bloom_match_host(fbuf.ctypes.data, foff.ctypes.data, flen.ctypes.data,
                                  len(filters), qf.ctypes.data, kbuf.ctypes.data,
                                  koff.ctypes.data, klen.ctypes.data, len(queries),
                                  m.ctypes.data),
          "lgs_bloom_match_host")
    return m


def build(d_keys, d_key_off, d_key_len, d_first, bits_per_key, d_out, d_out_off, stream=None):
    """Asynchronously build int(d_first.numel()) - 1 filters on the device."""
    n = int(d_first.numel()) - 1
    check(_L.lgs_bloom_build_dev(d_keys.data_ptr(), d_key_off.data_ptr(), d_key_len.data_ptr(),
                                 d_first.data_ptr(), n, bits_per_key, d_out.data_ptr(),
                                 d_out_off.data_ptr(), _stream_ptr(stream)),
          "lgs_bloom_build_dev")


def match(d_filters, d_filter_off, d_filter_len, d_query_filter, d_keys, d_key_off, d_key_len,
          d_match, stream=None):
    """Asynchronously probe int(d_query_filter.numel()) (filter, key) pairs."""
    n = int(d_query_filter.numel())
    check(_L.lgs_bloom_match_dev(d_filters.data_ptr(), d_filter_off.data_ptr(),
                                 d_filter_len.data_ptr(), d_query_filter.data_ptr(),
                                 d_keys.data_ptr(), d_key_off.data_ptr(), d_key_len.data_ptr(),
                                 d_match.data_ptr(), n, _stream_ptr(stream)),
          "lgs_bloom_match_dev")


# ---- the filter block of one table (filter_block.c) ----

def filter_block_bound(nkeys: int, nblocks: int, data_end: int, bits_per_key: int = 10) -> int:
    return int(_L.lgs_filter_block_bound(nkeys, nblocks, data_end, bits_per_key))


def filter_block_scratch(data_end: int) -> int:
    return int(_L.lgs_filter_block_scratch(data_end))


def filter_block_host(blocks: Sequence[Sequence[bytes]], block_off: Sequence[int], data_end: int,
                      bits_per_key: int = 10, internal_keys: bool = False) -> bytes:
    """blocks[b] = the keys of data block b in file order, block_off[b] its
    file offset, data_end the offset after the last data block."""
    import ctypes as C
    keys = [k for g in blocks for k in g]
    buf, offs, lens = _pack(keys)
    first = np.zeros(len(blocks) + 1, dtype=np.uint32)
    first[1:] = np.cumsum([len(g) for g in blocks], dtype=np.uint64)
    boff = np.array(list(block_off) + [0], dtype=np.uint64)
    cap = filter_block_bound(len(keys), len(blocks), data_end, bits_per_key)
    out = np.zeros(cap + 1, dtype=np.uint8)
    size = C.c_size_t(0)
    check(_L.lgs_filter_block_build_host(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                         first.ctypes.data, boff.ctypes.data, len(blocks),
                                         data_end, bits_per_key, int(internal_keys),
                                         out.ctypes.data, cap, C.byref(size)),
          "lgs_filter_block_build_host")
    return out[:size.value].tobytes()


def filter_block_match_host(block: bytes, queries: Sequence[tuple[int, bytes]],
                            internal_keys: bool = False) -> np.ndarray:
    """uint8 array: ldb_filter_matches(block, data block offset, key) per query."""
    bb = np.frombuffer(bytes(block) + b"\0" * 16, dtype=np.uint8)
    kbuf, koff, klen = _pack([k for _, k in queries])
    qo = np.array([o for o, _ in queries] + [0], dtype=np.uint64)
    m = np.zeros(len(queries), dtype=np.uint8)
    check(_L.lgs_filter_block_match_host(bb.ctypes.data, len(block), qo.ctypes.data,
                                         kbuf.ctypes.data, koff.ctypes.data, klen.ctypes.data,
                                         len(queries), int(internal_keys), m.ctypes.data),
          "lgs_filter_block_match_host")
    return m


def filter_block_build(d_keys, d_key_off, d_key_len, d_block_first, d_block_off, data_end,
                       bits_per_key, d_out, d_size, d_scratch, internal_keys=False, stream=None):
    """Asynchronously build the filter block of int(d_block_first.numel()) - 1
    data blocks into d_out (length -> d_size[0])."""
    nb = int(d_block_first.numel()) - 1
    check(_L.lgs_filter_block_build_dev(d_keys.data_ptr(), d_key_off.data_ptr(),
                                        d_key_len.data_ptr(), int(d_key_len.numel()),
                                        d_block_first.data_ptr(), d_block_off.data_ptr(), nb,
                                        data_end, bits_per_key, int(internal_keys),
                                        d_out.data_ptr(), d_out.numel(), d_size.data_ptr(),
                                        d_scratch.data_ptr(), d_scratch.numel(),
                                        _stream_ptr(stream)),
          "lgs_filter_block_build_dev")


def filter_block_match(d_block, block_len, d_block_offset, d_keys, d_key_off, d_key_len, d_match,
                       internal_keys=False, stream=None):
    """Asynchronously answer int(d_block_offset.numel()) filter-block queries."""
    n = int(d_block_offset.numel())
    check(_L.lgs_filter_block_match_dev(d_block.data_ptr(), block_len, d_block_offset.data_ptr(),
                                        d_keys.data_ptr(), d_key_off.data_ptr(),
                                        d_key_len.data_ptr(), n, int(internal_keys),
                                        d_match.data_ptr(), _stream_ptr(stream)),
          "lgs_filter_block_match_dev")
