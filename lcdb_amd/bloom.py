"""lcdb's bloom filter on the GPU.

Python face of the batched C ABI (``include/lcdb_gpu_snappy.h``):

* ``build_host(groups, bits_per_key)``: one filter per key group, each byte
  for byte what ``ldb_bloom_build`` appends (src/util/bloom.c:102-119);
* ``match_host(filters, queries)``: ``ldb_bloom_match`` per (filter, key)
  (bloom.c:121-165);
* ``build`` / ``match`` on device tensors (int64 offsets, int32 lengths).

Everything runs through ``liblcdb_gpu_snappy.so``; there is no CPU fallback.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import _native
from ._native import check
from .snappy import _stream_ptr

_L = _native.lib()

__all__ = ["filter_size", "build_host", "match_host", "build", "match"]


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
