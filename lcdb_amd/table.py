"""SSTable block framing on the GPU.

lcdb stores every table block as ``contents | type | masked crc32c`` and
reads one back through ``ldb_read_block``.  This module is the Python face of
the batched C ABI that does both for many blocks per launch
(``include/lcdb_gpu_snappy.h``):

* ``crc32c_batch``    -- ``ldb_crc32c_value``/``extend``/``mask`` per block
  (src/util/crc32c.c:1147, crc32c.h:46-50);
* ``write_blocks``    -- ``ldb_tablegen_write_block`` for n data blocks
  (src/table/table_builder.c:123-213): encode, 12.5 % rule, trailer, packing;
* ``read_blocks``     -- ``ldb_read_block`` for n handles
  (src/table/format.c:162-270): truncation, checksum, type, raw or decode;
* ``*_host`` variants on host bytes (pinned staging inside the library);
* ``index_host``      -- ``ldb_table_open``'s footer, index-block handles and
  metaindex filter handle (src/table/table.c:78-180), the handles the batched
  read takes.

Everything runs through ``liblcdb_gpu_snappy.so``; there is no CPU fallback.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import _native
from ._native import (LGS_NO_COMPRESSION, LGS_SNAPPY_COMPRESSION, LGS_ST_BADCRC,
                      LGS_ST_BADTYPE, LGS_ST_CORRUPT, LGS_ST_IOERR, LGS_ST_NOSPACE, LGS_ST_OK,
                      LGS_TRAILER_SIZE, check)
from .snappy import _stream_ptr

_L = _native.lib()

__all__ = [
    "crc32c_batch", "write_blocks", "read_blocks", "write_blocks_host", "read_blocks_host",
    "index_host", "FILTER_NAME",
    "LGS_NO_COMPRESSION", "LGS_SNAPPY_COMPRESSION", "LGS_TRAILER_SIZE", "LGS_ST_OK",
    "LGS_ST_CORRUPT", "LGS_ST_NOSPACE", "LGS_ST_IOERR", "LGS_ST_BADCRC", "LGS_ST_BADTYPE",
]


def _torch():
    import torch
    return torch


# ---------------------------------------------------------------------------
# Device-resident (torch tensors in HBM): offsets int64, lengths int32.
# ---------------------------------------------------------------------------

def crc32c_batch(d_in, d_off, d_len, d_type=None, masked: bool = True, d_crc=None, stream=None):
    """CRC32C of every block (followed by d_type[i] when given), masked by
    default: with a type this is each block's trailer crc field."""
    torch = _torch()
    n = int(d_len.numel())
    if d_crc is None:
        d_crc = torch.empty(n, dtype=torch.int32, device=d_in.device)
    check(_L.lgs_crc32c_batch_dev(d_in.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                  d_type.data_ptr() if d_type is not None else None,
                                  1 if masked else 0, d_crc.data_ptr(), n, _stream_ptr(stream)),
          "lgs_crc32c_batch_dev")
    return d_crc


def write_buffers(n: int, raw_total: int, device, base: int = 0):
    """The output and scratch tensors of write_blocks, allocated once (a
    caller framing the same shape repeatedly passes them as `bufs`)."""
    torch = _torch()
    nscr = int(_L.lgs_table_write_scratch(n, raw_total))
    return (torch.empty(raw_total + LGS_TRAILER_SIZE * n + 16, dtype=torch.uint8, device=device),
            torch.empty(n, dtype=torch.int64, device=device),
            torch.empty(n, dtype=torch.int64, device=device),
            torch.full((1,), base, dtype=torch.int64, device=device),
            torch.empty(max(nscr, 1), dtype=torch.uint8, device=device))


def write_blocks(d_raw, d_off, d_len, compression: int = LGS_SNAPPY_COMPRESSION, base: int = 0,
                 max_len: Optional[int] = None, raw_total: Optional[int] = None, stream=None,
                 bufs=None):
    """Frame n raw data blocks into a contiguous file region.

    Returns (d_file, d_handle_off, d_handle_size, d_end): d_file[j] is file
    offset base + j, d_end[0] = base + bytes written (read it after the
    stream syncs).  d_raw must stay readable 16 bytes past every block.
    bufs: write_buffers(n, raw_total, device, base), reused."""
    torch = _torch()
    n = int(d_len.numel())
    dev = d_raw.device
    if max_len is None or raw_total is None:
        lens = d_len.to(torch.int64)
        max_len = int(lens.max()) if n else 0
        raw_total = int(lens.sum()) if n else 0
    d_file, hoff, hsize, end, scr = bufs if bufs is not None else write_buffers(n, raw_total, dev, base)
    nscr = int(scr.numel())
    check(_L.lgs_table_write_dev(d_raw.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                 int(max_len), int(raw_total), int(compression), int(base),
                                 d_file.data_ptr(), hoff.data_ptr(), hsize.data_ptr(),
                                 end.data_ptr(), scr.data_ptr(), nscr, _stream_ptr(stream)),
          "lgs_table_write_dev")
    return d_file, hoff, hsize, end


def read_blocks(d_file, file_len: int, d_hoff, d_hsize, d_out, d_out_off, d_out_cap,
                max_out_cap: int, verify: bool = True, d_out_len=None, d_status=None,
                stream=None, scratch=None):
    """ldb_read_block for every handle; returns (d_out_len, d_status).
    d_file must stay readable 16 bytes past file_len.  scratch: a uint8
    tensor of lgs_table_read_scratch(n) bytes, reused."""
    torch = _torch()
    n = int(d_hoff.numel())
    dev = d_file.device
    if d_out_len is None:
        d_out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    if d_status is None:
        d_status = torch.zeros(n, dtype=torch.uint8, device=dev)
    if scratch is None:
        scratch = torch.empty(max(int(_L.lgs_table_read_scratch(n)), 1), dtype=torch.uint8,
                              device=dev)
    scr = scratch
    nscr = int(scr.numel())
    check(_L.lgs_table_read_dev(d_file.data_ptr(), int(file_len), d_hoff.data_ptr(),
                                d_hsize.data_ptr(), n, 1 if verify else 0, d_out.data_ptr(),
                                d_out_off.data_ptr(), d_out_cap.data_ptr(), int(max_out_cap),
                                d_out_len.data_ptr(), d_status.data_ptr(), scr.data_ptr(), nscr,
                                _stream_ptr(stream)),
          "lgs_table_read_dev")
    return d_out_len, d_status


# ---------------------------------------------------------------------------
# Host bytes.
# ---------------------------------------------------------------------------

def write_blocks_host(blocks: Sequence[bytes], compression: int = LGS_SNAPPY_COMPRESSION,
                      base: int = 0):
    """Returns (region bytes for file offsets [base, end), handle_off, handle_size, end)."""
    n = len(blocks)
    lens = np.array([len(b) for b in blocks], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(blocks) + b"\0" * 16, dtype=np.uint8)
    cap = int(lens.sum()) + LGS_TRAILER_SIZE * n + 16
    file = np.empty(cap, dtype=np.uint8)
    hoff = np.zeros(n, dtype=np.uint64)
    hsize = np.zeros(n, dtype=np.uint64)
    end = np.zeros(1, dtype=np.uint64)
    check(_L.lgs_table_write_host(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                                  int(compression), int(base), file.ctypes.data, cap,
                                  hoff.ctypes.data, hsize.ctypes.data, end.ctypes.data),
          "lgs_table_write_host")
    e = int(end[0])
    return file[:e - base].tobytes(), hoff, hsize, e


def read_blocks_host(file, handle_off, handle_size, caps, verify: bool = True):
    """Returns (list of contents or None, status array) for every handle."""
    img = np.frombuffer(bytes(file), dtype=np.uint8) if not isinstance(file, np.ndarray) else file
    n = len(handle_off)
    hoff = np.ascontiguousarray(handle_off, dtype=np.uint64)
    hsize = np.ascontiguousarray(handle_size, dtype=np.uint64)
    cap = np.ascontiguousarray(caps, dtype=np.uint32)
    ooff = np.zeros(n, dtype=np.uint64)
    if n:
        ooff[1:] = np.cumsum(cap[:-1].astype(np.uint64))
    out = np.empty(int(cap.astype(np.uint64).sum()) + 16, dtype=np.uint8)
    olen = np.zeros(n, dtype=np.uint32)
    st = np.zeros(n, dtype=np.uint8)
    check(_L.lgs_table_read_host(img.ctypes.data if len(img) else None, len(img),
                                 hoff.ctypes.data, hsize.ctypes.data, n, 1 if verify else 0,
                                 out.ctypes.data, ooff.ctypes.data, cap.ctypes.data,
                                 olen.ctypes.data, st.ctypes.data),
          "lgs_table_read_host")
    res = [out[int(o):int(o) + int(k)].tobytes() if s == LGS_ST_OK else None
           for o, k, s in zip(ooff, olen, st)]
    return res, st


FILTER_NAME = "filter.leveldb.BuiltinBloomFilter2"   # "filter." + bloom.c's policy name


def index_host(file, paranoid_checks: bool = False, internal_keys: bool = False,
               filter_name: str | None = FILTER_NAME, cap: int | None = None):
    """ldb_table_open's view of a table file (lgs_table_index_host): returns
    (handles [(offset, size)], separator keys, filter handle or None, status)."""
    import ctypes as C
    raw = bytes(file)
    img = np.frombuffer(raw + b"\0", dtype=np.uint8)
    cap = cap if cap is not None else max(1, len(raw) // 8)
    hoff = np.zeros(cap, dtype=np.uint64)
    hsize = np.zeros(cap, dtype=np.uint64)
    keys = np.zeros(max(1, len(raw)), dtype=np.uint8)
    koff = np.zeros(cap + 1, dtype=np.uint64)
    count = C.c_uint32(0)
    foff, fsize = C.c_uint64(0), C.c_uint64(0)
    st = C.c_uint8(0)
    check(_L.lgs_table_index_host(img.ctypes.data, len(raw), int(paranoid_checks),
                                  int(internal_keys),
                                  filter_name.encode() if filter_name else None,
                                  hoff.ctypes.data, hsize.ctypes.data, cap, C.byref(count),
                                  keys.ctypes.data, len(keys), koff.ctypes.data, C.byref(foff),
                                  C.byref(fsize), C.byref(st)),
          "lgs_table_index_host")
    n = count.value
    handles = [(int(hoff[i]), int(hsize[i])) for i in range(n)]
    ks = [keys[int(koff[i]):int(koff[i + 1])].tobytes() for i in range(n)]
    fh = None if foff.value == (1 << 64) - 1 else (foff.value, fsize.value)
    return handles, ks, fh, st.value
