"""Python face of the gfx950 Snappy codec.

Two layers, mirroring ``include/lcdb_gpu_snappy.h``:

* the reference's four entry points (lcdb ``src/util/snappy.h:28-38``), same
  names, argument meaning and failure behaviour, on host bytes:
  ``encode_size``, ``encode``, ``decode_size``, ``decode``;
* the batched device-resident API over torch tensors already in HBM
  (``encode_batch`` / ``decode_batch``) and its host-buffer variant
  (``encode_batch_host`` / ``decode_batch_host``).

Every call runs on the GPU through ``liblcdb_gpu_snappy.so``; there is no CPU
fallback (importing this module raises if the library is missing).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _native
from ._native import LGS_ST_CORRUPT, LGS_ST_NOSPACE, LGS_ST_OK, check

_L = _native.lib()

__all__ = [
    "encode_size", "encode", "decode_size", "decode",
    "encode_bound", "encode_batch", "decode_batch", "encode_batch_host", "decode_batch_host",
    "DeviceBatch", "LGS_ST_OK", "LGS_ST_CORRUPT", "LGS_ST_NOSPACE",
]


# ---------------------------------------------------------------------------
# Reference entry points (snappy.h:28-38).  Failures follow the reference:
# encode_size / decode_size return None where the C function returns 0,
# decode returns None where ldb_snappy_decode returns 0 (corrupt input).
# ---------------------------------------------------------------------------

def encode_size(n: int) -> Optional[int]:
    """``snappy_encode_size`` (snappy.c:347-362): worst-case output bytes."""
    zn = C.c_size_t(0)
    return zn.value if _L.ldb_snappy_encode_size(C.byref(zn), n) else None


def encode(data: bytes) -> bytes:
    """``snappy_encode`` (snappy.c:364-384), computed on the GPU."""
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    bound = encode_size(len(src))
    if bound is None:
        raise ValueError("input too large for snappy")
    dst = np.empty(bound, dtype=np.uint8)
    n = _L.ldb_snappy_encode(dst.ctypes.data, src.ctypes.data if len(src) else None, len(src))
    return dst[:n].tobytes()


def decode_size(data: bytes) -> Optional[int]:
    """``snappy_decode_size`` (snappy.c:386-399): the varint32 length header."""
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    zn = C.c_size_t(0)
    ok = _L.ldb_snappy_decode_size(C.byref(zn), src.ctypes.data if len(src) else None, len(src))
    return zn.value if ok else None


def decode(data: bytes) -> Optional[bytes]:
    """``snappy_decode`` (snappy.c:401-412) on the GPU; None if corrupt."""
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    want = decode_size(data)
    if want is None:
        return None
    dst = np.empty(max(want, 1), dtype=np.uint8)
    ok = _L.ldb_snappy_decode(dst.ctypes.data, src.ctypes.data if len(src) else None, len(src))
    return dst[:want].tobytes() if ok else None


def encode_bound(n: int) -> int:
    return int(_L.lgs_encode_bound(n))


# ---------------------------------------------------------------------------
# Batched, device-resident (torch tensors in HBM).  Offsets are int64, lengths
# and capacities int32 (they are < 2**31), status uint8.
# ---------------------------------------------------------------------------

@dataclass
class DeviceBatch:
    """Blocks packed in one device buffer: block i = buf[off[i] : off[i]+len[i]]."""
    buf: "object"     # torch.uint8 cuda tensor
    off: "object"     # torch.int64 cuda tensor
    len: "object"     # torch.int32 cuda tensor
    max_len: int


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


def encode_batch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, max_in_len: int,
                 stream=None) -> None:
    """Asynchronously encode every block (``lgs_encode_batch_dev``)."""
    n = int(d_in_len.numel())
    check(_L.lgs_encode_batch_dev(d_in.data_ptr(), d_in_off.data_ptr(), d_in_len.data_ptr(),
                                  d_out.data_ptr(), d_out_off.data_ptr(), d_out_len.data_ptr(),
                                  n, int(max_in_len), _stream_ptr(stream)),
          "lgs_encode_batch_dev")


def decode_batch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                 max_out_cap: int, stream=None) -> None:
    """Asynchronously decode every block (``lgs_decode_batch_dev``)."""
    n = int(d_in_len.numel())
    check(_L.lgs_decode_batch_dev(d_in.data_ptr(), d_in_off.data_ptr(), d_in_len.data_ptr(),
                                  d_out.data_ptr(), d_out_off.data_ptr(), d_out_cap.data_ptr(),
                                  d_out_len.data_ptr(), d_status.data_ptr(), n,
                                  int(max_out_cap), _stream_ptr(stream)),
          "lgs_decode_batch_dev")


# ---------------------------------------------------------------------------
# Batched, host buffers (numpy); pinned staging inside the library.
# ---------------------------------------------------------------------------

def _pack(blocks: Sequence[bytes]):
    lens = np.array([len(b) for b in blocks], dtype=np.uint32)
    offs = np.zeros(len(blocks), dtype=np.uint64)
    if len(blocks):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(blocks) + b"\0" * 16, dtype=np.uint8)
    return buf, offs, lens


def encode_batch_host(blocks: Sequence[bytes]) -> list[bytes]:
    """Encode a list of blocks in one GPU launch."""
    n = len(blocks)
    if n == 0:
        return []
    buf, offs, lens = _pack(blocks)
    bounds = np.array([encode_bound(int(x)) for x in lens], dtype=np.uint64)
    ooff = np.zeros(n, dtype=np.uint64)
    ooff[1:] = np.cumsum(bounds[:-1])
    out = np.empty(int(bounds.sum()) + 16, dtype=np.uint8)
    olen = np.zeros(n, dtype=np.uint32)
    check(_L.lgs_encode_batch_host(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                   out.ctypes.data, ooff.ctypes.data, olen.ctypes.data, n),
          "lgs_encode_batch_host")
    return [out[int(o):int(o) + int(k)].tobytes() for o, k in zip(ooff, olen)]


def decode_batch_host(blocks: Sequence[bytes], caps: Sequence[int]):
    """Decode blocks; returns (outputs, status) with None for failed blocks."""
    n = len(blocks)
    if n == 0:
        return [], np.zeros(0, dtype=np.uint8)
    buf, offs, lens = _pack(blocks)
    cap = np.array(caps, dtype=np.uint32)
    ooff = np.zeros(n, dtype=np.uint64)
    ooff[1:] = np.cumsum(cap[:-1].astype(np.uint64))
    out = np.empty(int(cap.sum()) + 16, dtype=np.uint8)
    olen = np.zeros(n, dtype=np.uint32)
    st = np.zeros(n, dtype=np.uint8)
    check(_L.lgs_decode_batch_host(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                   out.ctypes.data, ooff.ctypes.data, cap.ctypes.data,
                                   olen.ctypes.data, st.ctypes.data, n),
          "lgs_decode_batch_host")
    res = [out[int(o):int(o) + int(k)].tobytes() if s == LGS_ST_OK else None
           for o, k, s in zip(ooff, olen, st)]
    return res, st
