"""oracle -- TEST INFRASTRUCTURE ONLY: the CPU parity checker.

Loads (ctypes) two CPU codecs with lcdb's snappy.h interface:

* ``liboracle.so``: our C89 restatement of lcdb src/util/snappy.c
  (snappy_oracle.c, every function citing the reference file:line);
* ``_ref/libref_snappy.so``: the reference's own snappy.c compiled unmodified
  by oracle/Makefile (present wherever it was built; it travels to the GPU
  box as a prebuilt .so, the reference sources do not).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package, and only as the checker / the timed CPU baseline.  The product
(lcdb_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import time
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_snappy.so")


class Codec:
    """One CPU snappy implementation behind lcdb's 4-function interface."""

    def __init__(self, path: str, prefix: str, name: str):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.name = name
        self.path = path
        self.lib = C.CDLL(path, mode=C.RTLD_LOCAL)
        vp, sz = C.c_void_p, C.c_size_t
        self.f_encode_size = getattr(self.lib, prefix + "encode_size")
        self.f_encode_size.restype, self.f_encode_size.argtypes = C.c_int, [C.POINTER(sz), sz]
        self.f_encode = getattr(self.lib, prefix + "encode")
        self.f_encode.restype, self.f_encode.argtypes = sz, [vp, vp, sz]
        self.f_decode_size = getattr(self.lib, prefix + "decode_size")
        self.f_decode_size.restype, self.f_decode_size.argtypes = C.c_int, [C.POINTER(sz), vp, sz]
        self.f_decode = getattr(self.lib, prefix + "decode")
        self.f_decode.restype, self.f_decode.argtypes = C.c_int, [vp, vp, sz]

    def encode_size(self, n: int) -> Optional[int]:
        z = C.c_size_t(0)
        return z.value if self.f_encode_size(C.byref(z), n) else None

    def encode(self, data: bytes) -> bytes:
        src = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8)
        dst = np.empty(self.encode_size(len(data)) or 0, dtype=np.uint8)
        n = self.f_encode(dst.ctypes.data, src.ctypes.data, len(data))
        return dst[:n].tobytes()

    def decode_size(self, data: bytes) -> Optional[int]:
        src = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
        z = C.c_size_t(0)
        return z.value if self.f_decode_size(C.byref(z), src.ctypes.data, len(data)) else None

    def decode(self, data: bytes) -> Optional[bytes]:
        want = self.decode_size(data)
        if want is None:
            return None
        src = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
        dst = np.empty(max(want, 1), dtype=np.uint8)
        ok = self.f_decode(dst.ctypes.data, src.ctypes.data, len(data))
        return dst[:want].tobytes() if ok else None

    # -- batches (pthreads, static round-robin partition: cpu_batch.c) --

    def _batch(self, mode: int, fn, threads, buf, off, ln, out, ooff, olen, status):
        drv = _driver()
        rc = drv.cpu_batch_run(mode, C.cast(fn, C.c_void_p), threads,
                               buf.ctypes.data, off.ctypes.data, ln.ctypes.data,
                               out.ctypes.data, ooff.ctypes.data,
                               olen.ctypes.data if olen is not None else None,
                               status.ctypes.data if status is not None else None,
                               int(ln.shape[0]))
        if rc != 0:
            raise RuntimeError("cpu_batch_run failed")

    def encode_batch(self, buf, off, ln, threads: int = 1):
        """Encode a corpus; returns (out, out_off, out_len), bound-spaced."""
        bounds = (ln.astype(np.uint64) * 7 // 6 + 48) // 16 * 16
        ooff = np.zeros_like(off)
        if len(ln):
            ooff[1:] = np.cumsum(bounds[:-1])
        out = np.zeros(int(bounds.sum()) + 16, dtype=np.uint8)
        olen = np.zeros(len(ln), dtype=np.uint32)
        self._batch(0, self.f_encode, threads, buf, off, ln, out, ooff, olen, None)
        return out, ooff, olen

    def decode_batch(self, buf, off, ln, caps, threads: int = 1):
        """Decode a corpus into cap-spaced slots; returns (out, out_off, status)."""
        caps64 = (caps.astype(np.uint64) + 15) // 16 * 16
        ooff = np.zeros(len(ln), dtype=np.uint64)
        if len(ln):
            ooff[1:] = np.cumsum(caps64[:-1])
        out = np.zeros(int(caps64.sum()) + 16, dtype=np.uint8)
        st = np.zeros(len(ln), dtype=np.uint8)
        self._batch(1, self.f_decode, threads, buf, off, ln, out, ooff, None, st)
        return out, ooff, st


_drv = None


def _driver():
    global _drv
    if _drv is None:
        d = C.CDLL(ORACLE_SO, mode=C.RTLD_LOCAL)
        d.cpu_batch_run.restype = C.c_int
        d.cpu_batch_run.argtypes = [C.c_int, C.c_void_p, C.c_int] + [C.c_void_p] * 7 + [C.c_uint32]
        _drv = d
    return _drv


_oracle = None
_ref = None


def restatement() -> Codec:
    """Our C89 restatement (always available once built)."""
    global _oracle
    if _oracle is None:
        _oracle = Codec(ORACLE_SO, "oracle_snappy_", "oracle")
    return _oracle


def reference() -> Optional[Codec]:
    """lcdb's own snappy.c compiled unmodified, or None if not built."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        _ref = Codec(REF_SO, "ldb_snappy_", "reference")
    return _ref


def best() -> Codec:
    """The reference build when present, else the restatement."""
    return reference() or restatement()


def time_cpu(codec: Codec, mode: str, buf, off, ln, threads: int, comp=None,
             min_seconds: float = 1.0, max_reps: int = 50) -> tuple[float, int]:
    """Median wall seconds of one pass over the corpus (encode or decode)."""
    times = []
    if mode == "decode":
        caps = np.full(len(ln), int(comp[3].max()) if len(ln) else 0, dtype=np.uint32)
    t_end = time.perf_counter() + min_seconds
    reps = 0
    while reps < 3 or (time.perf_counter() < t_end and reps < max_reps):
        t0 = time.perf_counter()
        if mode == "encode":
            codec.encode_batch(buf, off, ln, threads)
        else:
            codec.decode_batch(comp[0], comp[1], comp[2], caps, threads)
        times.append(time.perf_counter() - t0)
        reps += 1
    return float(np.median(times)), reps
