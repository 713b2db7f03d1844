"""ctypes binding of ``liblcdb_gpu_snappy.so`` (C ABI: include/lcdb_gpu_snappy.h).

There is no fallback: if the library is missing or fails to load, importing
the codec raises.  The library is loaded from the package directory only.
"""
from __future__ import annotations

import ctypes as C
import os

from .build import LIB

LGS_OK = 0
LGS_EINVAL, LGS_EHIP, LGS_ENODEV, LGS_ENOMEM, LGS_ENOSPC, LGS_EINTERNAL = -1, -2, -3, -4, -5, -6
LGS_ST_CORRUPT, LGS_ST_OK, LGS_ST_NOSPACE = 0, 1, 2
LGS_ST_IOERR, LGS_ST_BADCRC, LGS_ST_BADTYPE = 3, 4, 5
LGS_NO_COMPRESSION, LGS_SNAPPY_COMPRESSION = 0, 1
LGS_TRAILER_SIZE = 5

_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p

_SIGS = {
    "ldb_snappy_encode_size": (C.c_int, [C.POINTER(C.c_size_t), C.c_size_t]),
    "ldb_snappy_encode": (C.c_size_t, [_vp, _vp, C.c_size_t]),
    "ldb_snappy_decode_size": (C.c_int, [C.POINTER(C.c_size_t), _vp, C.c_size_t]),
    "ldb_snappy_decode": (C.c_int, [_vp, _vp, C.c_size_t]),
    "lgs_encode_bound": (C.c_size_t, [C.c_size_t]),
    "lgs_encode_batch_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, C.c_uint32, C.c_uint32, _vp]),
    "lgs_decode_batch_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_uint32,
                                       C.c_uint32, _vp]),
    "lgs_encode_batch_host": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, C.c_uint32]),
    "lgs_decode_batch_host": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_uint32]),
    "lgs_crc32c_batch_dev": (C.c_int, [_vp, _vp, _vp, _vp, C.c_int, _vp, C.c_uint32, _vp]),
    "lgs_table_write_scratch": (C.c_size_t, [C.c_uint32, C.c_uint64]),
    "lgs_table_write_dev": (C.c_int, [_vp, _vp, _vp, C.c_uint32, C.c_uint32, C.c_uint64, C.c_int,
                                      C.c_uint64, _vp, _vp, _vp, _vp, _vp, C.c_size_t, _vp]),
    "lgs_table_write_host": (C.c_int, [_vp, _vp, _vp, C.c_uint32, C.c_int, C.c_uint64, _vp,
                                       C.c_size_t, _vp, _vp, _vp]),
    "lgs_table_read_scratch": (C.c_size_t, [C.c_uint32]),
    "lgs_table_read_dev": (C.c_int, [_vp, C.c_uint64, _vp, _vp, C.c_uint32, C.c_int, _vp, _vp,
                                     _vp, C.c_uint32, _vp, _vp, _vp, C.c_size_t, _vp]),
    "lgs_table_read_host": (C.c_int, [_vp, C.c_uint64, _vp, _vp, C.c_uint32, C.c_int, _vp, _vp,
                                      _vp, _vp, _vp]),
    "lgs_table_index_host": (C.c_int, [_vp, C.c_uint64, C.c_int, C.c_int, C.c_char_p, _vp, _vp,
                                       C.c_uint32, _vp, _vp, C.c_size_t, _vp, _vp, _vp, _vp]),
    "lgs_bloom_filter_size": (C.c_size_t, [C.c_uint32, C.c_int]),
    "lgs_bloom_build_dev": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, C.c_int, _vp, _vp, _vp]),
    "lgs_bloom_match_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_uint32, _vp]),
    "lgs_bloom_build_host": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint32, C.c_int, _vp, _vp]),
    "lgs_bloom_match_host": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, _vp, _vp,
                                       C.c_uint32, _vp]),
    "lgs_filter_block_bound": (C.c_size_t, [C.c_uint32, C.c_uint32, C.c_uint64, C.c_int]),
    "lgs_filter_block_scratch": (C.c_size_t, [C.c_uint64]),
    "lgs_filter_block_build_dev": (C.c_int, [_vp, _vp, _vp, C.c_uint32, _vp, _vp, C.c_uint32,
                                             C.c_uint64, C.c_int, C.c_int, _vp, C.c_size_t, _vp,
                                             _vp, C.c_size_t, _vp]),
    "lgs_filter_block_build_host": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_uint32, C.c_uint64,
                                              C.c_int, C.c_int, _vp, C.c_size_t,
                                              C.POINTER(C.c_size_t)]),
    "lgs_filter_block_match_dev": (C.c_int, [_vp, C.c_size_t, _vp, _vp, _vp, _vp, C.c_uint32,
                                             C.c_int, _vp, _vp]),
    "lgs_filter_block_match_host": (C.c_int, [_vp, C.c_size_t, _vp, _vp, _vp, _vp, C.c_uint32,
                                              C.c_int, _vp]),
    "lgs_dropin_footprint": (C.c_int, [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t),
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_size_t)]),
    "lgs_service_quiesce": (C.c_int, []),
    "lgs_service_resume": (C.c_int, []),
    "lgs_set_option": (C.c_int, [C.c_char_p, C.c_char_p]),
    "lgs_hbm_copy_dev": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "lgs_device_count": (C.c_int, []),
    "lgs_set_device": (C.c_int, [C.c_int]),
    "lgs_last_error": (C.c_char_p, []),
    "lgs_version": (C.c_char_p, []),
}

# Every symbol include/lcdb_gpu_snappy.h declares.
EXPORTED = tuple(_SIGS)

_lib = None


def lib() -> C.CDLL:
    """Load (once) and return the native library; raises if it is absent."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch's wheel bundles its own
        # libamdhip64/libhsa-runtime64 and its libraries NEED the unversioned
        # "libamdhip64.so", while ours NEEDs the soname "libamdhip64.so.7".
        # Loading torch first makes our NEEDED entries resolve (by soname) to
        # the runtime torch already loaded; loading ours first would make
        # torch bring up a second HSA runtime that then finds no GPU.
        import torch  # noqa: F401
        if not os.path.exists(LIB):
            raise ImportError(
                f"lcdb_amd native library not built: {LIB} is missing "
                "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
        handle = C.CDLL(LIB, mode=C.RTLD_LOCAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


class LgsError(RuntimeError):
    pass


def set_option(name: str, value: str) -> None:
    """lgs_set_option: process-wide kernel choice ("decoder", "split")."""
    check(lib().lgs_set_option(name.encode(), value.encode()), f"lgs_set_option({name})")


def dropin_footprint() -> dict:
    """Bytes the drop-in's staging slots hold (lgs_dropin_footprint)."""
    p, d, n, cap = C.c_size_t(0), C.c_size_t(0), C.c_uint32(0), C.c_size_t(0)
    check(lib().lgs_dropin_footprint(C.byref(p), C.byref(d), C.byref(n), C.byref(cap)),
          "lgs_dropin_footprint")
    return {"pinned": p.value, "device": d.value, "slots": n.value, "slot_bytes": cap.value}


def check(rc: int, what: str) -> None:
    if rc != LGS_OK:
        msg = lib().lgs_last_error().decode(errors="replace")
        raise LgsError(f"{what} failed ({rc}): {msg}")
