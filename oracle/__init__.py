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

    def _batch(self, mode: int, fn, threads, buf, off, ln, out, ooff, olen, status,
               partition: int = 0, reps: int = 1):
        drv = _driver()
        rc = drv.cpu_batch_run3(mode, C.cast(fn, C.c_void_p), threads, partition, reps,
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
        d.cpu_batch_run2.restype = C.c_int
        d.cpu_batch_run2.argtypes = ([C.c_int, C.c_void_p, C.c_int, C.c_int] + [C.c_void_p] * 7
                                     + [C.c_uint32])
        d.cpu_batch_run3.restype = C.c_int
        d.cpu_batch_run3.argtypes = ([C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_uint32]
                                     + [C.c_void_p] * 7 + [C.c_uint32])
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


# -- block framing (table_oracle.c): CRC32C trailers, data-block writes,
#    block reads; plus the reference's own crc32c.c (_ref/libref_crc32c.so) --

REF_CRC_SO = os.path.join(HERE, "_ref", "libref_crc32c.so")
ST_CORRUPT, ST_OK, ST_NOSPACE, ST_IOERR, ST_BADCRC, ST_BADTYPE = 0, 1, 2, 3, 4, 5

_tab = None
_refcrc = None


def _table_lib():
    global _tab
    if _tab is None:
        d = C.CDLL(ORACLE_SO, mode=C.RTLD_LOCAL)
        vp, u64 = C.c_void_p, C.c_uint64
        d.oracle_crc32c_extend.restype = C.c_uint32
        d.oracle_crc32c_extend.argtypes = [C.c_uint32, vp, C.c_size_t]
        d.oracle_crc32c_mask.restype = C.c_uint32
        d.oracle_crc32c_mask.argtypes = [C.c_uint32]
        d.oracle_crc32c_unmask.restype = C.c_uint32
        d.oracle_crc32c_unmask.argtypes = [C.c_uint32]
        d.oracle_table_write_blocks.restype = C.c_int
        d.oracle_table_write_blocks.argtypes = [vp, vp, vp, C.c_uint32, C.c_int, u64, vp, vp, vp,
                                                vp, vp]
        d.oracle_table_read_block.restype = C.c_int
        d.oracle_table_read_block.argtypes = [vp, u64, u64, u64, C.c_int, vp, C.c_size_t,
                                              C.POINTER(C.c_size_t)]
        _tab = d
    return _tab


def _buf(data: bytes):
    return np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)


def crc32c(data: bytes, init: int = 0) -> int:
    """ldb_crc32c_extend(init, data) (crc32c.c:643-750), restated."""
    buf = _buf(data)   # keep the array alive across the call
    return int(_table_lib().oracle_crc32c_extend(init, buf.ctypes.data, len(data)))


def crc32c_mask(c: int) -> int:
    return int(_table_lib().oracle_crc32c_mask(c))


def crc32c_unmask(c: int) -> int:
    return int(_table_lib().oracle_crc32c_unmask(c))


def reference_crc32c() -> Optional[C.CDLL]:
    """lcdb's own crc32c.c compiled unmodified (ldb_crc32c_extend), or None."""
    global _refcrc
    if _refcrc is None and os.path.exists(REF_CRC_SO):
        d = C.CDLL(REF_CRC_SO, mode=C.RTLD_LOCAL)
        d.ldb_crc32c_extend.restype = C.c_uint32
        d.ldb_crc32c_extend.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        _refcrc = d
    return _refcrc


def table_write_blocks(blocks, compression: int = 1, base: int = 0):
    """ldb_tablegen_write_block per block (table_builder.c:123-213), restated.
    Returns (region bytes, handle_off, handle_size, end)."""
    n = len(blocks)
    lens = np.array([len(b) for b in blocks], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    raw = np.frombuffer(b"".join(blocks) + b"\0" * 16, dtype=np.uint8)
    file = np.zeros(int(lens.sum()) + 5 * n + 16, dtype=np.uint8)
    scratch = np.zeros(int(lens.max()) * 7 // 6 + 64 if n else 64, dtype=np.uint8)
    hoff = np.zeros(n, dtype=np.uint64)
    hsize = np.zeros(n, dtype=np.uint64)
    end = np.zeros(1, dtype=np.uint64)
    _table_lib().oracle_table_write_blocks(raw.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                           n, compression, base, file.ctypes.data,
                                           hoff.ctypes.data, hsize.ctypes.data, end.ctypes.data,
                                           scratch.ctypes.data)
    e = int(end[0])
    return file[:e - base].tobytes(), hoff, hsize, e


def table_read_block(file, off: int, size: int, verify: bool, cap: int):
    """ldb_read_block (format.c:162-270) on a file image, restated.
    Returns (status, contents or None)."""
    img = np.frombuffer(bytes(file) + b"\0" * 8, dtype=np.uint8)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    olen = C.c_size_t(0)
    st = _table_lib().oracle_table_read_block(img.ctypes.data, len(img) - 8, off, size,
                                              1 if verify else 0, out.ctypes.data, cap,
                                              C.byref(olen))
    return st, (out[:olen.value].tobytes() if st == ST_OK else None)


# -- bloom filter (bloom_oracle.c) and the reference's own bloom.c + hash.c
#    behind oracle/harness/bloom_ref.c (_ref/lcdb/libref_bloom.so) --

REF_BLOOM_SO = os.path.join(HERE, "_ref", "lcdb", "libref_bloom.so")


class Bloom:
    """ldb_hash / ldb_bloom_build / ldb_bloom_match behind one interface."""

    def __init__(self, path: str, hash_fn: str, build_fn: str, match_fn: str, name: str,
                 with_cap: bool):
        d = C.CDLL(path, mode=C.RTLD_LOCAL)
        vp, sz = C.c_void_p, C.c_size_t
        self.name, self.with_cap = name, with_cap
        self.f_hash = getattr(d, hash_fn)
        self.f_hash.restype, self.f_hash.argtypes = C.c_uint32, [vp, sz, C.c_uint32]
        self.f_build = getattr(d, build_fn)
        self.f_build.restype = sz
        self.f_build.argtypes = [vp, vp, vp, sz, C.c_int, vp] + ([sz] if with_cap else [])
        self.f_match = getattr(d, match_fn)
        self.f_match.restype, self.f_match.argtypes = C.c_int, [vp, sz, vp, sz]
        pre = "ref" if with_cap else "oracle"
        self.f_fb = getattr(d, pre + "_filter_block_build")
        self.f_fb.restype = sz
        self.f_fb.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, C.c_uint64, C.c_int,
                              C.c_int if with_cap else C.c_uint32, vp,
                              sz if with_cap else vp]
        self.f_fm = getattr(d, pre + "_filter_matches")
        self.f_fm.restype = C.c_int
        self.f_fm.argtypes = [vp, sz, C.c_uint64, vp, sz, C.c_int if with_cap else C.c_uint32]

    def hash(self, data: bytes, seed: int) -> int:
        b = _buf(data)
        return int(self.f_hash(b.ctypes.data, len(data), seed))

    def build(self, keys, bits_per_key: int = 10) -> bytes:
        lens = np.array([len(k) for k in keys], dtype=np.uint32)
        offs = np.zeros(len(keys), dtype=np.uint64)
        if len(keys):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        base = np.frombuffer(b"".join(keys) + b"\0" * 8, dtype=np.uint8)
        cap = max(64, len(keys) * max(bits_per_key, 0)) // 8 + 16
        out = np.zeros(cap, dtype=np.uint8)
        args = [base.ctypes.data, offs.ctypes.data, lens.ctypes.data, len(keys), bits_per_key,
                out.ctypes.data] + ([cap] if self.with_cap else [])
        n = self.f_build(*args)
        return out[:n].tobytes()

    def match(self, filt: bytes, key: bytes) -> bool:
        f, k = _buf(filt), _buf(key)
        return bool(self.f_match(f.ctypes.data, len(filt), k.ctypes.data, len(key)))

    # -- the filter block (filter_block.c), see oracle_filter_block_build --
    def filter_block(self, blocks, block_off, data_end: int, bits_per_key: int = 10,
                     internal: bool = False) -> bytes:
        """blocks[b] = the keys of data block b (file order); block_off[b] =
        its file offset; data_end = the offset after the last data block."""
        keys = [k for blk in blocks for k in blk]
        lens = np.array([len(k) for k in keys], dtype=np.uint32)
        offs = np.zeros(len(keys), dtype=np.uint64)
        if len(keys):
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        base = np.frombuffer(b"".join(keys) + b"\0" * 8, dtype=np.uint8)
        first = np.zeros(len(blocks) + 1, dtype=np.uint32)
        first[1:] = np.cumsum([len(b) for b in blocks], dtype=np.uint64)
        boff = np.array(list(block_off) + [0], dtype=np.uint64)
        nf = data_end // 2048 + 2
        cap = len(keys) * max(bits_per_key, 0) // 8 + 10 * (len(blocks) + 1) + 4 * nf + 64
        out = np.zeros(cap, dtype=np.uint8)
        if self.with_cap:
            n = self.f_fb(base.ctypes.data, offs.ctypes.data, lens.ctypes.data, first.ctypes.data,
                          boff.ctypes.data, len(blocks), data_end, bits_per_key, int(internal),
                          out.ctypes.data, cap)
        else:
            scratch = np.zeros(nf, dtype=np.uint32)
            n = self.f_fb(base.ctypes.data, offs.ctypes.data, lens.ctypes.data, first.ctypes.data,
                          boff.ctypes.data, len(blocks), data_end, bits_per_key,
                          8 if internal else 0, out.ctypes.data, scratch.ctypes.data)
        assert n > 0
        return out[:n].tobytes()

    def filter_matches(self, block: bytes, block_offset: int, key: bytes,
                       internal: bool = False) -> bool:
        f, k = _buf(block), _buf(key)
        flag = int(internal) if self.with_cap else (8 if internal else 0)
        return bool(self.f_fm(f.ctypes.data, len(block), block_offset, k.ctypes.data, len(key),
                              flag))


_bloom_orc = None
_bloom_ref = None


def bloom_restatement() -> Bloom:
    global _bloom_orc
    if _bloom_orc is None:
        _bloom_orc = Bloom(ORACLE_SO, "oracle_hash", "oracle_bloom_build", "oracle_bloom_match",
                           "oracle", False)
    return _bloom_orc


def bloom_reference() -> Optional[Bloom]:
    """lcdb's own bloom.c + hash.c (oracle/lcdb.mk), or None if not built."""
    global _bloom_ref
    if _bloom_ref is None and os.path.exists(REF_BLOOM_SO):
        _bloom_ref = Bloom(REF_BLOOM_SO, "ref_hash", "ref_bloom_build", "ref_bloom_match",
                           "reference", True)
    return _bloom_ref


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


def _affinity_cores(cpus) -> int | None:
    """Physical cores (package, core id) behind a set of logical CPUs."""
    cores = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            with open(base + "core_id") as f:
                core = f.read().strip()
            with open(base + "physical_package_id") as f:
                pkg = f.read().strip()
        except OSError:
            return None
        cores.add((pkg, core))
    return len(cores) or None


def cores_for_threads(threads: int) -> int:
    """Physical cores `threads` busy threads occupy at most on this host's
    affinity set (the scheduler spreads them over cores before SMT
    siblings): min(threads, physical cores in the affinity set)."""
    phys = _affinity_cores(sorted(os.sched_getaffinity(0)))
    return min(threads, phys) if phys else threads


def cpu_model() -> dict:
    """CPU model name, physical cores (whole host and this process's affinity
    set) and NUMA nodes of this host."""
    model, phys = "unknown", set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as f:
            for line in f.read().splitlines() + [""]:
                if not line.strip():
                    if "core id" in cur:
                        phys.add((cur.get("physical id", "0"), cur["core id"]))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name" and model == "unknown":
                    model = v.strip()
    except OSError:
        pass
    aff = sorted(os.sched_getaffinity(0))
    try:
        numa = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")
                    and d[4:].isdigit()])
    except OSError:
        numa = None
    return {"model": model, "physical_cores": len(phys) or None,
            "logical_cpus": os.cpu_count(), "affinity_cpus": len(aff),
            "affinity_physical_cores": _affinity_cores(aff), "numa_nodes": numa,
            "cgroup_cpu_quota": cgroup_cpu_quota()}


def cgroup_cpu_quota() -> float | None:
    """CPUs' worth of time this process's cgroup may use (cgroup v2 cpu.max,
    or v1 cfs_quota/cfs_period), None when unlimited or unknown.  A shared GPU
    box can show every CPU in the affinity mask while capping the container
    at its share: threads beyond the quota only time-slice."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def baseline_plan(codec: Codec, buf, off, ln, thread_counts, reps: int = 5,
                  partitions=(0,)) -> dict:
    """BASELINE.md "CPU-baseline plan": the codec over the same blocks the GPU
    timed, once per thread count and block partition (cpu_batch.c: 0 static
    round-robin, 1 contiguous), one untimed warm-up, then the median of
    `reps` timed runs, encode and decode separately.  The outputs are fresh,
    untouched buffers for every (threads, partition): the warm-up's worker
    threads fault their own pages in, so on a multi-socket host each thread
    writes memory of its own NUMA node (buffers reused from a run with
    another partition would keep that run's placement), and the timed runs
    reuse those pre-faulted pages.  Each timed call makes enough passes over
    the blocks (>= ~0.2 s) that starting the threads does not count.
    Returns GiB/s per (threads, partition)
    plus the compressed output (for the byte-for-byte check against the
    GPU's)."""
    n = int(ln.shape[0])
    raw = int(ln.sum(dtype=np.uint64))
    bounds = (ln.astype(np.uint64) * 7 // 6 + 48) // 16 * 16
    ooff = np.zeros(n, dtype=np.uint64)
    if n:
        ooff[1:] = np.cumsum(bounds[:-1])
    caps64 = (ln.astype(np.uint64) + 15) // 16 * 16
    doff = np.zeros(n, dtype=np.uint64)
    if n:
        doff[1:] = np.cumsum(caps64[:-1])
    res, keep = {}, None
    for t in thread_counts:
        for part in (partitions if t > 1 else (0,)):
            comp = np.empty(int(bounds.sum()) + 16, dtype=np.uint8)    # untouched pages
            dec = np.empty(int(caps64.sum()) + 16, dtype=np.uint8)
            olen = np.zeros(n, dtype=np.uint32)
            st = np.zeros(n, dtype=np.uint8)
            te, td = [], []
            ie = idd = 1               # passes per timed call (amortises thread start-up)
            for r in range(reps + 1):
                t0 = time.perf_counter()
                codec._batch(0, codec.f_encode, t, buf, off, ln, comp, ooff, olen, None, part, ie)
                t1 = time.perf_counter()
                codec._batch(1, codec.f_decode, t, comp, ooff, olen, dec, doff, None, st, part,
                             idd)
                t2 = time.perf_counter()
                if r:                      # run 0 is the warm-up
                    te.append((t1 - t0) / ie)
                    td.append((t2 - t1) / idd)
                else:                      # size the timed calls to >= ~0.2 s each
                    ie = max(1, min(64, int(0.2 / max(t1 - t0, 1e-6)) + 1))
                    idd = max(1, min(64, int(0.2 / max(t2 - t1, 1e-6)) + 1))
            if not bool((st == 1).all()):
                raise RuntimeError("CPU baseline: reference decode rejected its own output")
            e, d = float(np.median(te)), float(np.median(td))
            res[(t, part)] = {"encode_GiBps": raw / e / 2**30, "decode_GiBps": raw / d / 2**30,
                              "roundtrip_GiBps": raw / (e + d) / 2**30,
                              "encode_s_median": e, "decode_s_median": d}
            keep = (comp, ooff, olen)
            del dec
    return {"per_threads": res, "raw_bytes": raw, "comp": keep}
