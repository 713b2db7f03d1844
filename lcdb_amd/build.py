"""Build the native pieces in-tree (gfx950 only).

* ``lcdb_amd/liblcdb_gpu_snappy.so`` -- HIP kernels + C ABI (hipcc,
  ``--offload-arch=gfx950``), declared in ``include/lcdb_gpu_snappy.h``.
* ``lcdb_amd/libcorpus.so`` -- host C generator of db_bench-shaped blocks.
* ``oracle/`` -- the parity checker (``make -C oracle``); test infrastructure
  only, built here so the GPU box receives it prebuilt.

The built ``.so`` files are git-ignored but travel to the GPU box with the
repo snapshot; nothing is JIT-compiled at import time.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "lcdb_amd")
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "liblcdb_gpu_snappy.so")
CORPUS_LIB = os.path.join(PKG, "libcorpus.so")
# Test-only: the product sources plus the decoders that lost their A/B
# (lgs_decode_probe.hip, -DLGS_PROBE_DECODERS).  Never loaded by lcdb or the
# product path; tests/test_gpu_probe_decoders.py runs it in a subprocess.
PROBE_LIB = os.path.join(PKG, "liblcdb_gpu_snappy_probe.so")
PROBE_SOURCES = ["lgs_decode_probe.hip", "lgs_decode_group.hip", "lgs_decode_chain.hip"]

HIP_SOURCES = ["lgs_api.cpp", "lgs_encode_service.hip", "lgs_decode.hip",
               "lgs_table.hip", "lgs_bloom.hip", "lgs_table_index.cpp", "lgs_probe.hip"]
HIP_HEADERS = ["lgs_device.h", "lgs_launch.h", "lgs_decode_common.h", "lgs_probe_hooks.h",
               "lgs_service.h", "lgs_crc.h"]
# Only ldb_snappy_* and lgs_* are exported (the library is loaded into lcdb).
EXPORTS_MAP = os.path.join(CSRC, "exports.map")
# The files that define the two profiled codec kernels and how they are
# launched (grid, LDS class, split); the host runtime, table and bloom
# sources do not change what encode_kernel / decode_ring_kernel execute.
CODEC_KERNEL_FILES = ["lgs_encode.hip", "lgs_encode_service.hip", "lgs_decode.hip", "lgs_device.h", "lgs_launch.h",
                      "lgs_decode_common.h", "lgs_probe_hooks.h", "lgs_service.h"]
ARCH = "gfx950"
# The batch encode kernels only: LLVM's max-ILP machine scheduler (C2 encode
# 538 -> 531 us, profiles/r6v_sched_strategy_ab.txt); the service kernel is
# compiled without it (lgs_encode_service.hip).
ENC_BATCH_FLAGS = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
# If-conversion thresholds: hipcc's defaults leave small two-way branches as
# exec-mask regions; these fold them into selects (the ring decoder's trip:
# 84 -> 70 s_and_saveexec regions; C2 decode 280 -> 274 us, encode unchanged,
# profiles/r4f_session.txt).
FOLD_FLAGS = ["-mllvm", "-phi-node-folding-threshold=8",
              "-mllvm", "-two-entry-phi-node-folding-threshold=16"]


def kernel_sources_sha() -> str:
    """SHA-256 (16 hex) of the codec's kernel sources: PMC traffic figures in
    profiles/traffic_latest.json are only reported by bench.py when they were
    taken from these exact sources."""
    import hashlib
    h = hashlib.sha256()
    for name in sorted(CODEC_KERNEL_FILES):
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    h.update(" ".join(FOLD_FLAGS + ENC_BATCH_FLAGS).encode())
    return h.hexdigest()[:16]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build lcdb_amd)")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def build_hip(force: bool = False, extra: list[str] | None = None, out: str = LIB) -> str:
    """The codec library; `out` / `extra` make probe builds (tools/probe_ab.py).
    The batch encode kernels (lgs_encode.hip) are compiled on their own with
    ENC_BATCH_FLAGS, then linked with everything else."""
    srcs = [os.path.join(CSRC, s) for s in HIP_SOURCES]
    enc = os.path.join(CSRC, "lgs_encode.hip")
    deps = srcs + [enc] + [os.path.join(CSRC, h) for h in HIP_HEADERS] + [EXPORTS_MAP,
        os.path.join(ROOT, "include", "lcdb_gpu_snappy.h")]
    if force or _stale(out, deps):
        tmp = out + ".tmp"
        obj = out + ".enc.o"
        defines = [x for x in (extra or []) if x.startswith("-D")]
        common = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wall", "-Wextra",
                  *FOLD_FLAGS]
        _run([_hipcc(), *common, *ENC_BATCH_FLAGS, "-DLGS_ENCODE_BATCH_ONLY", *defines, "-c", enc,
              "-o", obj])
        _run([_hipcc(), *common, "-shared", "-pthread", f"-Wl,--version-script={EXPORTS_MAP}",
              *srcs, *(extra or []), "-x", "none", obj, "-o", tmp])
        os.replace(tmp, out)
        os.remove(obj)
    return out


def build_probe(force: bool = False) -> str:
    """The probe library (tests only): product sources + lgs_decode_probe.hip."""
    deps = [os.path.join(CSRC, s) for s in PROBE_SOURCES]
    if force or _stale(PROBE_LIB, deps + [LIB]):
        build_hip(force=True, out=PROBE_LIB,
                  extra=["-DLGS_PROBE_DECODERS"] + deps)
    return PROBE_LIB


def build_corpus(force: bool = False) -> str:
    src = os.path.join(CSRC, "corpus.c")
    if force or _stale(CORPUS_LIB, [src]):
        tmp = CORPUS_LIB + ".tmp"
        _run(["gcc", "-std=gnu99", "-O2", "-Wall", "-Wextra", "-fPIC", "-shared", src,
              "-o", tmp])
        os.replace(tmp, CORPUS_LIB)
    return CORPUS_LIB


def build_oracle() -> None:
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def build_lcdb_harness() -> None:
    """lcdb compiled in place + its tests linked to the drop-in (oracle/lcdb.mk);
    a no-op where /root/reference is absent (prebuilt binaries travel)."""
    _run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "oracle"), "-f", "lcdb.mk"])


def build_all(force: bool = False) -> None:
    build_corpus(force)
    build_oracle()
    build_hip(force)
    build_probe(force)
    build_lcdb_harness()


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
