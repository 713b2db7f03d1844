"""The C-ABI library loads and exports every symbol include/*.h declares;
host-only entry points (size bound, size header) match the oracle.  No GPU
compute happens here."""
from __future__ import annotations

import glob
import os
import re
import subprocess

import oracle
from lcdb_amd import _native, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared() -> set[str]:
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\([^;{]*\)\s*;", text, re.M):
            names.add(m.group(1))
    return names


def _dynsyms(path: str) -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_header_declares_dropin_and_batch():
    d = _declared()
    for name in ("ldb_snappy_encode_size", "ldb_snappy_encode", "ldb_snappy_decode_size",
                 "ldb_snappy_decode", "lgs_encode_batch_dev", "lgs_decode_batch_dev"):
        assert name in d
    assert d == set(_native.EXPORTED)


def test_library_exports_every_declared_symbol():
    syms = _dynsyms(build.LIB)
    missing = _declared() - syms
    assert not missing, missing
    lib = _native.lib()
    for name in _declared():
        assert getattr(lib, name) is not None


def test_library_exports_only_the_c_abi():
    # The library is loaded into lcdb's process: nothing but the drop-in
    # (ldb_snappy_*) and the batched ABI (lgs_*) may be exported, so no
    # helper can interpose on the host's symbols (lcdb_amd/csrc/exports.map).
    extra = {s for s in _dynsyms(build.LIB) if not s.startswith(("ldb_snappy_", "lgs_"))}
    assert not extra, sorted(extra)[:20]
    assert _dynsyms(build.LIB) == _declared()


def test_product_does_not_link_the_oracle():
    syms = _dynsyms(build.LIB)
    assert not any(s.startswith(("oracle_", "cpu_batch")) for s in syms)
    ldd = subprocess.run(["ldd", build.LIB], capture_output=True, text=True).stdout
    assert "oracle" not in ldd and "libref_snappy" not in ldd


def test_gfx950_code_object():
    blob = open(build.LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"--gfx9" not in blob.replace(b"--gfx950", b"")   # gfx950 only


def test_host_side_size_functions_match_oracle(vectors):
    from lcdb_amd import snappy  # loads the library; size calls need no GPU
    orc = oracle.restatement()
    for n in (0, 1, 16, 17, 4096, 65536, 1 << 20, 0x7FFFFFFF, 0x80000000, 1 << 40):
        assert snappy.encode_size(n) == orc.encode_size(n)
    for v in vectors:
        s = v.a if v.kind == 1 else v.b
        assert snappy.decode_size(s) == orc.decode_size(s), v.name


def test_host_side_bloom_and_filter_block_sizes_match_oracle():
    """lgs_bloom_filter_size equals the reference filter's length, and
    lgs_filter_block_bound covers every filter block the oracle builds
    (pure host functions: no GPU)."""
    import random

    from lcdb_amd import bloom
    from test_bloom_oracle import random_table_layout
    orc = oracle.bloom_restatement()
    for n in (0, 1, 5, 36, 1000):
        for bpk in (0, 1, 10, 16, 50):
            keys = [b"%08d" % k for k in range(n)]
            want = len(orc.build(keys, bpk)) if n else 0
            assert bloom.filter_size(n, bpk) == want, (n, bpk)
    rng = random.Random(9)
    for _ in range(200):
        internal = rng.random() < 0.5
        blocks, off, end = random_table_layout(rng, internal)
        bpk = rng.choice([0, 1, 10, 16, 44])
        fb = orc.filter_block(blocks, off, end, bpk, internal)
        nkeys = sum(len(b) for b in blocks)
        assert len(fb) <= bloom.filter_block_bound(nkeys, len(blocks), end, bpk)
        assert bloom.filter_block_scratch(end) > 0


def test_integration_recipe_names_the_built_sources():
    """INTEGRATION.md §1's hand-written hipcc line compiles exactly the
    sources build.py compiles, with the export map, and every one exists."""
    import re

    from lcdb_amd import build
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index("## 1. Build the library"):text.index("## 2.")]
    named = re.findall(r"lcdb_amd/csrc/(\w+\.(?:cpp|hip))", block)
    assert sorted(named) == sorted(build.HIP_SOURCES + ["lgs_encode.hip"])   # + the batch object
    assert "--version-script=lcdb_amd/csrc/exports.map" in block
    for s in named:
        assert os.path.exists(os.path.join(ROOT, "lcdb_amd", "csrc", s))


def test_product_has_only_the_kept_decoders():
    """the decoders that lost their A/B (quad, two-pass, trips)
    live in the probe library only.  The product library neither contains
    their kernels nor accepts their options (lgs_set_option needs no GPU)."""
    blob = open(build.LIB, "rb").read()
    for k in (b"decode_quad_kernel", b"tag_scan_kernel", b"op_exec_kernel",
              b"decode_trips_kernel", b"decode_group_kernel", b"decode_chain_kernel"):
        assert k not in blob, k
    for k in (b"decode_ring_kernel", b"decode_wide_kernel", b"decode_kernel"):
        assert k in blob, k
    lib = _native.lib()
    for name, value in (("decoder", "quad"), ("decoder", "ops"), ("decoder", "group"),
                        ("decoder", "chain"), ("wide", "trips"), ("wide", "group")):
        assert lib.lgs_set_option(name.encode(), value.encode()) == _native.LGS_EINVAL, value
    for name, value in (("decoder", "ring"), ("decoder", "wave"), ("decoder", "auto"),
                        ("wide", "walk")):
        assert lib.lgs_set_option(name.encode(), value.encode()) == _native.LGS_OK, value
    probe = open(build.PROBE_LIB, "rb").read()
    assert b"decode_quad_kernel" in probe and b"op_exec_kernel" in probe
    assert b"decode_group_kernel" in probe and b"decode_chain_kernel" in probe


def test_service_option_and_kernels():
    """The drop-in service: its two resident kernels are in the
    product, and lgs_set_option("service", ...) takes 0 or 1 only (no GPU)."""
    blob = open(build.LIB, "rb").read()
    assert b"encode_service_kernel" in blob and b"decode_service_kernel" in blob
    lib = _native.lib()
    for v in ("2", "", "on"):
        assert lib.lgs_set_option(b"service", v.encode()) == _native.LGS_EINVAL, v
    for v in ("0", "1"):
        assert lib.lgs_set_option(b"service", v.encode()) == _native.LGS_OK, v
