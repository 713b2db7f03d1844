"""lcdb itself on top of the drop-in (BASELINE config 5).

oracle/lcdb.mk compiles lcdb's own sources in place (all but
src/util/snappy.c) and links each program twice: ``.cpu`` with lcdb's
snappy.c, ``.gpu`` with liblcdb_gpu_snappy.so.  The GPU tests run lcdb's
unchanged test suites against the drop-in, and build the same SSTable both
ways through src/builder.c (which also re-reads it through the table cache,
i.e. decodes every block) and compare the files byte for byte.
"""
from __future__ import annotations

import filecmp
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "lcdb")
SUITES = ["snappy", "table", "corruption", "db", "simple", "recovery"]


def _bin(name: str) -> str:
    p = os.path.join(BIN, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (make -C oracle -f lcdb.mk, needs /root/reference)")
    return p


def _run(args, tmp_path, timeout=600):
    env = dict(os.environ, TEST_TMPDIR=str(tmp_path))
    return subprocess.run(args, cwd=tmp_path, env=env, capture_output=True, text=True,
                          timeout=timeout)


@pytest.mark.parametrize("suite", ["snappy", "table"])
def test_reference_suites_pass_with_reference_codec(suite, tmp_path):
    # The harness itself: lcdb's tests pass with lcdb's own codec.
    r = _run([_bin(f"t-{suite}.cpu")], tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]


def test_build_table_cpu_harness(tmp_path):
    r = _run([_bin("build_table.cpu"), str(tmp_path / "db"), "20000"], tmp_path)
    assert r.returncode == 0 and "rc=0" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("suite", SUITES)
def test_reference_suites_pass_with_gpu_dropin(gpu, suite, tmp_path):
    r = _run([_bin(f"t-{suite}.gpu")], tmp_path, timeout=900)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-2000:])


@pytest.mark.gpu
@pytest.mark.parametrize("entries,block_size", [(200000, 4096), (40000, 65536), (3000, 256)])
def test_build_table_gpu_identical_to_cpu(gpu, tmp_path, entries, block_size):
    outs = {}
    for kind in ("cpu", "gpu"):
        d = tmp_path / kind
        r = _run([_bin(f"build_table.{kind}"), str(d), str(entries), str(block_size)], tmp_path)
        assert r.returncode == 0 and "rc=0" in r.stdout, (kind, r.stdout, r.stderr[-2000:])
        outs[kind] = d / "000001.ldb"
    assert os.path.getsize(outs["cpu"]) > 0
    assert filecmp.cmp(outs["cpu"], outs["gpu"], shallow=False)
