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
import hashlib
import json
import os
import subprocess
import time

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


@pytest.mark.gpu
def test_c5_2gib_table_through_gpu_dropin(gpu, tmp_path, digests):
    """BASELINE config 5 at its stated size: src/builder.c writes a 2.0 GiB
    .ldb (32 768 000 fillseq entries, ~915 000 data blocks, a 34 MB index
    block = 527 chunks of 64 KiB) through the drop-in, re-opens it through
    the table cache and iterates it (builder.c:99, every block decoded,
    the index block through the over-slot path); the file must equal the one
    lcdb's own codec writes (size + SHA-256 pinned in digests.json by
    tests/golden/make_golden.py from build_table.cpu).  The build takes
    minutes, so progress goes to gpurun_out/c5_progress.log."""
    d = digests["C5_table_2GiB"]
    exe = _bin("build_table.gpu")
    out = tmp_path / "gpu"
    prog_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(prog_dir, exist_ok=True)
    progress = os.path.join(prog_dir, "c5_progress.log")
    env = dict(os.environ, TEST_TMPDIR=str(tmp_path))
    t0 = time.time()
    p = subprocess.Popen([exe, str(out), str(d["entries"]), str(d["block_size"])], cwd=tmp_path,
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    f = out / "000001.ldb"
    with open(progress, "a") as log:
        while p.poll() is None:
            time.sleep(10)
            size = f.stat().st_size if f.exists() else 0
            log.write(f"{time.time() - t0:6.0f} s  build_table.gpu: {size} bytes written\n")
            log.flush()
            if time.time() - t0 > 1500:
                p.kill()
    stdout, stderr = p.communicate()
    wall = time.time() - t0
    assert p.returncode == 0 and "rc=0" in stdout, (stdout, stderr[-2000:])
    assert f.stat().st_size == d["file_size"]
    h = hashlib.sha256()
    with open(f, "rb") as fh:
        for piece in iter(lambda: fh.read(1 << 24), b""):
            h.update(piece)
    assert h.hexdigest() == d["sha256"]
    with open(os.path.join(prog_dir, "c5_result.json"), "w") as fh:
        json.dump({"entries": d["entries"], "file_size": d["file_size"], "sha256_ok": True,
                   "build_and_verify_seconds": round(wall, 1)}, fh)
