"""lcdb itself on top of the drop-in (BASELINE config 5).

oracle/lcdb.mk compiles lcdb's own sources in place (all but
src/util/snappy.c) and links each program twice: ``.cpu`` with lcdb's
snappy.c, ``.gpu`` with liblcdb_gpu_snappy.so.  The GPU tests run lcdb's
unchanged test suites against the drop-in, and build the same SSTable both
ways through src/builder.c and compare the files byte for byte.  builder.c's
own check (builder.c:96-105) only re-opens the table (footer + index block);
the data blocks are read back separately, through lcdb's ldb_read_block in
oracle/harness/dump_blocks.c, linked both ways.
"""
from __future__ import annotations

import filecmp
import hashlib
import json
import os
import struct
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
    """lcdb's builder on the drop-in, and the batched harness
    (build_table_batched.gpu: one lgs_table_write_host + one
    lgs_table_read_host), both equal lcdb's builder on its own codec."""
    outs = {}
    for kind in ("cpu", "gpu", "batched.gpu"):
        d = tmp_path / kind
        exe = "build_table_batched.gpu" if kind == "batched.gpu" else f"build_table.{kind}"
        r = _run([_bin(exe), str(d), str(entries), str(block_size)], tmp_path)
        assert r.returncode == 0 and "rc=0" in r.stdout, (kind, r.stdout, r.stderr[-2000:])
        outs[kind] = d / "000001.ldb"
    assert os.path.getsize(outs["cpu"]) > 0
    assert filecmp.cmp(outs["cpu"], outs["gpu"], shallow=False)
    assert filecmp.cmp(outs["cpu"], outs["batched.gpu"], shallow=False)


def _sha256(path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for piece in iter(lambda: fh.read(1 << 24), b""):
            h.update(piece)
    return h.hexdigest()


def _run_logged(args, cwd, label, watch=None, budget=1500, env_extra=None):
    """Run a multi-minute harness, logging progress to
    gpurun_out/c5_progress.log every 10 s (a GPU call with no new output for
    3 minutes is taken as hung).  Returns (returncode, stdout, stderr, seconds)."""
    prog_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(prog_dir, exist_ok=True)
    env = dict(os.environ, TEST_TMPDIR=str(cwd), **(env_extra or {}))
    t0 = time.time()
    p = subprocess.Popen(args, cwd=cwd, env=env, stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    with open(os.path.join(prog_dir, "c5_progress.log"), "a") as log:
        while True:
            try:
                stdout, stderr = p.communicate(timeout=10)
                break
            except subprocess.TimeoutExpired:
                size = watch.stat().st_size if watch is not None and watch.exists() else 0
                log.write(f"{time.time() - t0:6.0f} s  {label}: {size} bytes written\n")
                log.flush()
                if time.time() - t0 > budget:
                    p.kill()
    return p.returncode, stdout, stderr, time.time() - t0


def _fields(stdout: str) -> dict:
    """key=value pairs of a harness's result line."""
    out = {}
    for tok in stdout.split():
        if "=" in tok:
            k, v = tok.split("=", 1)
            try:
                out[k] = float(v)
            except ValueError:
                out[k] = v
    return out


def _record(**kv) -> None:
    """Merge timings into gpurun_out/c5_result.json (profiles/ keeps a copy)."""
    p = os.path.join(ROOT, "gpurun_out", "c5_result.json")
    cur = {}
    if os.path.exists(p):
        with open(p) as fh:
            try:
                cur = json.load(fh)
            except ValueError:
                cur = {}
    cur.update(kv)
    with open(p, "w") as fh:
        json.dump(cur, fh, indent=1)


@pytest.fixture(scope="module")
def c5_gpu_table(tmp_path_factory, digests):
    """BASELINE config 5 at its stated size, written once per module by
    src/builder.c through the drop-in: a 2.0 GiB .ldb of 32 768 000 fillseq
    entries (~915 000 data blocks and a 34 MB index block, which goes through
    the drop-in as 527 chunks of 64 KiB and, when builder.c re-opens the
    table, back through the over-slot decode path)."""
    d = digests["C5_table_2GiB"]
    exe = _bin("build_table.gpu")
    tmp = tmp_path_factory.mktemp("c5")
    out = tmp / "gpu"
    rc, stdout, stderr, wall = _run_logged([exe, str(out), str(d["entries"]), str(d["block_size"])],
                                           tmp, "build_table.gpu", out / "000001.ldb")
    assert rc == 0 and "rc=0" in stdout, (stdout, stderr[-2000:])
    return tmp, out / "000001.ldb", wall, _fields(stdout)


@pytest.mark.gpu
def test_c5_2gib_table_through_gpu_dropin(gpu, c5_gpu_table, digests):
    """The drop-in's config-5 table equals the one lcdb's own codec writes
    (size + SHA-256 pinned in digests.json by tests/golden/make_golden.py
    from build_table.cpu)."""
    d = digests["C5_table_2GiB"]
    _, f, wall, fields = c5_gpu_table
    assert f.stat().st_size == d["file_size"]
    assert _sha256(f) == d["sha256"]
    _record(entries=d["entries"], file_size=d["file_size"], sha256_ok=True,
            gpu_dropin_process_seconds=round(wall, 1),
            gpu_dropin_memtable_fill_s=fields.get("fill_s"),
            gpu_dropin_build_table_s=fields.get("build_s"))


@pytest.mark.gpu
def test_c5_cpu_codec_build_time(c5_gpu_table, digests):
    """The same build with lcdb's own snappy.c, timed on the same host beside
    the drop-in's (no GPU used; gpu-marked so both numbers come from the box)."""
    d = digests["C5_table_2GiB"]
    tmp = c5_gpu_table[0]
    out = tmp / "cpu"
    rc, stdout, stderr, wall = _run_logged(
        [_bin("build_table.cpu"), str(out), str(d["entries"]), str(d["block_size"])], tmp,
        "build_table.cpu", out / "000001.ldb")
    assert rc == 0 and "rc=0" in stdout, (stdout, stderr[-2000:])
    f = out / "000001.ldb"
    assert f.stat().st_size == d["file_size"] and _sha256(f) == d["sha256"]
    fields = _fields(stdout)
    _record(cpu_codec_process_seconds=round(wall, 1), cpu_codec_memtable_fill_s=fields.get("fill_s"),
            cpu_codec_build_table_s=fields.get("build_s"))
    f.unlink()


@pytest.mark.gpu
def test_c5_every_block_reads_back_through_dropin(gpu, c5_gpu_table):
    """Every block of the config-5 table (each data block named by the index,
    then the metaindex and the index block) read with lcdb's ldb_read_block,
    checksums verified: through the drop-in (dump_blocks.gpu, one
    ldb_snappy_decode per block) and through lcdb's own codec
    (dump_blocks.cpu) give the same status and content digest for every
    block."""
    tmp, f, _, _ = c5_gpu_table
    res = {}
    for kind in ("cpu", "gpu"):
        out = tmp / f"digests.{kind}"
        rc, stdout, stderr, wall = _run_logged([_bin(f"dump_blocks.{kind}"), str(f), str(out), "1"],
                                               tmp, f"dump_blocks.{kind}", out,
                                               env_extra={"DUMP_DIGEST": "1"})
        assert rc == 0, (kind, stderr[-2000:])
        res[kind] = (out.read_bytes(), wall)
    cpu, gpu_ = res["cpu"][0], res["gpu"][0]
    assert cpu == gpu_
    (count,) = struct.unpack_from("<I", cpu, 40)
    recs = [struct.unpack_from("<QQiIQ", cpu, 44 + 32 * i) for i in range(count)]
    assert len(cpu) == 44 + 32 * count
    assert count > 900000 and all(r[2] == 0 and r[3] > 0 for r in recs)
    _record(readback_blocks=count, readback_dropin_s=round(res["gpu"][1], 1),
            readback_cpu_codec_s=round(res["cpu"][1], 1), readback_identical=True)


@pytest.mark.gpu
def test_c5_batched_table_write_and_read(gpu, c5_gpu_table, digests):
    """Config 5 through the batched entry points (oracle/harness/
    build_table_batched.c): one lgs_table_write_host for every data block,
    lcdb's metaindex / index / footer, one lgs_table_read_host reading every
    data block back.  The file equals the pinned SHA-256 and every block
    reads back as written."""
    d = digests["C5_table_2GiB"]
    tmp = c5_gpu_table[0]
    out = tmp / "batched"
    rc, stdout, stderr, wall = _run_logged(
        [_bin("build_table_batched.gpu"), str(out), str(d["entries"]), str(d["block_size"])], tmp,
        "build_table_batched.gpu", out / "000001.ldb")
    assert rc == 0 and "rc=0" in stdout, (stdout, stderr[-2000:])
    fields = _fields(stdout)
    assert fields["read_bad"] == 0
    f = out / "000001.ldb"
    assert f.stat().st_size == d["file_size"] and _sha256(f) == d["sha256"]
    _record(batched_process_seconds=round(wall, 1),
            **{f"batched_{k}": fields[k] for k in ("blocks", "raw_bytes", "cut_s", "init_s",
                                                   "write_s", "write_warm_s", "finish_s",
                                                   "io_s", "read_s")})
    f.unlink()
