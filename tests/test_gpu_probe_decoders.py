"""The decoders that lost their A/B against the reference.

They are compiled only into the probe library
(lcdb_amd/liblcdb_gpu_snappy_probe.so: lgs_decode_probe.hip, built by
build.py with -DLGS_PROBE_DECODERS), never into the product that lcdb loads.
Their parity tests are test_gpu_parity.py's own, parametrized over the probe
decoders when LGS_TEST_PROBE=1: this test runs them in a child process that
loads the probe library instead of the product (conftest.py), so the two
libraries never share a process.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_probe_decoders_parity():
    env = dict(os.environ, LGS_TEST_PROBE="1")
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        "-m", "gpu and probe", "--timeout", "300", "--timeout-method", "thread",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1100)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    m = re.search(r"(\d+) passed", r.stdout)
    # quad and ops: golden, C2 (one test), C3, runahead; ops rejects; trips: two wide
    assert m and int(m.group(1)) >= 10, tail
    assert not re.search(r"\d+ (skipped|failed|error)", r.stdout), tail
