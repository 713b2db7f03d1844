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


# Every probe case test_gpu_parity.py defines (its parametrizations over the
# quad, ops, group, chain, trips decoders): the child must pass exactly these,
# so a case that silently stops being collected fails here.
EXPECTED = {
    "test_decode_kernel_variants_golden[quad]", "test_decode_kernel_variants_golden[ops]",
    "test_decode_kernel_variants_golden[group]", "test_decode_kernel_variants_golden[chain]",
    "test_decode_kernels_c2_full_size[kernels1]",
    "test_decode_ring_c3_mixed_and_odd_slots[quad]", "test_decode_ring_c3_mixed_and_odd_slots[ops]",
    "test_decode_ring_c3_mixed_and_odd_slots[group]",
    "test_decode_ops_rejects_overflow_and_jumps",
    "test_decode_in_place_runahead[quad]", "test_decode_in_place_runahead[ops]",
    "test_decode_in_place_runahead[group]", "test_decode_in_place_runahead[chain]",
    "test_decode_wide_far_copies_long_literals_and_rejects[trips]",
    "test_decode_wide_dependent_copies_and_c3[trips]",
    "test_decode_wide_dependent_copies_and_c3[group]",
    "test_decode_small_batch_kernels_and_rejects[group-4608]",
    "test_decode_small_batch_kernels_and_rejects[group-16896]",
    "test_decode_small_batch_kernels_and_rejects[group-66048]",
    "test_decode_small_batch_kernels_and_rejects[chain-4608]",
    "test_decode_small_batch_kernels_and_rejects[chain-16896]",
    "test_op_streams[ops]",
}


def test_probe_decoders_parity():
    env = dict(os.environ, LGS_TEST_PROBE="1")
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-v", "-p", "no:cacheprovider",
                        "-m", "gpu and probe", "--timeout", "300", "--timeout-method", "thread",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1100)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    passed = set(re.findall(r"test_gpu_parity\.py::(\S+) PASSED", r.stdout))
    assert passed == EXPECTED, (sorted(EXPECTED - passed), sorted(passed - EXPECTED), tail)
    assert not re.search(r"\d+ (skipped|failed|error)", r.stdout), tail
