"""Shared pytest setup.

Markers: ``gpu`` = needs an MI355X (the driver runs ``-m gpu`` on the GPU box
and ``-m "not gpu"`` here).  Native libraries are built in-tree on first use
if missing (hipcc cross-compiles for gfx950 without a GPU).
"""
from __future__ import annotations

import json
import os
import sys

import pytest

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

import golden_io  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: multi-second CPU test")
    config.addinivalue_line("markers", "probe: covers a probe-library decoder (LGS_TEST_PROBE=1)")


def _ensure_built():
    from lcdb_amd import build
    need = [build.LIB, build.PROBE_LIB, build.CORPUS_LIB,
            os.path.join(ROOT, "oracle", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        build.build_all()


_ensure_built()

if os.environ.get("LGS_TEST_PROBE") == "1":
    # tests/test_gpu_probe_decoders.py: this process tests the probe library
    # (product sources + the decoders that lost their A/B).
    from lcdb_amd import build as _build
    _build.LIB = _build.PROBE_LIB


@pytest.fixture(scope="session")
def vectors():
    return golden_io.read()


@pytest.fixture(scope="session")
def digests():
    with open(golden_io.DIGESTS) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu():
    """The GPU codec module; fails (never skips) when no device is visible."""
    from lcdb_amd import _native
    n = _native.lib().lgs_device_count()
    if n <= 0:
        pytest.fail("gpu test needs a visible MI355X (lgs_device_count() == 0)")
    from lcdb_amd import snappy
    return snappy


@pytest.fixture
def force():
    """force(name, value): lgs_set_option for one test, reset afterwards."""
    from lcdb_amd import _native
    touched = []

    def set_(name: str, value: str) -> None:
        _native.set_option(name, value)
        touched.append(name)

    yield set_
    for name in touched:
        _native.set_option(name, {"decoder": "auto", "split": "1", "wide": "walk", "service": "1",
                             "verify_overlap": "1"}[name])
