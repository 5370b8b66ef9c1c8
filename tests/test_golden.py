"""The golden fixtures (tests/golden/, made by make_golden.py from the oracle)
are frozen by SHA-256; the oracle must keep reproducing them bit for bit, and
its fp64 twin must agree with it under the parity policy (a restatement that
is numerically unstable would fail here before it fails on the GPU)."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
from parity import assert_parity, compare
from golden.make_golden import FIXTURES, frame_for

GOLD = Path(__file__).resolve().parent / "golden"
MANIFEST = json.loads((GOLD / "MANIFEST.json").read_text())


def load_fixture(name):
    z = np.load(GOLD / f"{name}.npz")
    return z["rgba"], z["steps"]


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_fixture_integrity_and_oracle_reproduces(name):
    rgba, steps = load_fixture(name)
    m = MANIFEST[name]
    assert hashlib.sha256(rgba.tobytes()).hexdigest() == m["sha256_rgba"]
    assert hashlib.sha256(steps.tobytes()).hexdigest() == m["sha256_steps"]
    r2, s2 = oracle.render(frame_for(name), nthreads=2)
    assert np.array_equal(r2.view(np.uint32), rgba.view(np.uint32))
    assert np.array_equal(s2, steps)


@pytest.mark.parametrize("name", ["ref_160x90_p0", "c3_160x90_p0", "c2_160x90_p0"])
def test_fp64_twin_agrees(name):
    rgba, steps = load_fixture(name)
    t64, s64 = oracle.render(frame_for(name), twin=True)
    # outliers must be explained by the fp32 oracle stopped at the twin's
    # own step counts (forced-step replay, parity.py)
    rep = compare(frame_for(name), t64, s64, rgba, steps)
    assert_parity(rep, what=name)


def test_oracle_threads_deterministic():
    f = frame_for("c3_160x90_p0")
    a, sa = oracle.render(f, nthreads=1)
    b, sb = oracle.render(f, nthreads=4)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(sa, sb)


def test_baseline_build_is_the_same_oracle():
    """bench.py's CPU baseline runs the x86-64-v4 build of the oracle
    (oracle/Makefile): the same IEEE arithmetic, so the same frame bit for
    bit (skipped on a host without AVX-512)."""
    import pytest
    if "avx512f" not in open("/proc/cpuinfo").read():
        pytest.skip("host CPU lacks AVX-512")
    from sdf3d_amd import scenes
    f = scenes.config("C3", 96, 54, pose=1)
    a, sa = oracle.render(f)
    b, sb = oracle.render(f, variant="baseline")
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(sa, sb)
