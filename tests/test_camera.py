"""Arcball navigation (sdf3d_amd.camera): V_mat stays a rigid transform,
orbit keeps the camera distance, motion decays with the reference's decay
time constant (main.cpp:39)."""
import math

import numpy as np
import pytest

import oracle
from sdf3d_amd import scenes
from sdf3d_amd.camera import Arcball


def test_starts_at_identity():
    assert np.array_equal(Arcball().view(), np.eye(4, dtype=np.float32).reshape(-1))


def test_orbit_is_rotation_and_keeps_distance():
    a = Arcball()
    v = a.update(0.016, dx=0.1, dy=0.05, orbit=True)
    m = v.reshape(4, 4).T.astype(np.float64)
    assert np.allclose(m[:3, :3] @ m[:3, :3].T, np.eye(3), atol=1e-6)
    f = scenes.reference(32, 18)
    scenes.set_view(f, v)
    u = oracle.uniforms(f.camera, f.params)
    assert np.linalg.norm(u["cam"]) == pytest.approx(math.hypot(0.2, 2.0), rel=1e-5)


def test_release_decays_velocity():
    a = Arcball()
    a.update(0.016, dx=0.1, orbit=True)
    y0 = a.yaw
    a.update(1.25)                        # one decay time without input
    assert a.yaw > y0 and abs(a._vyaw) == pytest.approx(0.1 / 0.016 * math.exp(-1), rel=1e-6)


def test_pan_translates_view():
    a = Arcball()
    v = a.update(0.1, dx=0.02, dy=-0.01, pan=True)
    m = v.reshape(4, 4).T
    assert m[0, 3] == pytest.approx(5.0 * 0.02) and m[1, 3] == pytest.approx(5.0 * -0.01)
