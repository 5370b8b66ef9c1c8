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


def nav_input(a: Arcball, i: int):
    """The scripted navigation input of frame i (examples/sdf_main.cpp nav_input)."""
    dt = 1.0 / 60.0
    ph = i % 90
    if ph < 30:
        return a.update(dt, 0.004, 0.0015, orbit=True)
    if ph < 45:
        return a.update(dt, -0.002, 0.001, pan=True)
    if ph < 60:
        return a.update(dt)
    if ph < 80:
        return a.gamepad(dt, 0.8, -0.5, 0.2, 0.35)
    return a.gamepad(dt, 0.1, 0.0, 0.0, 0.0)


def nav_views(n: int) -> np.ndarray:
    a = Arcball()
    return np.stack([nav_input(a, i) for i in range(n)])


def test_gamepad_deadzone_and_rate():
    a = Arcball()
    a.gamepad(0.5, 0.25, -0.2, 0.0, 0.0)          # inside the 0.30 deadzone: nothing moves
    assert a.yaw == 0.0 and a.pitch == 0.0
    a.gamepad(0.1, 1.0, 0.0, 0.0, 0.65)           # full left stick: 1 rev/s
    assert a.yaw == pytest.approx(2 * math.pi * 0.1)
    assert a.pan_y == pytest.approx(0.1 * (0.65 - 0.3) / 0.7)


def test_cpp_arcball_matches_python():
    """sdf::Arcball (include/sdf3d.hpp), driven by sdf_main's scripted input,
    produces the same V_mat sequence as sdf3d_amd.camera.Arcball, bit for bit
    (mouse orbit and pan drags, release with decay, gamepad sticks)."""
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parent.parent / "sdf3d_amd" / "bin" / "sdf_main"
    assert exe.exists(), "build() must produce sdf3d_amd/bin/sdf_main"
    n = 200
    r = subprocess.run([str(exe), "--views", str(n)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    cpp = np.array([[int(w, 16) for w in line.split()] for line in r.stdout.splitlines()],
                   dtype=np.uint32)
    assert cpp.shape == (n, 16)
    py = nav_views(n).view(np.uint32)
    assert np.array_equal(cpp, py)
    # the sequence really moves: orbit, pan and gamepad phases all change V_mat
    assert len({tuple(v) for v in py}) > n // 2
