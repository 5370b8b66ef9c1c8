"""Arcball navigation producing the V_mat uniform.

The reference gets V_mat from Neutrino's mouse and gamepad navigation
(/root/reference/Code/src/main.cpp:37-45 rates, :93-94 calls), whose
implementation is external and not vendored: the dynamics below are this
framework's own (parity unpinned).  Orbit and pan follow the input while it
is active and keep their velocity afterwards, decaying with the given time
constant (the reference's `ms_decaytime` / `gmp_decaytime`); a gamepad stick
inside the deadzone (`gmp_deadzone`) counts as released.  The C++ host API
(include/sdf3d.hpp sdf::Arcball) computes the same sequence bit for bit
(tests/test_camera.py runs both).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


@dataclass
class Arcball:
    orbit_rate: float = 1.0      # main.cpp:37 ms_orbit_rate
    pan_rate: float = 5.0        # main.cpp:38 ms_pan_rate
    decay_time: float = 1.25     # main.cpp:39 ms_decaytime (s)
    pad_orbit_rate: float = 1.0  # main.cpp:42 gmp_orbit_rate (rev/s)
    pad_pan_rate: float = 1.0    # main.cpp:43 gmp_pan_rate
    pad_decay_time: float = 1.25  # main.cpp:44 gmp_decaytime (s)
    pad_deadzone: float = 0.30   # main.cpp:45 gmp_deadzone
    yaw: float = 0.0             # radians
    pitch: float = 0.0
    pan_x: float = 0.0
    pan_y: float = 0.0
    _vyaw: float = 0.0
    _vpitch: float = 0.0
    _vpx: float = 0.0
    _vpy: float = 0.0

    def update(self, dt: float, dx: float = 0.0, dy: float = 0.0, orbit: bool = False,
               pan: bool = False) -> np.ndarray:
        """Mouse: advance by dt seconds with a pointer motion (dx, dy) in
        normalised screen units; returns V_mat (16 float32, column-major)."""
        if dt > 0:
            if orbit:
                self._vyaw, self._vpitch = self.orbit_rate * dx / dt, self.orbit_rate * dy / dt
            if pan:
                self._vpx, self._vpy = self.pan_rate * dx / dt, self.pan_rate * dy / dt
            self._integrate(dt, not orbit, not pan, self.decay_time)
        return self.view()

    def gamepad(self, dt: float, lx: float = 0.0, ly: float = 0.0, rx: float = 0.0,
                ry: float = 0.0) -> np.ndarray:
        """Gamepad: left stick (lx, ly) orbits at pad_orbit_rate rev/s, right
        stick (rx, ry) pans at pad_pan_rate, values in [-1, 1] rescaled from
        [deadzone, 1] to [0, 1]; returns V_mat."""
        if dt > 0:
            ax, ay, bx, by = (self._dead(v) for v in (lx, ly, rx, ry))
            orbit, pan = ax != 0.0 or ay != 0.0, bx != 0.0 or by != 0.0
            two_pi = 2.0 * math.pi
            if orbit:
                self._vyaw = self.pad_orbit_rate * two_pi * ax
                self._vpitch = self.pad_orbit_rate * two_pi * ay
            if pan:
                self._vpx, self._vpy = self.pad_pan_rate * bx, self.pad_pan_rate * by
            self._integrate(dt, not orbit, not pan, self.pad_decay_time)
        return self.view()

    def _dead(self, a: float) -> float:
        z, m = self.pad_deadzone, abs(a)
        if not m > z:
            return 0.0
        return math.copysign(min((m - z) / (1.0 - z), 1.0), a)

    def _integrate(self, dt, decay_orbit, decay_pan, tau):
        self.yaw += self._vyaw * dt
        self.pitch = max(-math.pi / 2, min(math.pi / 2, self.pitch + self._vpitch * dt))
        self.pan_x += self._vpx * dt
        self.pan_y += self._vpy * dt
        if decay_orbit or decay_pan:
            k = math.exp(-dt / tau) if tau > 0 else 0.0
            if decay_orbit:
                self._vyaw *= k
                self._vpitch *= k
            if decay_pan:
                self._vpx *= k
                self._vpy *= k

    def view(self) -> np.ndarray:
        """V_mat = T(pan) * Rx(pitch) * Ry(yaw), column-major float32 (each
        element one product, rounded once, as sdf::Arcball::view)."""
        cy, sy = math.cos(self.yaw), math.sin(self.yaw)
        cp, sp = math.cos(self.pitch), math.sin(self.pitch)
        m = np.array([[cy, 0.0, sy, self.pan_x], [sp * sy, cp, -sp * cy, self.pan_y],
                      [-cp * sy, sp, cp * cy, 0.0], [0.0, 0.0, 0.0, 1.0]], dtype=np.float64)
        return m.T.reshape(-1).astype(np.float32)
