"""Arcball navigation producing the V_mat uniform.

The reference gets V_mat from Neutrino's mouse and gamepad navigation
(/root/reference/Code/src/main.cpp:37-45 rates, :93-94 calls), whose
implementation is external and not vendored: the dynamics below are this
framework's own (parity unpinned).  Orbit and pan follow the input while it
is active and keep their velocity afterwards, decaying with the given time
constant (the reference's `ms_decaytime`).
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
        """Advance by dt seconds with a pointer motion (dx, dy) in normalised
        screen units; returns V_mat (16 float32, column-major)."""
        if dt > 0:
            if orbit:
                self._vyaw, self._vpitch = self.orbit_rate * dx / dt, self.orbit_rate * dy / dt
            if pan:
                self._vpx, self._vpy = self.pan_rate * dx / dt, self.pan_rate * dy / dt
            self.yaw += self._vyaw * dt
            self.pitch = max(-math.pi / 2, min(math.pi / 2, self.pitch + self._vpitch * dt))
            self.pan_x += self._vpx * dt
            self.pan_y += self._vpy * dt
            if not orbit or not pan:
                decay = math.exp(-dt / self.decay_time) if self.decay_time > 0 else 0.0
                if not orbit:
                    self._vyaw *= decay
                    self._vpitch *= decay
                if not pan:
                    self._vpx *= decay
                    self._vpy *= decay
        return self.view()

    def view(self) -> np.ndarray:
        """V_mat = T(pan) * Rx(pitch) * Ry(yaw), column-major float32."""
        cy, sy = math.cos(self.yaw), math.sin(self.yaw)
        cp, sp = math.cos(self.pitch), math.sin(self.pitch)
        ry = np.array([[cy, 0, sy, 0], [0, 1, 0, 0], [-sy, 0, cy, 0], [0, 0, 0, 1]])
        rx = np.array([[1, 0, 0, 0], [0, cp, -sp, 0], [0, sp, cp, 0], [0, 0, 0, 1]])
        t = np.eye(4)
        t[0, 3], t[1, 3] = self.pan_x, self.pan_y
        return (t @ rx @ ry).T.reshape(-1).astype(np.float32)
