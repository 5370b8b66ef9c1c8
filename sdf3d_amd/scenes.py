"""Scene, camera and configuration presets.

``reference()`` reproduces the values the reference hard-codes in its shader
(/root/reference/Code/shader/voxel_fragment.frag:15-23, :54-81, :178-189, :205)
through the library's own ``sdf_defaults``.  The other presets are the
BASELINE.json configurations; their scenes are build-defined
extensions with no reference counterpart (DESIGN.md "Scene spec").
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .abi import (FLAG_AO, FLAG_SHADOW, NORMAL_CENTRAL, NORMAL_TETRA, OP_SMOOTH_UNION,
                  OP_UNION, PRIM_BOX, PRIM_CAPSULE, PRIM_CYLINDER, PRIM_PLANE,
                  PRIM_ROUND_BOX, PRIM_SPHERE, PRIM_TORUS, PRECISION_EXACT, PRECISION_FAST,
                  SCENE_MANDELBULB, SCENE_PRIMITIVES)


@dataclass
class Frame:
    """Everything one sdf_render call needs besides the tiling and outputs."""
    scene: abi.sdf_scene
    camera: abi.sdf_camera
    light: abi.sdf_light
    material: abi.sdf_material
    params: abi.sdf_params
    name: str = ""
    meta: dict = field(default_factory=dict)

    def copy(self) -> "Frame":
        def dup(s):
            d = type(s)()
            C.memmove(C.addressof(d), C.addressof(s), C.sizeof(s))
            return d
        return Frame(dup(self.scene), dup(self.camera), dup(self.light), dup(self.material),
                     dup(self.params), self.name, dict(self.meta))


def orbit_view(yaw_deg: float = 0.0, pitch_deg: float = 0.0) -> np.ndarray:
    """V_mat for an orbit about the origin: V = Rx(pitch) * Ry(yaw), returned
    column-major as 16 float32 (GLSL mat4 uniform order).  camera.pos =
    inverse(V) * eye then circles the scene (the reference's arcball produces
    V_mat inside Neutrino: main.cpp:93-94, external)."""
    y, p = math.radians(yaw_deg), math.radians(pitch_deg)
    ry = np.array([[math.cos(y), 0, math.sin(y), 0], [0, 1, 0, 0],
                   [-math.sin(y), 0, math.cos(y), 0], [0, 0, 0, 1]], dtype=np.float64)
    rx = np.array([[1, 0, 0, 0], [0, math.cos(p), -math.sin(p), 0],
                   [0, math.sin(p), math.cos(p), 0], [0, 0, 0, 1]], dtype=np.float64)
    v = rx @ ry
    return v.T.reshape(-1).astype(np.float32)  # column-major


# (yaw, pitch) per seed, SURVEY.md 8(d) "Camera poses"
POSES = [(0.0, 0.0), (15.0, 5.0), (-30.0, 10.0), (60.0, -5.0)]


def set_view(frame: Frame, view16) -> Frame:
    v = np.asarray(view16, dtype=np.float32).reshape(16)
    for i in range(16):
        frame.camera.view[i] = float(v[i])
    return frame


def reference(width: int = 800, height: int = 600) -> Frame:
    """The reference scene and shading exactly (a1-a12 of SURVEY.md 8(a))."""
    lib = abi.load_library()
    f = Frame(abi.sdf_scene(), abi.sdf_camera(), abi.sdf_light(), abi.sdf_material(),
              abi.sdf_params(), name="reference")
    abi.check(lib.sdf_defaults(C.byref(f.scene), C.byref(f.camera), C.byref(f.light),
                               C.byref(f.material), C.byref(f.params), width, height),
              "sdf_defaults")
    return f


def _prim(scene: abi.sdf_scene, i: int, kind: int, op: int, k: float, *p: float) -> None:
    pr = scene.prims[i]
    pr.kind, pr.op, pr.k = kind, op, k
    for j, v in enumerate(p):
        pr.p[j] = v


def set_sphere_only(scene: abi.sdf_scene) -> None:
    """C1: the reference sphere (voxel_fragment.frag:56-59) without the plane."""
    C.memset(C.addressof(scene.prims), 0, C.sizeof(scene.prims))
    scene.kind = SCENE_PRIMITIVES
    scene.count = 1
    _prim(scene, 0, PRIM_SPHERE, OP_UNION, 0.0, 0.0, 0.4, 0.0, 0.2)


CSG8_K = 0.1


def set_csg8(scene: abi.sdf_scene) -> None:
    """C3/C4: 8-primitive smooth-min CSG scene (build-defined).
    The ground plane and the reference sphere keep their reference places."""
    C.memset(C.addressof(scene.prims), 0, C.sizeof(scene.prims))
    scene.kind = SCENE_PRIMITIVES
    scene.count = 8
    k = CSG8_K
    _prim(scene, 0, PRIM_PLANE, OP_UNION, 0.0, 0.0, 1.0, 0.0, 0.0)
    _prim(scene, 1, PRIM_SPHERE, OP_SMOOTH_UNION, k, 0.0, 0.4, 0.0, 0.2)
    _prim(scene, 2, PRIM_BOX, OP_SMOOTH_UNION, k, -0.7, 0.15, -0.3, 0.15, 0.15, 0.15)
    _prim(scene, 3, PRIM_TORUS, OP_SMOOTH_UNION, k, 0.7, 0.1, -0.3, 0.2, 0.06)
    _prim(scene, 4, PRIM_CAPSULE, OP_SMOOTH_UNION, k, -0.35, 0.1, 0.4, 0.05, 0.45, 0.3, 0.07)
    _prim(scene, 5, PRIM_CYLINDER, OP_SMOOTH_UNION, k, 0.45, 0.25, 0.35, 0.12, 0.25)
    _prim(scene, 6, PRIM_ROUND_BOX, OP_SMOOTH_UNION, k, 0.0, 0.12, -0.8, 0.5, 0.12, 0.1, 0.04)
    _prim(scene, 7, PRIM_SPHERE, OP_SMOOTH_UNION, k, 0.25, 0.55, -0.15, 0.12)


def set_mandelbulb(scene: abi.sdf_scene, iterations: int = 12, bailout: float = 2.0) -> None:
    """C5: power-8 Mandelbulb (build-defined)."""
    scene.kind = SCENE_MANDELBULB
    scene.count = 0
    scene.bulb_center[0], scene.bulb_center[1], scene.bulb_center[2] = 0.0, 0.3, 0.0
    scene.bulb_scale = 0.45
    scene.bulb_iterations = iterations
    scene.bulb_bailout = bailout


CONFIGS = {
    # name: (width, height, description)
    "C1": (512, 512, "single sphere, 64 max steps, primary + shadow + shading (CPU plumbing)"),
    "C2": (1920, 1080, "sphere + ground plane, 128 steps, primary rays only"),
    "C3": (1920, 1080, "8-primitive smooth-min CSG + soft shadow + 5-tap AO + tetra normals"),
    "C4": (3840, 2160, "8-primitive smooth-min CSG + soft shadow + 5-tap AO + tetra normals, "
                       "3840x2160"),
    "C5": (3840, 2160, "Mandelbulb power 8, 12-iteration DE, shadow + AO + tetra normals"),
    "REF": (800, 600, "the reference shader exactly (plane + sphere, 100 steps, shadow)"),
}


def config(name: str, width: int | None = None, height: int | None = None,
           precision: int = PRECISION_EXACT, pose: int = 0) -> Frame:
    """Build a configuration preset (optionally at another resolution)."""
    w0, h0, desc = CONFIGS[name]
    w, h = width or w0, height or h0
    f = reference(w, h)
    f.name = name
    f.meta["description"] = desc
    p = f.params
    if name == "C1":
        set_sphere_only(f.scene)
        p.max_steps = 64
    elif name == "C2":
        p.max_steps = 128
        p.flags = 0
    elif name in ("C3", "C4"):
        set_csg8(f.scene)
        p.max_steps = 128
        p.flags = FLAG_SHADOW | FLAG_AO
        p.normal_mode = NORMAL_TETRA
    elif name == "C5":
        set_mandelbulb(f.scene)
        p.max_steps = 128
        p.flags = FLAG_SHADOW | FLAG_AO
        p.normal_mode = NORMAL_TETRA
    elif name != "REF":
        raise KeyError(name)
    p.precision = precision
    if pose:
        set_view(f, orbit_view(*POSES[pose]))
    f.meta["pose"] = pose
    return f


__all__ = ["Frame", "orbit_view", "POSES", "reference", "config", "CONFIGS", "set_view",
           "set_sphere_only", "set_csg8", "set_mandelbulb", "PRECISION_EXACT", "PRECISION_FAST",
           "NORMAL_CENTRAL", "NORMAL_TETRA"]
