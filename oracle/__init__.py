"""CPU oracle for the SDF hot path -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/build/liboracle.so, the plain-C restatement of the
reference fragment shader (/root/reference/Code/shader/voxel_fragment.frag;
see oracle/oracle_core.h for the line-by-line mapping and the parity status:
pinned by analytic known-answer tests only, "parity unpinned" against
reference-produced outputs, because the GLSL reference cannot run here).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / CPU baseline.  The product path
(sdf3d_amd, libsdf3d.so) never imports or calls it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

from sdf3d_amd import abi  # struct layouts of include/sdf_abi.h (types only)

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboracle.so"
# the contracted fp32 reading (FMA-fused multiply-adds, which GLSL permits
# outside `precise`; see oracle/Makefile) -- diagnosis only
FMA_LIB_PATH = HERE / "build" / "liboracle_fma.so"
# the CPU-baseline build (x86-64-v4, same IEEE arithmetic; oracle/Makefile)
BASELINE_LIB_PATH = HERE / "build" / "liboracle_baseline.so"
_libs = {}


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def load(variant: str = "ieee") -> C.CDLL:
    if variant in _libs:
        return _libs[variant]
    path = {"ieee": LIB_PATH, "fma": FMA_LIB_PATH, "baseline": BASELINE_LIB_PATH}[variant]
    if not path.exists():
        build()
    lib = C.CDLL(str(path))
    P = C.POINTER
    frame_args = [P(abi.sdf_scene), P(abi.sdf_camera), P(abi.sdf_light), P(abi.sdf_material),
                  P(abi.sdf_params)]
    lib.sdf_oracle_defaults.argtypes = frame_args + [C.c_int, C.c_int]
    lib.sdf_oracle_defaults.restype = C.c_int
    for fn in (lib.sdf_oracle_render, lib.sdf_oracle_render_f64):
        fn.argtypes = frame_args + [P(abi.sdf_tiling), C.c_void_p, C.c_void_p, C.c_int]
        fn.restype = C.c_int
    lib.sdf_oracle_replay.argtypes = frame_args + [P(abi.sdf_tiling), C.c_void_p, C.c_void_p,
                                                   C.c_void_p, C.c_int]
    lib.sdf_oracle_replay.restype = C.c_int
    if hasattr(lib, "sdf_oracle_render_terms"):
        lib.sdf_oracle_render_terms.argtypes = frame_args + [P(abi.sdf_tiling), C.c_void_p,
                                                             C.c_int]
        lib.sdf_oracle_render_terms.restype = C.c_int
    lib.sdf_oracle_owned_rows.argtypes = [C.c_int, P(abi.sdf_tiling)]
    lib.sdf_oracle_owned_rows.restype = C.c_int
    lib.sdf_oracle_scene_sdf.argtypes = [P(abi.sdf_scene), C.c_float, C.c_float, C.c_float]
    lib.sdf_oracle_scene_sdf.restype = C.c_float
    lib.sdf_oracle_uniforms.argtypes = [P(abi.sdf_camera), P(abi.sdf_params), C.c_void_p]
    lib.sdf_oracle_uniforms.restype = C.c_int
    F3 = C.POINTER(C.c_float)
    lib.sdf_oracle_raymarch.argtypes = [P(abi.sdf_scene), P(abi.sdf_params), F3, F3,
                                        P(C.c_int)]
    lib.sdf_oracle_raymarch.restype = C.c_float
    lib.sdf_oracle_shadow.argtypes = [P(abi.sdf_scene), P(abi.sdf_params), F3, F3, C.c_float,
                                      P(C.c_int)]
    lib.sdf_oracle_shadow.restype = C.c_float
    lib.sdf_oracle_normal.argtypes = [P(abi.sdf_scene), P(abi.sdf_params), F3, F3]
    lib.sdf_oracle_normal.restype = None
    _libs[variant] = lib
    return lib


def _f3(v):
    return (C.c_float * 3)(*[float(x) for x in v])


def raymarch(scene, params, pos, direction):
    """(distance, steps) of the fp32 raymarch (voxel_fragment.frag:86-103)."""
    n = C.c_int(0)
    d = load().sdf_oracle_raymarch(C.byref(scene), C.byref(params), _f3(pos), _f3(direction),
                                   C.byref(n))
    return float(d), n.value


def shadow(scene, params, pos, direction, k=10.0):
    """(shadow, steps) of the fp32 soft shadow (voxel_fragment.frag:105-132)."""
    n = C.c_int(0)
    s = load().sdf_oracle_shadow(C.byref(scene), C.byref(params), _f3(pos), _f3(direction),
                                 float(k), C.byref(n))
    return float(s), n.value


def normal(scene, params, pos):
    out = (C.c_float * 3)()
    load().sdf_oracle_normal(C.byref(scene), C.byref(params), _f3(pos), out)
    return np.array(list(out), dtype=np.float32)


def default_threads() -> int:
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit():
        return max(1, int(n))
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def defaults(width: int = 800, height: int = 600):
    """The oracle's own statement of the reference defaults (5 structs)."""
    s, c, l, m, p = (abi.sdf_scene(), abi.sdf_camera(), abi.sdf_light(), abi.sdf_material(),
                     abi.sdf_params())
    rc = load().sdf_oracle_defaults(C.byref(s), C.byref(c), C.byref(l), C.byref(m), C.byref(p),
                                    width, height)
    assert rc == 0
    return s, c, l, m, p


def owned_rows(height: int, t=None) -> int:
    if t is None:
        return height
    return load().sdf_oracle_owned_rows(height, C.byref(t))


def render(frame, t=None, nthreads: int | None = None, twin: bool = False,
           variant: str = "ieee"):
    """Render `frame` (sdf3d_amd.scenes.Frame) on the CPU.

    Returns (rgba float32 [rows, W, 4], steps int32 [rows, W, 2]).
    `twin=True` runs the fp64 twin (diagnosis only); variant="fma" runs the
    contracted fp32 reading (diagnosis only); variant="baseline" the
    x86-64-v4 build of the IEEE restatement (bench.py's CPU baseline)."""
    lib = load(variant)
    p = frame.params
    rows = owned_rows(p.height, t)
    rgba = np.empty((rows, p.width, 4), dtype=np.float32)
    steps = np.empty((rows, p.width, 2), dtype=np.int32)
    fn = lib.sdf_oracle_render_f64 if twin else lib.sdf_oracle_render
    rc = fn(C.byref(frame.scene), C.byref(frame.camera), C.byref(frame.light),
            C.byref(frame.material), C.byref(frame.params),
            C.byref(t) if t is not None else None,
            rgba.ctypes.data_as(C.c_void_p), steps.ctypes.data_as(C.c_void_p),
            nthreads if nthreads is not None else default_threads())
    if rc != 0:
        raise RuntimeError(f"oracle render failed: {rc}")
    return rgba, steps


def render_terms(frame, t=None, nthreads: int | None = None, variant: str = "ieee"):
    """Each pixel's shading terms (ao, dif, max(N.H, 0), 1) of the fp32
    restatement instead of its colour: the reference of SDF_FORMAT_SHADE32F
    (what the TILES wire carries).  Returns float32 [rows, W, 4]."""
    lib = load(variant)
    p = frame.params
    rows = owned_rows(p.height, t)
    out = np.empty((rows, p.width, 4), dtype=np.float32)
    rc = lib.sdf_oracle_render_terms(C.byref(frame.scene), C.byref(frame.camera),
                                     C.byref(frame.light), C.byref(frame.material),
                                     C.byref(frame.params), C.byref(t) if t is not None else None,
                                     out.ctypes.data_as(C.c_void_p),
                                     nthreads if nthreads is not None else default_threads())
    if rc != 0:
        raise RuntimeError(f"oracle render_terms failed: {rc}")
    return out


def colour_from_terms(frame, terms):
    """The colour from the terms in the restatement's own operation order
    (oracle_core.h shade_pixel, voxel_fragment.frag:204-210): fp32 products
    and sums, pow in fp64 rounded once.  [.., 4] float32 -> [.., 4] float32."""
    f32 = np.float32
    m, li = frame.material, frame.light
    ao, dif, x = (terms[..., i].astype(f32) for i in range(3))
    with np.errstate(all="ignore"):
        spec = np.power(x.astype(np.float64), np.float64(f32(m.shininess))).astype(f32)
        out = np.empty(terms.shape, dtype=f32)
        for c in range(3):
            amb = f32(f32(li.ambient) * f32(m.amb[c]))
            out[..., c] = (f32(amb) * ao + dif * f32(m.dif[c])) + spec * f32(m.ref[c])
    out[..., 3] = 1.0
    return out


def replay(frame, steps, t=None, mask=None, nthreads: int | None = None, variant: str = "ieee"):
    """Forced-step REPLAY (diagnosis only): the fp32 restatement of `frame`
    with each pixel's primary and shadow marches run for exactly the
    iterations in `steps` ([rows, W, 2], e.g. a kernel's recorded counts;
    capped at max_steps) instead of the shader's break tests
    (voxel_fragment.frag:97-99, :126).  Only pixels where `mask` is true are
    evaluated (all if None); the others are NaN with steps -1.

    Returns (rgba float32 [rows, W, 4], steps int32 [rows, W, 2])."""
    lib = load(variant)
    p = frame.params
    rows = owned_rows(p.height, t)
    force = np.ascontiguousarray(np.asarray(steps, dtype=np.int32).reshape(rows, p.width, 2))
    if mask is not None:
        force = force.copy()
        force[~np.asarray(mask, dtype=bool).reshape(rows, p.width), 0] = -2
    rgba = np.full((rows, p.width, 4), np.nan, dtype=np.float32)
    out_steps = np.full((rows, p.width, 2), -1, dtype=np.int32)
    rc = lib.sdf_oracle_replay(C.byref(frame.scene), C.byref(frame.camera), C.byref(frame.light),
                               C.byref(frame.material), C.byref(frame.params),
                               C.byref(t) if t is not None else None,
                               force.ctypes.data_as(C.c_void_p), rgba.ctypes.data_as(C.c_void_p),
                               out_steps.ctypes.data_as(C.c_void_p),
                               nthreads if nthreads is not None else default_threads())
    if rc != 0:
        raise RuntimeError(f"oracle replay failed: {rc}")
    return rgba, out_steps


def scene_sdf(scene, x: float, y: float, z: float) -> float:
    return float(load().sdf_oracle_scene_sdf(C.byref(scene), x, y, z))


def uniforms(camera, params) -> dict:
    out = np.zeros(21, dtype=np.float32)
    rc = load().sdf_oracle_uniforms(C.byref(camera), C.byref(params),
                                    out.ctypes.data_as(C.c_void_p))
    assert rc == 0
    return {"inv_view": out[:16].copy(), "cam": out[16:19].copy(), "focal": float(out[19]),
            "aspect": float(out[20])}
