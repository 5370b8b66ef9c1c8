"""ctypes mirror of ``include/sdf_abi.h`` and the loader for ``libsdf3d.so``.

The struct layouts here must match the C header byte for byte;
``tests/test_abi.py`` checks every size against the C library's own view.
The loader raises if the in-tree HIP library is missing: there is no CPU
fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

SDF_ABI_VERSION = 11
MAX_DECODE_PARTS = 64   # SDF_MAX_DECODE_PARTS
SDF_MAX_PRIMS = 16

# status codes
SDF_OK = 0
SDF_E_INVALID_ARG = -1
SDF_E_UNSUPPORTED = -2
SDF_E_HIP = -3
SDF_E_NO_DEVICE = -4
SDF_E_COMM = -5
SDF_E_TIMEOUT = -6
COMM_ID_BYTES = 128
DRIVER_ROOT_AS_PEER = 0x1

# primitive kinds
PRIM_SPHERE, PRIM_PLANE, PRIM_BOX, PRIM_ROUND_BOX, PRIM_TORUS, PRIM_CAPSULE, PRIM_CYLINDER = range(7)
PRIM_NAMES = ["sphere", "plane", "box", "round_box", "torus", "capsule", "cylinder"]
# CSG ops
OP_UNION, OP_SMOOTH_UNION, OP_SUBTRACT, OP_INTERSECT, OP_SMOOTH_SUBTRACT, OP_SMOOTH_INTERSECT = range(6)
OP_COUNT = 6
OP_NAMES = ["union", "smooth_union", "subtract", "intersect", "smooth_subtract", "smooth_intersect"]
# scene kinds
SCENE_PRIMITIVES, SCENE_MANDELBULB = 0, 1
# flags / modes
FLAG_SHADOW, FLAG_AO = 0x1, 0x2
NORMAL_CENTRAL, NORMAL_TETRA = 0, 1
PRECISION_EXACT, PRECISION_FAST = 0, 1
DISPATCH_AUTO, DISPATCH_GENERIC, DISPATCH_UNCULLED = 0, 1, 2
FORMAT_RGBA32F, FORMAT_RGBA16F, FORMAT_RGBA8, FORMAT_RGB32F, FORMAT_TILES = 0, 1, 2, 3, 4
FORMAT_SHADE32F = 5   # the pixels' shading terms (ao, dif, x, 1): what TILES carries
TILING_FRAME_ROWS = 1
FORMAT_NAMES = {"rgba32f": FORMAT_RGBA32F, "rgba16f": FORMAT_RGBA16F, "rgba8": FORMAT_RGBA8,
                "rgb32f": FORMAT_RGB32F, "shade32f": FORMAT_SHADE32F}
# TILES (the frame losslessly compressed, the multi-device wire) is a byte
# stream of per-frame length, not a pixel format: see Renderer.alloc
FORMAT_CHANNELS = {FORMAT_RGBA32F: 4, FORMAT_RGBA16F: 4, FORMAT_RGBA8: 4, FORMAT_RGB32F: 3,
                   FORMAT_SHADE32F: 4}
TILES_HEADER_BYTES = 64   # used, ntiles, shade mode, 0, shading constants (sdf_abi.h)
# sdf_tiles_decode_checked status bits (sdf_abi.h SDF_TILES_BAD_*)
TILES_BAD_HEADER, TILES_BAD_TILE, TILES_BAD_FIELD = 0x1, 0x100, 0x10000


class sdf_primitive(C.Structure):
    _fields_ = [("kind", C.c_int32), ("op", C.c_int32), ("k", C.c_float),
                ("reserved", C.c_float), ("p", C.c_float * 12)]


class sdf_scene(C.Structure):
    _fields_ = [("kind", C.c_int32), ("count", C.c_int32),
                ("prims", sdf_primitive * SDF_MAX_PRIMS),
                ("bulb_center", C.c_float * 3), ("bulb_scale", C.c_float),
                ("bulb_iterations", C.c_int32), ("bulb_bailout", C.c_float),
                ("reserved", C.c_int32 * 2)]


class sdf_camera(C.Structure):
    _fields_ = [("view", C.c_float * 16), ("eye", C.c_float * 3), ("fov_deg", C.c_float),
                ("aspect", C.c_float), ("pi", C.c_float)]


class sdf_light(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("ambient", C.c_float), ("color", C.c_float * 3),
                ("reserved", C.c_float)]


class sdf_material(C.Structure):
    _fields_ = [("amb", C.c_float * 3), ("dif", C.c_float * 3), ("ref", C.c_float * 3),
                ("shininess", C.c_float)]


class sdf_params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("max_steps", C.c_int32),
                ("max_dist", C.c_float), ("eps", C.c_float), ("shadow_k", C.c_float),
                ("normal_eps", C.c_float), ("shadow_offset", C.c_float),
                ("flags", C.c_int32), ("normal_mode", C.c_int32), ("ao_taps", C.c_int32),
                ("ao_step", C.c_float), ("ao_base", C.c_float), ("ao_falloff", C.c_float),
                ("ao_strength", C.c_float), ("precision", C.c_int32),
                ("dispatch", C.c_int32), ("output_format", C.c_int32),
                ("reserved", C.c_int32 * 2)]


class sdf_tiling(C.Structure):
    _fields_ = [("block_rows", C.c_int32), ("first_block", C.c_int32),
                ("block_stride", C.c_int32), ("flags", C.c_int32),
                ("block_run", C.c_int32), ("run_step", C.c_int32)]


class sdf_driver_config(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("share_root", C.c_int32),
                ("share_peer", C.c_int32), ("nbuf", C.c_int32), ("lag", C.c_int32),
                ("flags", C.c_int32), ("timeout_ms", C.c_int32), ("batch", C.c_int32)]


STRUCT_SIZES = {
    "sdf_primitive": 64, "sdf_scene": 8 + 64 * SDF_MAX_PRIMS + 32, "sdf_camera": 88,
    "sdf_light": 32, "sdf_material": 40, "sdf_params": 80, "sdf_tiling": 24,
    "sdf_driver_config": 36,
}

# every entry point of include/sdf_abi.h: name -> (restype, argtypes)
_P = C.POINTER
SIGNATURES = {
    "sdf_abi_version": (C.c_int, []),
    "sdf_defaults": (C.c_int, [_P(sdf_scene), _P(sdf_camera), _P(sdf_light), _P(sdf_material),
                               _P(sdf_params), C.c_int32, C.c_int32]),
    "sdf_validate": (C.c_int, [_P(sdf_scene), _P(sdf_camera), _P(sdf_light), _P(sdf_material),
                               _P(sdf_params), _P(sdf_tiling)]),
    "sdf_owned_rows": (C.c_int, [C.c_int32, _P(sdf_tiling)]),
    "sdf_share_tiling": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P(sdf_tiling)]),
    "sdf_render": (C.c_int, [_P(sdf_scene), _P(sdf_camera), _P(sdf_light), _P(sdf_material),
                             _P(sdf_params), _P(sdf_tiling), C.c_void_p, C.c_void_p, C.c_void_p]),
    "sdf_deinterleave": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                   C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "sdf_format_bytes": (C.c_int, [C.c_int32]),
    "sdf_tiles_bytes": (C.c_int64, [C.c_int32, C.c_int32]),
    "sdf_jit_count": (C.c_int, []),
    "sdf_kernel_id": (C.c_char_p, [C.c_int32]),
    "sdf_scene_bounds": (C.c_int, [_P(sdf_scene), _P(C.c_float), _P(C.c_float), _P(C.c_int32)]),
    "sdf_tiles_decode": (C.c_int, [C.c_void_p, C.c_int32, C.c_int64, C.c_int32, C.c_int32,
                                   C.c_int32, C.c_void_p, C.c_void_p]),
    "sdf_tiles_decode_tilings": (C.c_int, [C.c_void_p, C.c_int32, C.c_int64, _P(sdf_tiling),
                                           C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "sdf_schedule_create": (C.c_int, [C.c_int32, C.c_int32, _P(C.c_void_p)]),
    "sdf_schedule_destroy": (C.c_int, [C.c_void_p]),
    "sdf_schedule_order": (C.c_int, [C.c_void_p, _P(C.c_int32), C.c_int32]),
    "sdf_render_scheduled": (C.c_int, [_P(sdf_scene), _P(sdf_camera), _P(sdf_light),
                                       _P(sdf_material), _P(sdf_params), _P(sdf_tiling),
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sdf_tiles_decode_checked": (C.c_int, [C.c_void_p, C.c_int32, C.c_int64, _P(sdf_tiling),
                                           _P(C.c_int64), C.c_int32, C.c_int32, C.c_void_p,
                                           C.c_void_p, C.c_void_p]),
    "sdf_heatmap": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                              C.c_void_p, C.c_void_p]),
    "sdf_render_multi": (C.c_int, [_P(sdf_scene), _P(sdf_camera), _P(sdf_light),
                                   _P(sdf_material), _P(sdf_params), C.c_int32, C.c_void_p,
                                   C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "sdf_render_multi_release": (C.c_int, []),
    "sdf_render_frames": (C.c_int, [_P(sdf_scene), _P(sdf_camera), C.c_int32, _P(sdf_light),
                                    _P(sdf_material), _P(sdf_params), C.c_void_p, C.c_void_p,
                                    C.c_void_p]),
    "sdf_comm_unique_id": (C.c_int, [C.c_char_p, C.c_void_p]),
    "sdf_comm_create": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                  _P(C.c_void_p)]),
    "sdf_comm_destroy": (C.c_int, [C.c_void_p]),
    "sdf_driver_create": (C.c_int, [_P(sdf_scene), _P(sdf_camera), _P(sdf_light),
                                    _P(sdf_material), _P(sdf_params), _P(sdf_driver_config),
                                    C.c_void_p, C.c_void_p, _P(C.c_void_p)]),
    "sdf_driver_set_camera": (C.c_int, [C.c_void_p, _P(sdf_camera)]),
    "sdf_driver_step": (C.c_int, [C.c_void_p, _P(C.c_int64)]),
    "sdf_driver_drain": (C.c_int, [C.c_void_p]),
    "sdf_driver_frame": (C.c_int, [C.c_void_p, C.c_int64, _P(C.c_void_p)]),
    "sdf_driver_read_frame": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                        C.c_void_p]),
    "sdf_driver_stats": (C.c_int, [C.c_void_p, _P(C.c_double), C.c_int32]),
    "sdf_driver_destroy": (C.c_int, [C.c_void_p]),
    "sdf_strerror": (C.c_char_p, [C.c_int]),
}

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libsdf3d.so"
_lib = None


class SdfError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _strerror(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


def _strerror(code: int) -> str:
    try:
        return load_library().sdf_strerror(code).decode()
    except Exception:  # pragma: no cover - library missing
        return f"error {code}"


def load_library(path: Path | str | None = None, any_version: bool = False) -> C.CDLL:
    """Load the in-tree HIP library; raise if it has not been built.
    any_version: accept another ABI version (measurement tools timing an
    older build of the same entry points side by side)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(
            f"{p} is missing: build the HIP library first (python -m sdf3d_amd.build). "
            "There is no CPU fallback on the product path.")
    lib = C.CDLL(str(p))
    # the version first: a stale library lacks later entry points, and the
    # mismatch is the message to give, not a missing symbol
    lib.sdf_abi_version.restype = C.c_int
    lib.sdf_abi_version.argtypes = []
    v = lib.sdf_abi_version()
    if v != SDF_ABI_VERSION and not any_version:
        raise RuntimeError(f"libsdf3d ABI version {v} != {SDF_ABI_VERSION}: rebuild it "
                           "(python -m sdf3d_amd.build)")
    for name, (res, args) in SIGNATURES.items():
        if any_version and not hasattr(lib, name):
            continue   # an older build without a later entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(code: int, what: str = "") -> None:
    if code != SDF_OK:
        raise SdfError(code, what)
