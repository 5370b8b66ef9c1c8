"""C-ABI boundary tests that need no GPU: the library loads, exports every
entry point include/sdf_abi.h declares, agrees on struct layouts, restates the
reference defaults, and rejects bad requests with the documented codes."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import oracle
from sdf3d_amd import abi, renderer, scenes

ROOT = Path(__file__).resolve().parent.parent


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(sdf_\w+)\s*\(", text, flags=re.M))
    return names


def test_library_exports_every_declared_symbol():
    lib = abi.load_library()
    names = declared_functions()
    assert names == set(abi.SIGNATURES), names ^ set(abi.SIGNATURES)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.sdf_abi_version() == abi.SDF_ABI_VERSION


def test_struct_sizes_match_header():
    for name, size in abi.STRUCT_SIZES.items():
        assert C.sizeof(getattr(abi, name)) == size, name


def _as_bytes(s):
    return bytes(C.string_at(C.addressof(s), C.sizeof(s)))


@pytest.mark.parametrize("wh", [(0, 0), (1920, 1080), (37, 23)])
def test_defaults_match_oracle_statement(wh):
    """sdf_defaults restates voxel_fragment.frag:15-23,54-81,178-189,205 and
    main.cpp:4-11; the oracle restates them independently."""
    f = scenes.reference(*wh)
    s, c, l, m, p = oracle.defaults(*wh)
    for a, b in [(f.scene, s), (f.camera, c), (f.light, l), (f.material, m), (f.params, p)]:
        assert _as_bytes(a) == _as_bytes(b), type(a).__name__


def test_reference_constants():
    f = scenes.reference()
    assert np.float32(f.camera.pi) == np.float32(3.1415925359)   # :15 (the typo'd PI)
    assert np.float32(f.camera.pi) != np.float32(np.pi)
    assert f.params.max_steps == 100 and f.params.max_dist == 100.0      # :17-18
    assert np.float32(f.params.eps) == np.float32(0.01)                  # :19
    assert (f.params.width, f.params.height) == (800, 600)               # main.cpp:4-5
    assert f.scene.count == 2 and f.scene.prims[0].kind == abi.PRIM_PLANE
    assert list(f.scene.prims[1].p[:4]) == pytest.approx([0.0, 0.4, 0.0, 0.2])
    assert list(f.light.pos) == [5.0, 5.0, 0.0] and f.material.shininess == 12.0


def _validate(f, t=None):
    lib = abi.load_library()
    return lib.sdf_validate(C.byref(f.scene), C.byref(f.camera), C.byref(f.light),
                            C.byref(f.material), C.byref(f.params),
                            C.byref(t) if t is not None else None)


def test_validate_accepts_all_configs():
    for name in scenes.CONFIGS:
        assert _validate(scenes.config(name)) == abi.SDF_OK, name


@pytest.mark.parametrize("mutate", [
    lambda f: setattr(f.params, "width", 0),
    lambda f: setattr(f.params, "height", -5),
    lambda f: setattr(f.params, "max_steps", -1),
    lambda f: setattr(f.params, "flags", 0x80),
    lambda f: setattr(f.params, "normal_mode", 7),
    lambda f: setattr(f.params, "precision", 9),
    lambda f: setattr(f.params, "output_format", 7),
    lambda f: setattr(f.params, "dispatch", 3),
    lambda f: setattr(f.params, "dispatch", -1),
    lambda f: setattr(f.params, "eps", float("nan")),
    lambda f: setattr(f.scene, "count", abi.SDF_MAX_PRIMS + 1),
    lambda f: setattr(f.scene.prims[0], "kind", 99),
    lambda f: setattr(f.scene.prims[0], "op", 99),
    lambda f: (setattr(f.scene.prims[1], "op", abi.OP_SMOOTH_UNION),
               setattr(f.scene.prims[1], "k", 0.0)),
    lambda f: setattr(f.scene, "kind", 5),
    lambda f: [f.camera.view.__setitem__(i, 0.0) for i in range(16)],  # singular V_mat
    lambda f: f.camera.eye.__setitem__(0, float("inf")),
    # working range (no overflow, so the scene distance is never NaN)
    lambda f: f.scene.prims[1].p.__setitem__(3, 2e15),
    lambda f: f.camera.eye.__setitem__(1, -3e15),
    lambda f: f.light.pos.__setitem__(2, 1e16),
    lambda f: setattr(f.params, "max_dist", 1e16),
    lambda f: [f.camera.view.__setitem__(i, 1e-16 if i % 5 == 0 else 0.0) for i in range(15)],
    # every length the marches add stays in the working range
    lambda f: setattr(f.params, "normal_eps", 1e20),
    lambda f: setattr(f.params, "shadow_offset", -2e15),
    lambda f: setattr(f.params, "eps", 1e16),
    lambda f: setattr(f.params, "shadow_k", float("inf")),
    # a smooth blend radius below 2^-64 (the exact smooth-min's h h (k/4))
    lambda f: (setattr(f.scene.prims[1], "op", abi.OP_SMOOTH_UNION),
               setattr(f.scene.prims[1], "k", 1e-20)),
])
def test_validate_rejects(mutate):
    f = scenes.reference()
    mutate(f)
    assert _validate(f) == abi.SDF_E_INVALID_ARG


@pytest.mark.parametrize("field,value", [
    ("ao_base", float("nan")), ("ao_step", 1e16), ("ao_falloff", float("inf")),
    ("ao_strength", -1e20)])
def test_validate_rejects_ao_outside_range(field, value):
    f = scenes.config("C3")
    assert _validate(f) == abi.SDF_OK
    setattr(f.params, field, value)
    assert _validate(f) == abi.SDF_E_INVALID_ARG
    f.params.flags &= ~abi.FLAG_AO          # unused without AO
    assert _validate(f) == abi.SDF_OK


@pytest.mark.parametrize("center,scale", [
    ((2e38, 0.0, 0.0), 0.5), ((0.0, -2e15, 0.0), 1.0), ((0.0, 0.0, 0.0), 1e-20),
    ((0.0, 0.0, 0.0), 1e16), ((0.0, float("nan"), 0.0), 1.0)])
def test_validate_rejects_bulb_outside_range(center, scale):
    """The exact Mandelbulb's (p - c) * RN(1/scale) must stay finite (ADVICE
    r05: its Markstein steps give NaN where IEEE division gives INF)."""
    f = scenes.config("C5")
    assert _validate(f) == abi.SDF_OK
    for i, v in enumerate(center):
        f.scene.bulb_center[i] = v
    f.scene.bulb_scale = scale
    assert _validate(f) == abi.SDF_E_INVALID_ARG


def test_validate_rejects_bad_tiling():
    f = scenes.reference()
    for br, fb, bs in [(0, 0, 1), (8, -1, 1), (8, 0, 0)]:
        t = renderer.tiling(fb, bs, br) if bs else abi.sdf_tiling(br, fb, bs, 0)
        assert _validate(f, t) == abi.SDF_E_INVALID_ARG
    assert _validate(f, abi.sdf_tiling(8, 0, 1, 2)) == abi.SDF_E_INVALID_ARG    # unknown flag
    assert _validate(f, renderer.tiling(0, 2, 8, frame_rows=True)) == abi.SDF_OK
    f.params.output_format = abi.FORMAT_TILES        # a stream is packed tiles
    assert _validate(f, renderer.tiling(0, 2, 8, frame_rows=True)) == abi.SDF_E_INVALID_ARG


def test_render_rejects_null_output():
    f = scenes.reference()
    lib = abi.load_library()
    rc = lib.sdf_render(C.byref(f.scene), C.byref(f.camera), C.byref(f.light),
                        C.byref(f.material), C.byref(f.params), None, None, None, None)
    assert rc == abi.SDF_E_INVALID_ARG
    assert lib.sdf_deinterleave(None, 1, 1, 1, 1, 8, 0, None, None) == abi.SDF_E_INVALID_ARG
    assert [lib.sdf_format_bytes(f) for f in (0, 1, 2, 3, 4, 5, 6)] == \
        [16, 8, 4, 12, abi.SDF_E_UNSUPPORTED, 16, abi.SDF_E_INVALID_ARG]
    # the step heat map writes colours: not the shading-term format
    assert lib.sdf_heatmap(None, 0, 0, 128, abi.FORMAT_SHADE32F, None, None) == \
        abi.SDF_E_INVALID_ARG
    assert lib.sdf_tiles_decode(None, 1, 0, 8, 8, 8, None, None) == abi.SDF_E_INVALID_ARG


@pytest.mark.parametrize("wh", [(1, 1), (8, 8), (37, 23), (3840, 270)])
def test_tiles_capacity_matches_reference(wh):
    """sdf_tiles_bytes = the worst-case TILES stream restated in
    tests/tiles_ref.py (header, offset table, 16-B heads, 8 * 96 plane bytes
    per tile) plus the encoder's scratch: per-2048-tile scan totals and
    16-B aligned plane slots."""
    import tiles_ref
    lib = abi.load_library()
    n = ((wh[0] + 7) // 8) * ((wh[1] + 7) // 8)
    nb = (n + 2047) // 2048
    bsums = (tiles_ref.capacity(*wh) + 15) // 16 * 16
    slots = (bsums + 4 * nb + 15) // 16 * 16
    assert lib.sdf_tiles_bytes(*wh) == slots + n * 8 * 96
    assert lib.sdf_tiles_bytes(0, 8) == abi.SDF_E_INVALID_ARG


def test_tiles_offsets_fit_uint32():
    """TILES offsets and the `used` word are uint32, so a stream
    whose worst case exceeds 4 GiB is refused (SDF_E_UNSUPPORTED) by
    sdf_tiles_bytes and by the render plan, instead of wrapping."""
    lib = abi.load_library()
    assert lib.sdf_tiles_bytes(16384, 16384) > 0              # 4.2M tiles: 3.3 GB, fits
    assert lib.sdf_tiles_bytes(65536, 8192) == abi.SDF_E_UNSUPPORTED   # 8.4M tiles: 6.6 GB
    # (the render plan's refusal needs a device: test_gpu_parity.py)


def test_validate_accepts_tiles_format():
    f = scenes.reference()
    f.params.output_format = abi.FORMAT_TILES
    assert _validate(f) == abi.SDF_OK


@pytest.mark.parametrize("height", [1, 7, 8, 9, 23, 600, 1080, 2160])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_owned_rows_matches_oracle_and_partitions(height, world):
    total = 0
    for r in range(world):
        t = renderer.tiling(r, world, 8)
        n = renderer.owned_rows(height, t)
        assert n == oracle.owned_rows(height, t)
        total += n
    assert total == height
    # ranks owning no block at all (first_block beyond the last block)
    assert renderer.owned_rows(height, renderer.tiling((height + 7) // 8, 1, 8)) == 0


def tiling_rows(height, t):
    """Frame rows a tiling owns, in packed order, straight from the
    definition in include/sdf_abi.h (sdf_tiling)."""
    run, step = max(t.block_run, 1), max(t.run_step, 1)
    return [y for y in range(height)
            if y // t.block_rows >= t.first_block
            and (y // t.block_rows - t.first_block) % t.block_stride % step == 0
            and (y // t.block_rows - t.first_block) % t.block_stride // step < run]


@pytest.mark.parametrize("height", [1, 9, 71, 270, 1080, 2160])
@pytest.mark.parametrize("world,shares", [(2, (1, 2)), (3, (2, 3)), (4, (3, 1)), (8, (1, 2)),
                                          (8, (1, 3)), (8, (2, 5))])
def test_weighted_tiling_partitions_frame(height, world, shares):
    """Unequal shares (sdf_tiling.block_run, peers' runs spaced by
    run_step): every rank's rows as the library and the oracle count them,
    and together exactly the frame."""
    rows = []
    for r in range(world):
        t = renderer.tiling(r, world, 8, shares=shares)
        ys = tiling_rows(height, t)
        n = renderer.owned_rows(height, t)
        assert n == len(ys) == oracle.owned_rows(height, t)
        rows += ys
    assert sorted(rows) == list(range(height))
    # rank 0's share is a / (a + b (world - 1)) of whole periods
    a, b = shares
    period = 8 * (a + b * (world - 1))
    if height % period == 0:
        assert renderer.owned_rows(height, renderer.tiling(0, world, 8, shares=shares)) == \
            height // period * 8 * a


def test_tiling_run_validation():
    lib = abi.load_library()
    t = renderer.tiling(1, 4, 8)
    t.block_run = t.block_stride + 1          # a run longer than its period
    assert lib.sdf_owned_rows(100, C.byref(t)) == abi.SDF_E_INVALID_ARG
    t.block_run = -1
    assert lib.sdf_owned_rows(100, C.byref(t)) == abi.SDF_E_INVALID_ARG
    t.block_run = 0                           # 0 and 1 both mean one block
    n0 = lib.sdf_owned_rows(100, C.byref(t))
    t.block_run = 1
    assert lib.sdf_owned_rows(100, C.byref(t)) == n0 == len(tiling_rows(100, t))
    with pytest.raises(ValueError):
        renderer.tiling(0, 2, 8, shares=(0, 1))
    # spaced runs: the run must fit its period, and blocks hold whole 8-row tiles
    t = renderer.tiling(1, 8, 8, shares=(1, 3))
    assert (t.block_run, t.run_step, t.block_stride) == (3, 7, 22)
    t.run_step = 11                           # (3 - 1) * 11 = 22: past the period
    assert lib.sdf_owned_rows(100, C.byref(t)) == abi.SDF_E_INVALID_ARG
    t.run_step = -1
    assert lib.sdf_owned_rows(100, C.byref(t)) == abi.SDF_E_INVALID_ARG
    t.run_step, t.block_rows = 7, 4
    assert lib.sdf_owned_rows(100, C.byref(t)) == abi.SDF_E_INVALID_ARG
    t.run_step = 1                            # consecutive runs take any block size
    assert lib.sdf_owned_rows(100, C.byref(t)) == len(tiling_rows(100, t))


def test_strerror():
    lib = abi.load_library()
    for code in (abi.SDF_OK, abi.SDF_E_INVALID_ARG, abi.SDF_E_UNSUPPORTED, abi.SDF_E_HIP,
                 abi.SDF_E_NO_DEVICE, -1234):
        assert isinstance(lib.sdf_strerror(code), bytes)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        abi.load_library(tmp_path / "nope.so")


@pytest.mark.parametrize("bailout,ok", [(2.0, True), (2.0**32, True), (0.0, False), (-1.0, False),
                                        (2.0**33, False), (float("inf"), False),
                                        (float("nan"), False)])
def test_validate_mandelbulb_bailout(bailout, ok):
    """bailout in (0, 2^32]: its square stays finite (sdf_abi.h sdf_scene)."""
    f = scenes.config("C5", 64, 36)
    f.scene.bulb_bailout = bailout
    assert _validate(f) == (abi.SDF_OK if ok else abi.SDF_E_INVALID_ARG)


def test_validate_rejects_degenerate_capsule():
    """A capsule whose end points coincide has h = dot(pa, ba) / dot(ba, ba)
    = 0 / 0: refused (every primitive value must be a number)."""
    f = scenes.config("C3", 64, 64)
    cap = [i for i in range(f.scene.count) if f.scene.prims[i].kind == abi.PRIM_CAPSULE]
    assert cap
    pr = f.scene.prims[cap[0]]
    assert _validate(f) == abi.SDF_OK
    for j in range(3):
        pr.p[3 + j] = pr.p[j]
    assert _validate(f) == abi.SDF_E_INVALID_ARG


@pytest.mark.parametrize("length,ok", [(2.0**-15 * 1.01, True), (2.0**-15 * 0.99, False),
                                       (2.0**15 * 0.99, True), (2.0**15 * 1.01, False)])
def test_validate_capsule_length_range(length, ok):
    """Round 6: capsule lengths in [2^-15, 2^15) -- dot(ba, ba) in [2^-30,
    2^30), the exact kernel's Markstein division of h (render_kernel.inc
    sd_capsule)."""
    f = scenes.config("C3", 64, 64)
    cap = [i for i in range(f.scene.count) if f.scene.prims[i].kind == abi.PRIM_CAPSULE][0]
    pr = f.scene.prims[cap]
    pr.p[3], pr.p[4], pr.p[5] = pr.p[0] + length, pr.p[1], pr.p[2]
    assert _validate(f) == (abi.SDF_OK if ok else abi.SDF_E_INVALID_ARG)


def test_schedule_and_checked_decode_refuse_bad_arguments():
    """Host-side argument checks of the round-5 entry points (no device)."""
    lib = abi.load_library()
    h = C.c_void_p()
    for rows, period in [(0, 1), (-8, 1), (4097, 1), (64, 0)]:
        assert lib.sdf_schedule_create(rows, period, C.byref(h)) == abi.SDF_E_INVALID_ARG
        assert not h.value
    assert lib.sdf_schedule_create(64, 1, None) == abi.SDF_E_INVALID_ARG
    assert lib.sdf_schedule_destroy(None) == abi.SDF_OK
    assert lib.sdf_schedule_order(None, None, 0) == abi.SDF_E_INVALID_ARG
    t = (abi.sdf_tiling * 1)()
    for nparts in (0, abi.MAX_DECODE_PARTS + 1):
        assert lib.sdf_tiles_decode_checked(None, nparts, 0, t, None, 8, 8, None, None,
                                            None) == abi.SDF_E_INVALID_ARG
