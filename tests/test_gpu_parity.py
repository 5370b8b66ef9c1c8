"""GPU parity tests: the HIP kernels (through the C-ABI) against the CPU oracle.

Exact precision (IEEE div/sqrt, no contraction) must satisfy the parity policy
of tests/parity.py against the golden fixtures and fresh oracle renders; fast
precision (hardware sqrt/rcp, FMA) is held to the same policy, or, on
fp32-ill-conditioned frames, to the spread of the oracle's own alternative
readings (check_frame).  Full-size (BASELINE) frames are compared per pixel
with a live oracle render on the bench's own code path
(test_full_size_pixel_parity), and through size-independent properties:
step-count sums against the oracle's full-frame statistics, determinism,
tiling invariance, finiteness.
"""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
from golden.make_golden import FIXTURES, frame_for
from parity import (assert_parity, assert_parity_frame, assert_regression, compare,
                    full_size_conditioning, quantize, reading_spread, report)
from sdf3d_amd import abi, renderer as R, scenes

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"
RESULTS = {}


def gpu(rd, frame, t=None, steps=True):
    """Render `frame` both ways: without a steps buffer -- the code path the
    bench times, where the exact shadow skip (render_kernel.inc, shadow march
    skipped where clamp(N.L, 0, 1) = 0) is active -- and with one.  The two
    must agree bit for bit (the skip is result-neutral); returns the
    no-steps frame and, if `steps`, the per-pixel step counts."""
    import torch
    rgba, _ = rd.render(frame, t, steps=False)
    rgba_s, st = rd.render(frame, t, steps=True)
    torch.cuda.synchronize()
    rgba = rgba.cpu().numpy()
    assert np.array_equal(rgba.view(np.uint8), rgba_s.cpu().numpy().view(np.uint8)), \
        "steps=None (shadow skip) and steps=True renders differ"
    return rgba, (st.cpu().numpy() if steps else None)


def with_precision(frame, prec):
    f = frame.copy()
    f.params.precision = prec
    return f


def log(key, rep):
    RESULTS[key] = rep
    print(key, json.dumps(rep))


def check_frame(key, frame, rgba, steps, ref, ref_steps, t=None):
    """Parity of one GPU frame against the oracle, outliers diagnosed by the
    forced-step replay at the kernel's recorded step counts (parity.py).
    Exact precision: the strict policy.  Fast precision: the strict policy
    unless this frame is measured fp32-ill-conditioned (the fp64 twin or the
    contracted fp32 reading fails it against the oracle under the same
    replay diagnosis) or at the BASELINE size of its scene and pose
    (tests/golden/conditioning.json), then the readings' spread with its
    magnitude bound."""
    if frame.params.precision == abi.PRECISION_EXACT:
        rep = compare(frame, rgba, steps, ref, ref_steps, t)
        rep["policy"] = "strict"
        log(key, rep)
        assert_parity(rep, what=key)
        return rep
    readings = {"twin": oracle.render(frame, t, twin=True),
                "fma": oracle.render(frame, t, variant="fma")}
    rep = compare(frame, rgba, steps, ref, ref_steps, t, twin_rgba=readings["twin"][0],
                  alt_rgba=[readings["fma"][0]])
    spread = reading_spread(frame, ref, ref_steps, readings, t)
    rep["readings"] = {n: {k: r[k] for k in ("outliers", "replay_diagnosed", "undiagnosed",
                                             "undiagnosed_max_err", "over_max_err", "max_err")}
                       for n, r in spread.items()}
    full = full_size_conditioning(frame)
    rep["full_size_conditioning"] = None if full is None else {
        n: {k: full[n][k] for k in ("outlier_rate", "undiagnosed_rate", "undiagnosed_max_err")}
        for n in ("twin", "fma")}
    try:
        rep["policy"] = assert_parity_frame(rep, spread, what=key, full_size=full)
    finally:
        log(key, rep)
    return rep


@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_fixture_parity(renderer, name, prec):
    z = np.load(GOLD / f"{name}.npz")
    f = with_precision(frame_for(name), prec)
    rgba, steps = gpu(renderer, f)
    check_frame(f"fixture/{name}/{'exact' if prec == 0 else 'fast'}", f, rgba, steps,
                z["rgba"], z["steps"])


@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
@pytest.mark.parametrize("cfg,w,h,pose", [
    ("REF", 800, 600, 0), ("REF", 640, 360, 2), ("C1", 512, 512, 0), ("C2", 640, 360, 3),
    ("C3", 480, 270, 2), ("C5", 320, 180, 0)])
def test_fresh_oracle_parity(renderer, cfg, w, h, pose, prec):
    f = scenes.config(cfg, w, h, precision=prec, pose=pose)
    rgba, steps = gpu(renderer, f)
    ref_rgba, ref_steps = oracle.render(f)
    check_frame(f"fresh/{cfg}_{w}x{h}_p{pose}/{'exact' if prec == 0 else 'fast'}", f, rgba,
                steps, ref_rgba, ref_steps)


@pytest.mark.parametrize("cfg,pose", [("REF", 0), ("C1", 0), ("C3", 1), ("C5", 0)])
def test_specialised_matches_generic(renderer, cfg, pose):
    """The compile-time scene variants compute the generic kernel's result:
    bit-identical in exact precision, within the policy in fast precision."""
    for prec in (abi.PRECISION_EXACT, abi.PRECISION_FAST):
        f = scenes.config(cfg, 192, 108, precision=prec, pose=pose)
        a, sa = gpu(renderer, f)
        g = f.copy()
        g.params.dispatch = abi.DISPATCH_UNCULLED
        b, sb = gpu(renderer, g)
        if prec == abi.PRECISION_EXACT or cfg == "C5":
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(sa, sb)
        else:
            assert_parity(compare(f, a, sa, b, sb, ref_is_oracle=False), what=cfg)


def test_exact_mode_is_mostly_bit_exact(renderer):
    """Exact precision executes the oracle's fp32 operation sequence; only the
    transcendental pow (specular) may differ by an ulp."""
    f = scenes.config("REF", 320, 180)
    rgba, steps = gpu(renderer, f)
    ref, ref_steps = oracle.render(f)
    assert np.array_equal(steps, ref_steps)
    rep = report(rgba, steps, ref, ref_steps)
    log("bitexact/REF_320x180", rep)
    assert rep["max_err"] < 1e-6


@pytest.mark.parametrize("op", range(abi.OP_COUNT))
def test_every_csg_op(renderer, op):
    f = scenes.config("C3", 160, 90)
    for i in range(2, f.scene.count):
        f.scene.prims[i].op = op
        f.scene.prims[i].k = 0.1
    rgba, steps = gpu(renderer, f)
    ref, ref_steps = oracle.render(f)
    rep = compare(f, rgba, steps, ref, ref_steps)
    log(f"csg_op/{abi.OP_NAMES[op]}", rep)
    assert_parity(rep, what=abi.OP_NAMES[op])


@pytest.mark.parametrize("mutate,name", [
    (lambda f: setattr(f.params, "normal_mode", abi.NORMAL_TETRA), "ref_tetra"),
    (lambda f: setattr(f.params, "flags", abi.FLAG_SHADOW | abi.FLAG_AO), "ref_ao"),
    (lambda f: setattr(f.params, "flags", 0), "ref_noshadow"),
    (lambda f: setattr(f.params, "max_steps", 0), "max_steps_0"),
    (lambda f: setattr(f.params, "max_steps", 1), "max_steps_1"),
    (lambda f: setattr(f.params, "ao_taps", 1) or setattr(f.params, "flags", 3), "ao_1tap"),
    (lambda f: setattr(f.camera, "aspect", 2.5), "explicit_AR"),
])
def test_feature_variants(renderer, mutate, name):
    f = scenes.config("REF", 96, 64)
    mutate(f)
    rgba, steps = gpu(renderer, f)
    ref, ref_steps = oracle.render(f)
    rep = compare(f, rgba, steps, ref, ref_steps)
    log(f"variant/{name}", rep)
    assert_parity(rep, what=name)


@pytest.mark.parametrize("w,h", [(1, 1), (1, 9), (33, 1), (37, 23), (63, 65), (257, 9)])
def test_ragged_sizes(renderer, w, h):
    for prec in (abi.PRECISION_EXACT, abi.PRECISION_FAST):
        f = scenes.config("C3", w, h, precision=prec, pose=1)
        rgba, steps = gpu(renderer, f)
        ref, ref_steps = oracle.render(f)
        rep = compare(f, rgba, steps, ref, ref_steps)
        assert_parity(rep, what=f"{w}x{h}/{prec}")


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_tiling_and_deinterleave_reassemble_frame(renderer, world):
    """Pixels are independent: rendering interleaved row blocks per rank and
    scattering them back must reproduce the whole frame bit for bit."""
    import torch
    f = scenes.config("C3", 480, 270, precision=abi.PRECISION_FAST, pose=1)
    whole, _ = renderer.render(f)
    stride = R.owned_rows(f.params.height, R.tiling(0, world))
    parts = torch.zeros((world * stride, f.params.width, 4), dtype=torch.float32,
                        device=renderer.device)
    for r in range(world):
        t = R.tiling(r, world)
        n = R.owned_rows(f.params.height, t)
        renderer.render(f, t, out=parts[r * stride:r * stride + n])
    frame = renderer.deinterleave(parts, world, stride, f.params.width, f.params.height)
    torch.cuda.synchronize()
    assert torch.equal(frame.view(torch.int32), whole.view(torch.int32))
    # oracle agrees on one rank's packed part
    t = R.tiling(world - 1, world)
    part, pst = gpu(renderer, f, t)
    ref, ref_st = oracle.render(f, t)
    n = R.owned_rows(f.params.height, t)
    assert np.array_equal(part, parts[(world - 1) * stride:(world - 1) * stride + n].cpu().numpy())
    assert_parity(compare(f, part, pst, ref, ref_st, t), what="part")


@pytest.mark.parametrize("world,shares", [(3, (1, 2)), (8, (1, 3))])
def test_weighted_tiling_renders_its_rows(renderer, world, shares):
    """Runs of blocks (sdf_tiling.block_run, spaced by run_step): each
    rank's packed rows are the whole frame's rows it owns, bit for bit, and
    the oracle agrees on one."""
    import torch
    f = scenes.config("C3", 320, 183, precision=abi.PRECISION_FAST, pose=2)
    whole, _ = renderer.render(f)
    whole = whole.cpu().numpy()
    H = f.params.height
    for r in range(world):
        t = R.tiling(r, world, 8, shares=shares)
        run, step = max(t.block_run, 1), max(t.run_step, 1)
        ys = [y for y in range(H) if y // 8 >= t.first_block
              and (y // 8 - t.first_block) % t.block_stride % step == 0
              and (y // 8 - t.first_block) % t.block_stride // step < run]
        part, _ = renderer.render(f, t)
        torch.cuda.synchronize()
        assert part.shape[0] == len(ys)
        assert np.array_equal(part.cpu().numpy().view(np.uint32), whole[ys].view(np.uint32))
    t = R.tiling(1, world, 8, shares=shares)
    part, pst = gpu(renderer, f, t)
    ref, ref_st = oracle.render(f, t)
    assert_parity(compare(f, part, pst, ref, ref_st, t), what="weighted part")


def test_empty_tiling_is_noop(renderer):
    import torch
    f = scenes.config("REF", 64, 16)
    t = R.tiling(5, 8)          # owns no block of a 16-row frame
    assert R.owned_rows(16, t) == 0
    out = torch.empty((0, 64, 4), dtype=torch.float32, device=renderer.device)
    renderer.render(f, t, out=out)
    torch.cuda.synchronize()


def test_nondefault_stream_and_determinism(renderer):
    import torch
    f = scenes.config("C3", 640, 360, precision=abi.PRECISION_FAST, pose=3)
    s = torch.cuda.Stream(device=renderer.device)
    a, _ = renderer.render(f, stream=s)
    b, _ = renderer.render(f, stream=s)
    s.synchronize()
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))


@pytest.mark.parametrize("cfg", ["C4", "C2", "C5"])
@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
def test_full_size_properties(renderer, cfg, prec):
    """BASELINE-size frames: step sums match the oracle's full-frame statistics
    (tests/golden/stats_*.npz) row by row up to branch flips; output finite,
    alpha 1; two launches bit-identical."""
    import torch
    f = scenes.config(cfg, precision=prec)
    rgba, st = renderer.render(f, steps=True)
    rgba2, _ = renderer.render(f)
    torch.cuda.synchronize()
    assert torch.equal(rgba.view(torch.int32), rgba2.view(torch.int32))
    assert bool(torch.isfinite(rgba).all()) and bool((rgba[..., 3] == 1).all())
    z = np.load(GOLD / f"stats_{cfg}_p0.npz")
    sp = st[..., 0].sum(dim=1, dtype=torch.int64).cpu().numpy()
    ss = st[..., 1].sum(dim=1, dtype=torch.int64).cpu().numpy()
    tot_sp, tot_ss = z["row_sp"].sum(), z["row_ss"].sum()
    rel_sp = abs(sp.sum() - tot_sp) / max(tot_sp, 1)
    rel_ss = abs(ss.sum() - tot_ss) / max(tot_ss, 1)
    rows_equal = float(np.mean((sp == z["row_sp"]) & (ss == z["row_ss"])))
    log(f"fullsize/{cfg}/{'exact' if prec == 0 else 'fast'}",
        {"rel_sp": rel_sp, "rel_ss": rel_ss, "rows_equal": rows_equal})
    assert rel_sp < 1e-3 and rel_ss < 1e-3
    if prec == abi.PRECISION_EXACT:
        # the oracle's fp32 operation sequence (log/pow correctly rounded on
        # both sides): every row's step counts at the full BASELINE size equal
        # the oracle's exactly
        assert rows_equal == 1.0


FULL_CASES = [("C4", abi.PRECISION_FAST), ("C4", abi.PRECISION_EXACT),
              ("C3", abi.PRECISION_FAST), ("C3", abi.PRECISION_EXACT),
              ("C2", abi.PRECISION_FAST), ("C2", abi.PRECISION_EXACT),
              ("C5", abi.PRECISION_FAST), ("C5", abi.PRECISION_EXACT)]


@pytest.mark.parametrize("cfg,prec", FULL_CASES)
def test_full_size_pixel_parity(renderer, cfg, prec):
    """Per-pixel parity at the BASELINE size (C4/C5 3840x2160, C3/C2 1920x1080)
    on the bench's own code path: the frame rendered WITHOUT a steps buffer
    (exact shadow skip active), against a live oracle render of the same
    frame on all host threads (voxel_fragment.frag:160-211), under
    check_frame's policy: strict for exact precision; for fast precision
    strict unless the oracle's own alternative readings fail it at this size
    (then their spread).  The per-pixel step counts of the steps=True render
    (bit-identical colours) and the alternative readings diagnose outliers.
    Exact precision runs the oracle's fp32 operation sequence: its per-pixel
    step counts equal the oracle's everywhere."""
    import time

    import torch
    f = scenes.config(cfg, precision=prec)
    W, H = f.params.width, f.params.height
    rgba, _ = renderer.render(f, steps=False)
    rgba_s, st = renderer.render(f, steps=True)
    torch.cuda.synchronize()
    assert torch.equal(rgba.view(torch.int32), rgba_s.view(torch.int32))
    del rgba_s
    rgba, st = rgba.cpu().numpy(), st.cpu().numpy()
    t0 = time.perf_counter()
    ref, ref_st = oracle.render(f)
    t_oracle = time.perf_counter() - t0
    px_equal = float(np.mean(np.all(st == ref_st, axis=-1)))
    rep = check_frame(f"fullsize_pixels/{cfg}/{'exact' if prec == 0 else 'fast'}", f, rgba, st,
                      ref, ref_st)
    kid = abi.load_library().sdf_kernel_id(prec)
    rep.update(width=W, height=H, steps_equal_frac=px_equal, oracle_s=round(t_oracle, 2),
               path="steps=None (bench path, shadow skip active)", config=cfg,
               precision="exact" if prec == 0 else "fast",
               kernel_id=kid.decode() if kid else None)
    if prec == abi.PRECISION_EXACT:
        assert px_equal == 1.0
    else:
        # the kernel's own last full-size measurement (tests/golden/fast_regression.json)
        assert_regression(rep, f"{cfg}_p0", what=f"fullsize_pixels/{cfg}/fast")


def test_invalid_arguments_are_rejected_on_device(renderer):
    import torch
    lib = abi.load_library()
    f = scenes.reference(64, 64)
    f.params.max_steps = -3
    out = torch.empty((64, 64, 4), dtype=torch.float32, device=renderer.device)
    rc = lib.sdf_render(C.byref(f.scene), C.byref(f.camera), C.byref(f.light),
                        C.byref(f.material), C.byref(f.params), None,
                        C.c_void_p(out.data_ptr()), None, None)
    assert rc == abi.SDF_E_INVALID_ARG
    with pytest.raises(abi.SdfError):
        renderer.render(f, out=out)
    # a TILES render whose worst-case stream overflows its 32-bit offsets is
    # refused before any launch
    g = scenes.reference(65536, 8192)
    g.params.output_format = abi.FORMAT_TILES
    rc = lib.sdf_render(C.byref(g.scene), C.byref(g.camera), C.byref(g.light),
                        C.byref(g.material), C.byref(g.params), None,
                        C.c_void_p(out.data_ptr()), None, None)
    assert rc == abi.SDF_E_UNSUPPORTED


@pytest.mark.parametrize("fmt", [abi.FORMAT_RGBA16F, abi.FORMAT_RGBA8, abi.FORMAT_RGB32F])
@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
def test_output_formats(renderer, fmt, prec):
    """RGBA16F / RGBA8 framebuffers are the kernel's float colour converted
    exactly as the spec says (bit-exact against its own RGBA32F output), and
    agree with the quantised oracle except where a float sits within the
    kernel-vs-oracle difference of a rounding boundary."""
    import torch
    f = scenes.config("C3", 320, 180, precision=prec, pose=2)
    ref32, _ = gpu(renderer, f)
    g = f.copy()
    g.params.output_format = fmt
    out, _ = gpu(renderer, g)
    want = quantize(ref32, fmt)
    assert out.dtype == want.dtype
    assert np.array_equal(out.view(np.uint8), want.view(np.uint8))
    orc, ost = oracle.render(scenes.config("C3", 320, 180, pose=2))
    if fmt == abi.FORMAT_RGB32F:
        # a float format: the RGBA32F parity policy applies (alpha is 1)
        rgba = np.concatenate([out, np.ones_like(out[..., :1])], -1)
        _, gst = gpu(renderer, f)
        assert_parity(compare(f, rgba, gst, orc, ost), what="rgb32f")
    else:
        diff = np.abs(out.astype(np.float64) - quantize(orc, fmt).astype(np.float64))
        # one LSB at most; how often a boundary is crossed depends on the float
        # difference (exact: ~1e-7, fast: ~1e-5 against an fp16 step of ~5e-4)
        lsb = 1.0 if fmt == abi.FORMAT_RGBA8 else 1e-3
        frac = 1e-3 if prec == abi.PRECISION_EXACT else 2e-2
        assert (diff.max(axis=-1) > 0).mean() < frac and diff.max() <= max(lsb, 5e-3)
    # the multi-device scatter handles the narrow formats too
    world = 3
    stride = R.owned_rows(180, R.tiling(0, world))
    parts = torch.zeros((world * stride, 320, R.channels(fmt)), dtype=R.torch_dtype(fmt),
                        device=renderer.device)
    for r in range(world):
        t = R.tiling(r, world)
        n = R.owned_rows(180, t)
        renderer.render(g, t, out=parts[r * stride:r * stride + n])
    frame = renderer.deinterleave(parts, world, stride, 320, 180)
    torch.cuda.synchronize()
    # RGB32F wire parts come back as the RGBA32F frame (alpha restored = 1)
    full = ref32 if fmt == abi.FORMAT_RGB32F else out
    assert np.array_equal(frame.cpu().numpy().view(np.uint8), full.view(np.uint8))


def test_write_results():
    out = Path("gpurun_out")
    out.mkdir(exist_ok=True)
    (out / "parity_results.json").write_text(json.dumps(RESULTS, indent=1, sort_keys=True))
    # the full-size frames alone, keyed "<cfg>/<precision>" with the kernel_id
    # they were taken from: bench.py's `parity` object reads the committed
    # copy (profiles/parity_fullsize.json)
    full = {k.split("/", 1)[1]: v for k, v in RESULTS.items() if k.startswith("fullsize_pixels/")}
    if full:
        (out / "parity_fullsize.json").write_text(json.dumps(full, indent=1, sort_keys=True))


def read_ppm(path):
    data = Path(path).read_bytes()
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6"
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], dtype=np.uint8).reshape(h, w, 3)


@pytest.mark.parametrize("scene_name,cfg", [("ref", "REF"), ("csg8", "C3")])
def test_cpp_host_program(renderer, tmp_path, scene_name, cfg):
    """examples/sdf_main.cpp (C++ API in include/sdf3d.hpp) renders the same
    frame as the Python path; its PPM is the clamped 8-bit image."""
    import subprocess
    exe = Path(__file__).resolve().parent.parent / "sdf3d_amd" / "bin" / "sdf_main"
    assert exe.exists(), "build() must produce sdf3d_amd/bin/sdf_main"
    out = tmp_path / "f.ppm"
    r = subprocess.run([str(exe), "160", "90", "2", str(out), scene_name], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = read_ppm(out)
    f = scenes.config(cfg, 160, 90, precision=abi.PRECISION_EXACT)   # sdf_main's default
    scenes.set_view(f, scenes.orbit_view(180.0, 0.0))     # frame 1 of 2: yaw 180
    rgba, _ = gpu(renderer, f, steps=False)
    want = quantize(rgba, abi.FORMAT_RGBA8)[::-1, :, :3]
    assert np.abs(img.astype(int) - want.astype(int)).max() <= 1


@pytest.mark.parametrize("nproc,wire,shares", [(2, "auto", None), (3, "auto", None),
                                               (2, "rgb32f", None), (3, "tiles", "1:2"),
                                               (8, "auto", None)])
def test_multirank_bench_rehearsal(renderer, tmp_path, nproc, wire, shares):
    """bench.py with 2, 3 or 8 ranks sharing this GPU (gloo backend; RCCL needs one
    GPU per rank): the FrameDriver's GPU path -- alternating render streams,
    the TILES wire (auto: kernel-written compressed streams, per-frame size
    agreement, sdf_tiles_decode_tilings on the frame's render stream of rank
    0, unequal row shares) or the RGB32F wire (sdf_deinterleave) --
    assembles frames bit-identical to a single-device render."""
    import json
    import sys
    from netutil import run_launcher
    root = Path(__file__).resolve().parent.parent

    def cmd(port):
        c = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
             str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(port),
             str(root / "bench.py"), "--gpus", str(nproc), "--steps", "4", "--warmup", "2",
             "--backend", "gloo", "--config", "C3", "--wire", wire, "--no-display"]
        return c + (["--shares", shares] if shares else [])
    r = run_launcher(cmd, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == nproc and d["frame_verified"] is True
    assert d["config"]["wire"] == ("tiles" if wire == "auto" else wire)
    assert d["no_gather"]["value"] > 0
    if shares:
        assert d["config"]["tiling"].startswith("8-row blocks, rank 0 1 / others 2")
    if nproc == 8:  # the round-end N=8 run's default shares (multigpu.choose_shares)
        assert d["config"]["tiling"].startswith("8-row blocks, rank 0 1 / others 7")


def turbo_ref(steps, which, max_steps):
    """The reference's colormap (utilities.cl:7-284) applied to step counts:
    the fixture's fp32 table (tests/golden/turbo_lut.json, extracted from
    utilities.cl:12-267) at i = round(255 * intensity), half away from zero,
    clamped to [0, 255] (:269-281), intensity = count / max_steps in fp32."""
    lut = np.array(json.loads((GOLD / "turbo_lut.json").read_text())["fp32_bits"],
                   dtype=np.uint32).view(np.float32)
    s = steps.astype(np.int64)
    n = s[..., 0] if which == 0 else (s[..., 1] if which == 1 else s[..., 0] + s[..., 1])
    if max_steps > 0:
        t = n.astype(np.float32) / np.float32(max_steps)
    else:
        t = np.zeros(n.shape, np.float32)
    x = np.float32(255) * t                                    # fp32 product
    r = np.floor(np.abs(x) + np.float32(0.5)) * np.sign(x)     # half away from zero
    idx = np.clip(r, 0, 255).astype(np.int64)
    c = lut[idx]
    return np.concatenate([c, np.ones_like(c[..., :1])], -1), idx


@pytest.mark.parametrize("which", [0, 1, 2])
def test_heatmap(renderer, which):
    import torch
    f = scenes.config("C3", 256, 144, precision=abi.PRECISION_FAST, pose=1)
    _, st = renderer.render(f, steps=True)
    h32 = renderer.heatmap(st, which, f.params.max_steps, abi.FORMAT_RGBA32F)
    h8 = renderer.heatmap(st, which, f.params.max_steps, abi.FORMAT_RGBA8)
    torch.cuda.synchronize()
    want, _ = turbo_ref(st.cpu().numpy(), which, f.params.max_steps)
    assert np.array_equal(h32.cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert np.array_equal(h8.cpu().numpy(), quantize(h32.cpu().numpy(), abi.FORMAT_RGBA8))


@pytest.mark.parametrize("max_steps", [255, 100, 128, 64, 7, 0])
def test_heatmap_every_lut_entry(renderer, max_steps):
    """Every table entry, bit for bit, through crafted step counts: counts
    0..2*max_steps+3 hit each index the mapping can produce, the ties of
    max_steps = 100 (count 30 -> 76.5 -> 77, where rint would give 76) pin
    the half-away rounding, and counts past max_steps pin the clamp at 255."""
    import torch
    hi = 2 * max(max_steps, 1) + 4
    n = np.arange(hi, dtype=np.int32)
    st = np.stack([n, n[::-1]], -1).reshape(1, hi, 2)
    dev = torch.from_numpy(st).to(renderer.device)
    for which in (0, 1, 2):
        h = renderer.heatmap(dev, which, max_steps, abi.FORMAT_RGBA32F)
        torch.cuda.synchronize()
        want, idx = turbo_ref(st, which, max_steps)
        assert np.array_equal(h.cpu().numpy().view(np.uint32), want.view(np.uint32)), which
        if max_steps == 255 and which == 0:
            assert set(idx.ravel().tolist()) == set(range(256))
        if max_steps == 100 and which == 0:
            assert idx[0, 30] == 77 and idx[0, 10] == 26


def random_csg8(rng, spread, kmax):
    """A scene with the CSG8 signature (so the culled FixedScene variant runs)
    but random sizes, positions and blend radii."""
    f = scenes.config("C3", 160, 96)
    s = f.scene
    u = lambda a, b: float(rng.uniform(a, b))  # noqa: E731
    c = lambda: (u(-spread, spread), u(-0.2, spread), u(-spread, spread))  # noqa: E731
    s.prims[0].p[3] = u(-0.3, 0.3)                                  # plane offset
    for i in range(1, 8):
        pr = s.prims[i]
        pr.k = u(1e-3, kmax)
        x, y, z = c()
        pr.p[0], pr.p[1], pr.p[2] = x, y, z
        kind = pr.kind
        if kind == abi.PRIM_SPHERE:
            pr.p[3] = u(0.01, 0.6)
        elif kind in (abi.PRIM_BOX, abi.PRIM_ROUND_BOX):
            pr.p[3], pr.p[4], pr.p[5] = u(0.02, 0.5), u(0.02, 0.5), u(0.02, 0.5)
            if kind == abi.PRIM_ROUND_BOX:
                pr.p[6] = u(0.0, 0.5) * min(pr.p[3], pr.p[4], pr.p[5])
        elif kind == abi.PRIM_TORUS:
            pr.p[3], pr.p[4] = u(0.05, 0.5), u(0.01, 0.2)
        elif kind == abi.PRIM_CAPSULE:
            pr.p[3], pr.p[4], pr.p[5] = c()
            pr.p[6] = u(0.01, 0.3)
        elif kind == abi.PRIM_CYLINDER:
            pr.p[3], pr.p[4] = u(0.02, 0.4), u(0.02, 0.6)
    return f


@pytest.mark.parametrize("seed", range(12))
def test_culling_exact_on_random_scenes(renderer, seed):
    """The culled fixed-scene kernel equals the unculled generic kernel bit for
    bit (exact precision), step counts included, for random parameters of the
    CSG8 signature: overlapping objects, large blend radii, camera inside."""
    rng = np.random.default_rng(seed)
    spread = [0.5, 1.0, 2.5][seed % 3]
    kmax = [0.05, 0.3, 1.0][(seed // 3) % 3]
    f = random_csg8(rng, spread, kmax)
    if seed % 4 == 3:
        scenes.set_view(f, scenes.orbit_view(float(rng.uniform(-180, 180)),
                                              float(rng.uniform(-20, 20))))
    f.params.precision = abi.PRECISION_EXACT
    a, sa = gpu(renderer, f)
    u = f.copy()
    u.params.dispatch = abi.DISPATCH_UNCULLED
    b, sb = gpu(renderer, u)
    g = f.copy()
    g.params.dispatch = abi.DISPATCH_GENERIC          # generic kernel, culled
    c, sc = gpu(renderer, g)
    for x, sx in ((a, sa), (c, sc)):
        assert np.array_equal(sx, sb)
        assert np.array_equal(x.view(np.uint32), b.view(np.uint32))
    # fast precision: culled vs unculled within the parity policy
    for h in (f, u, g):
        h.params.precision = abi.PRECISION_FAST
    a, sa = gpu(renderer, f)
    b, sb = gpu(renderer, u)
    c, sc = gpu(renderer, g)
    assert_parity(compare(f, a, sa, b, sb, ref_is_oracle=False), what=f"seed {seed}")
    assert_parity(compare(f, c, sc, b, sb, ref_is_oracle=False), what=f"seed {seed} generic")


@pytest.mark.parametrize("light,k", [
    ((5.0, 5.0, 0.0), 10.0),      # the reference's light: slopes b ~ 0.5-0.8
    ((0.3, 40.0, 0.2), 10.0),     # nearly overhead: b above the 0.95 cap
    ((-6.0, 0.75, 2.0), 10.0),    # low light: b around the lim >= 1.01 threshold
    ((4.0, 2.0, -3.0), 2.0),      # soft k: lim < 1 for most slopes
    ((4.0, 2.0, -3.0), 60.0),     # hard k
    ((0.0, 0.3, -0.1), 10.0),     # light inside the cluster sphere
    ((3.0, -1.0, 0.0), 10.0),     # light below the plane: b < 0
    ((4.0, 2.0, -3.0), 0.05),     # tiny k: terms far below s (the exact march's
    ((4.0, 2.0, -3.0), 1.0e4),    # division skip never / almost always applies)
])
@pytest.mark.parametrize("prec", [abi.PRECISION_EXACT, abi.PRECISION_FAST])
def test_shadow_lit_tail_exact(renderer, light, k, prec):
    """The shadow march's lit tail (FixedScene::shadow_limit) ends the march
    early only on the no-steps path; it must not change one output bit.  gpu()
    asserts the no-steps frame equals the steps-on frame (full march) bit for
    bit, here over light positions that put the ray slopes on both sides of
    every condition, four poses, random CSG8 scenes and a tilted plane (a
    run-time specialised kernel with sd_plane as head).  Exact precision is
    also bit-exact with the oracle."""
    frames = [scenes.config("C3", 240, 136, pose=p) for p in range(4)]
    frames += [random_csg8(np.random.default_rng(s), 1.0, 0.3) for s in (3, 4)]
    tilt = scenes.config("C3", 240, 136)
    n = np.array([0.12, 1.0, -0.05]) / np.linalg.norm([0.12, 1.0, -0.05])
    tilt.scene.prims[0].kind = abi.PRIM_PLANE
    tilt.scene.prims[0].p[0], tilt.scene.prims[0].p[1], tilt.scene.prims[0].p[2] = (
        float(n[0]), float(n[1]), float(n[2]))
    frames.append(tilt)
    for i, f in enumerate(frames):
        f.light.pos[0], f.light.pos[1], f.light.pos[2] = light
        f.params.shadow_k = k
        f.params.precision = prec
        rgba, st = gpu(renderer, f)
        if prec == abi.PRECISION_EXACT:
            ref, ref_st = oracle.render(f)
            assert np.array_equal(st, ref_st), f"frame {i}: step counts"
            assert np.array_equal(rgba.view(np.uint32), ref.view(np.uint32)), f"frame {i}"


@pytest.mark.parametrize("normal_mode,h,ao_base,ao_step", [
    (abi.NORMAL_TETRA, -0.01, -0.01, -0.12), (abi.NORMAL_CENTRAL, -0.02, 0.3, -0.2),
    (abi.NORMAL_TETRA, 0.05, -0.4, 0.1)])
def test_culling_exact_with_negative_offsets(renderer, normal_mode, h, ao_base, ao_step):
    """Negative normal_eps / AO offsets are valid parameters (sdf_validate
    accepts any finite value): the culled kernel's path lengths for the
    normal and AO taps use |h|, so it still equals the unculled kernel bit for
    bit (exact precision), step counts included."""
    f = random_csg8(np.random.default_rng(7), 1.0, 0.3)
    f.params.normal_mode = normal_mode
    f.params.normal_eps = h
    f.params.ao_base, f.params.ao_step = ao_base, ao_step
    f.params.precision = abi.PRECISION_EXACT
    a, sa = gpu(renderer, f)
    u = f.copy()
    u.params.dispatch = abi.DISPATCH_UNCULLED
    b, sb = gpu(renderer, u)
    assert np.array_equal(sa, sb)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("peer_root", [False, True])
def test_cpp_frame_driver(renderer, tmp_path, peer_root):
    """The C++ host program's native frame-driver mode (sdf::FrameDriver over
    sdf_driver_*): whole frames at world 1, or with SDF3D_ROOT_AS_PEER=1 the
    multi-rank sequence (TILES, RCCL length all-gather and send/recv to rank
    0 = itself, decode) through a one-rank RCCL communicator whose ids travel
    through files; the last frame equals the Python path's render."""
    import os
    import subprocess
    exe = Path(__file__).resolve().parent.parent / "sdf3d_amd" / "bin" / "sdf_main"
    out = tmp_path / "d.ppm"
    env = dict(os.environ, SDF3D_DRIVER="1", SDF3D_ROOT_AS_PEER="1" if peer_root else "0",
               SDF3D_ID_DIR=str(tmp_path), SDF3D_RUN_ID=f"t{os.getpid()}",
               SDF3D_RCCL="/opt/rocm/lib/librccl.so.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([str(exe), "160", "90", "2", str(out), "csg8"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    assert "rank 0 of 1" in r.stdout
    img = read_ppm(out)
    f = scenes.config("C3", 160, 90, precision=abi.PRECISION_EXACT)   # sdf_main's default
    scenes.set_view(f, scenes.orbit_view(180.0, 0.0))     # frame 1 of 2: yaw 180
    rgba, _ = gpu(renderer, f, steps=False)
    want = quantize(rgba, abi.FORMAT_RGBA8)[::-1, :, :3]
    assert np.abs(img.astype(int) - want.astype(int)).max() <= 1
    assert not list(tmp_path.glob("*.id")), "rank 0 removes the spent id files"
