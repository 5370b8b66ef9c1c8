"""Frame sequences (sdf_render_frames, sdf3d_amd/csrc/frames.cpp): the
persistent kernel's frames equal one sdf_render per camera bit for bit, in
every precision, format and scene kind, across launch boundaries (16 frames
per launch), with step counts; and against the oracle at a parity size."""
import numpy as np
import pytest
import torch

from parity import assert_parity, report

pytestmark = pytest.mark.gpu


def _cams(cfg, W, H, prec, n):
    from sdf3d_amd import scenes
    frames = [scenes.config(cfg, W, H, precision=prec, pose=i % 4) for i in range(n)]
    for i, f in enumerate(frames):   # distinct cameras beyond the 4 poses
        if i >= 4:
            scenes.set_view(f, scenes.orbit_view(7.0 * i, 3.0 - i))
    return frames


def _check(rd, frames, fmt=None, with_steps=False):
    base = frames[0]
    if fmt is not None:
        for f in frames:
            f.params.output_format = fmt
    outs, steps = [], []
    for f in frames:
        o, st = rd.alloc(f, steps=with_steps)
        outs.append(o.fill_(7))
        if with_steps:
            steps.append(st.fill_(-1))
    rd.render_frames(base, [f.camera for f in frames], outs, steps if with_steps else None)
    torch.cuda.synchronize()
    for i, f in enumerate(frames):
        ref, rst = rd.render(f, steps=with_steps)
        torch.cuda.synchronize()
        assert torch.equal(outs[i].view(torch.uint8), ref.view(torch.uint8)), i
        if with_steps:
            assert torch.equal(steps[i], rst), i


@pytest.mark.parametrize("cfg,W,H,prec,n", [
    ("C4", 3840, 2160, 1, 3), ("C3", 320, 180, 0, 5), ("C3", 321, 179, 1, 17),
    ("C5", 256, 144, 1, 4), ("C2", 480, 270, 1, 2), ("REF", 37, 23, 0, 33),
    ("C1", 64, 64, 1, 1)])
def test_frames_match_single_renders(cfg, W, H, prec, n):
    from sdf3d_amd import Renderer
    rd = Renderer("cuda:0")
    _check(rd, _cams(cfg, W, H, prec, n))


@pytest.mark.parametrize("fmt", [1, 2, 3])
def test_frames_formats_and_steps(fmt):
    from sdf3d_amd import Renderer
    rd = Renderer("cuda:0")
    _check(rd, _cams("C3", 200, 112, 1, 3), fmt=fmt, with_steps=True)


def test_frames_generic_and_jit_scenes():
    """A dispatch-generic scene runs the persistent generic kernel; a scene
    with no built-in variant goes through its run-time specialised kernel,
    one launch per frame -- both equal sdf_render."""
    from sdf3d_amd import Renderer, abi
    rd = Renderer("cuda:0")
    frames = _cams("C3", 160, 90, 1, 3)
    for f in frames:
        f.params.dispatch = abi.DISPATCH_GENERIC
    _check(rd, frames)
    frames = _cams("C3", 160, 90, 1, 3)
    for f in frames:   # swap two primitives: no built-in signature
        p = f.scene.prims
        tmp = abi.sdf_primitive.from_buffer_copy(p[2])
        p[2] = p[3]
        p[3] = tmp
    _check(rd, frames)


def test_frames_oracle_parity():
    """The bench path of a sequence (no steps buffer: shadow skip active)
    against the oracle, exact precision, strict policy."""
    import oracle
    from sdf3d_amd import Renderer, abi
    rd = Renderer("cuda:0")
    frames = _cams("C3", 160, 90, abi.PRECISION_EXACT, 2)
    outs = [rd.alloc(f)[0] for f in frames]
    rd.render_frames(frames[0], [f.camera for f in frames], outs)
    torch.cuda.synchronize()
    for f, o in zip(frames, outs):
        ref, ref_steps = oracle.render(f)
        rep = report(o.cpu().numpy(), None, ref, ref_steps)
        assert_parity(rep, "frames/C3")
        assert rep["bit_exact"] == rep["pixels"]


def test_frames_rejects_bad_arguments():
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    f = scenes.config("C3", 64, 32, precision=abi.PRECISION_FAST)
    lib = abi.load_library()
    import ctypes as C
    o = rd.alloc(f)[0]
    cams = (abi.sdf_camera * 2)(f.camera, f.camera)
    ptrs = (C.c_void_p * 2)(o.data_ptr(), None)
    args = (C.byref(f.scene), cams, 2, C.byref(f.light), C.byref(f.material), C.byref(f.params))
    assert lib.sdf_render_frames(*args, ptrs, None, None) == abi.SDF_E_INVALID_ARG
    assert lib.sdf_render_frames(*args[:2], -1, *args[3:], ptrs, None, None) == \
        abi.SDF_E_INVALID_ARG
    assert lib.sdf_render_frames(*args[:2], 0, *args[3:], ptrs, None, None) == abi.SDF_OK
    bad = (abi.sdf_camera * 2)(f.camera, f.camera)
    bad[1].view[0] = float("nan")
    ptrs = (C.c_void_p * 2)(o.data_ptr(), o.data_ptr())
    assert lib.sdf_render_frames(args[0], bad, 2, *args[3:], ptrs, None, None) == \
        abi.SDF_E_INVALID_ARG
    g = f.copy()
    g.params.output_format = abi.FORMAT_TILES
    assert lib.sdf_render_frames(C.byref(g.scene), cams, 2, C.byref(g.light),
                                 C.byref(g.material), C.byref(g.params), ptrs, None,
                                 None) == abi.SDF_E_UNSUPPORTED
    # the refused calls left no stale HIP error: a normal render still works
    rd.render(f, out=o)
    torch.cuda.synchronize()
    assert np.isfinite(o.cpu().numpy()).all()
