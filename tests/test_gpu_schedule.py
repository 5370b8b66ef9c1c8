"""Render schedules (include/sdf_abi.h sdf_schedule, sdf_render_scheduled):
the row blocks are dispatched costliest first once the kernels' cost
counters have been read back, and every frame stays bit-identical to
sdf_render's -- any order renders every 8-row block exactly once (plain
formats, TILES streams, step counts, tilings, both precisions)."""
import numpy as np
import pytest

from sdf3d_amd import abi, renderer as R, scenes

pytestmark = pytest.mark.gpu


def _same(a, b):
    import torch
    if a.dtype == torch.uint8 and a.dim() == 1:   # TILES: the stream, not the scratch after it
        n = R.tiles_stream_bytes(a)
        return n == R.tiles_stream_bytes(b) and torch.equal(a[:n], b[:n])
    return torch.equal(a.contiguous().view(torch.uint8), b.contiguous().view(torch.uint8))


@pytest.mark.parametrize("cfg,w,h,pose,prec,fmt,tiling", [
    ("C3", 160, 90, 1, abi.PRECISION_FAST, abi.FORMAT_RGBA32F, None),
    ("C3", 200, 120, 2, abi.PRECISION_EXACT, abi.FORMAT_RGBA32F, None),
    ("C5", 96, 72, 0, abi.PRECISION_EXACT, abi.FORMAT_RGBA32F, None),
    ("REF", 128, 96, 3, abi.PRECISION_FAST, abi.FORMAT_RGBA8, None),
    ("C3", 160, 90, 1, abi.PRECISION_FAST, abi.FORMAT_TILES, None),
    ("C3", 192, 136, 0, abi.PRECISION_FAST, abi.FORMAT_RGBA32F, (1, 3, (1, 1))),
    ("C3", 192, 136, 0, abi.PRECISION_FAST, abi.FORMAT_TILES, (2, 4, (3, 4))),
    ("C2", 128, 72, 0, abi.PRECISION_FAST, abi.FORMAT_RGBA32F, (0, 8, (2, 7))),
])
def test_scheduled_render_is_bit_identical(renderer, cfg, w, h, pose, prec, fmt, tiling):
    import torch
    f = scenes.config(cfg, w, h, precision=prec, pose=pose)
    f.params.output_format = fmt
    t = None if tiling is None else R.tiling(tiling[0], tiling[1], 8, shares=tiling[2])
    ref, _ = renderer.render(f, t)
    torch.cuda.synchronize()
    rows = R.owned_rows(h, t)
    sch = renderer.schedule(rows, period=1)
    orders = []
    for _ in range(4):
        out, _ = renderer.render(f, t, schedule=sch)
        torch.cuda.synchronize()
        assert _same(out, ref)
        orders.append(sch.order())
    # the first launch ran in launch order; the later ones in a measured order
    nb = (rows + 7) // 8
    assert orders[0] == [] and sorted(orders[-1]) == list(range(nb)), orders[-1]
    if nb > 4:
        assert orders[-1] != list(range(nb))
    sch.close()


def test_scheduled_steps_and_other_shapes(renderer):
    """Step counts come out identical; a render whose row count is not the
    schedule's runs in launch order (and correctly)."""
    import torch
    f = scenes.config("C3", 120, 80, precision=abi.PRECISION_EXACT, pose=1)
    ref, rst = renderer.render(f, steps=True)
    sch = renderer.schedule(80)
    for _ in range(3):
        out, st = renderer.render(f, steps=True, schedule=sch)
        torch.cuda.synchronize()
        assert _same(out, ref) and _same(st, rst)
    g = scenes.config("C3", 120, 64, precision=abi.PRECISION_EXACT, pose=1)
    ref2, _ = renderer.render(g)
    out2, _ = renderer.render(g, schedule=sch)
    torch.cuda.synchronize()
    assert _same(out2, ref2)
    sch.close()
