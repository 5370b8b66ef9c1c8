"""GPU tests of the run-time scene specialiser (sdf3d_amd/csrc/jit.cpp).

A primitive scene whose (kind, op) sequence matches no built-in variant is
rendered, under SDF_DISPATCH_AUTO, by a FixedScene kernel compiled with hipRTC
for that sequence.  It must equal the unculled generic kernel bit for bit in
exact precision (step counts included) and within the parity policy in fast
precision, exactly as the built-in variants do (test_gpu_parity.py
test_specialised_matches_generic, test_culling_exact_on_random_scenes).
"""
import os

import numpy as np
import pytest

from parity import assert_parity, compare
from sdf3d_amd import abi, scenes

pytestmark = pytest.mark.gpu


def gpu(rd, frame, steps=True):
    import torch
    rgba, st = rd.render(frame, steps=steps)
    torch.cuda.synchronize()
    return rgba.cpu().numpy(), (st.cpu().numpy() if st is not None else None)


def jit_count(rd):
    return rd.lib.sdf_jit_count()


def custom_scene(rng, n, w=160, h=90):
    """n random primitives after the plane, random kinds and (union-family or
    CSG) ops: signatures no built-in variant has."""
    f = scenes.config("C3", w, h)
    f.scene.count = 1 + n
    kinds = [abi.PRIM_SPHERE, abi.PRIM_BOX, abi.PRIM_ROUND_BOX, abi.PRIM_TORUS,
             abi.PRIM_CAPSULE, abi.PRIM_CYLINDER]
    for i in range(1, 1 + n):
        p = f.scene.prims[i]
        p.kind = int(rng.choice(kinds))
        p.op = int(rng.choice([abi.OP_UNION, abi.OP_SMOOTH_UNION, abi.OP_SMOOTH_UNION,
                               abi.OP_SUBTRACT, abi.OP_INTERSECT, abi.OP_SMOOTH_SUBTRACT]))
        p.k = float(rng.uniform(0.02, 0.4))
        c = rng.uniform(-0.8, 0.8, 3) + np.array([0.0, 0.45, 0.0])
        vals = list(c) + list(rng.uniform(0.08, 0.3, 6))
        if p.kind == abi.PRIM_CAPSULE:
            vals = list(c) + list(c + rng.uniform(-0.4, 0.4, 3)) + [float(rng.uniform(0.05, 0.15))]
        if p.kind == abi.PRIM_ROUND_BOX:
            vals[6] = float(rng.uniform(0.01, 0.05))
        for j, v in enumerate(vals[:9]):
            p.p[j] = float(v)
    return f


@pytest.mark.parametrize("seed", range(8))
def test_jit_kernel_matches_unculled(renderer, seed):
    rng = np.random.default_rng(100 + seed)
    f = custom_scene(rng, 2 + seed % 7)
    before = jit_count(renderer)
    for prec in (abi.PRECISION_EXACT, abi.PRECISION_FAST):
        f.params.precision = prec
        a, sa = gpu(renderer, f)
        u = f.copy()
        u.params.dispatch = abi.DISPATCH_UNCULLED
        b, sb = gpu(renderer, u)
        if prec == abi.PRECISION_EXACT:
            assert np.array_equal(sa, sb)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
        else:
            assert_parity(compare(f, a, sa, b, sb, ref_is_oracle=False), what=f"jit seed {seed}")
    # a new signature compiles once per precision; the second frame reuses it
    assert jit_count(renderer) - before in (0, 1, 2)
    n = jit_count(renderer)
    gpu(renderer, f)
    assert jit_count(renderer) == n


def test_jit_used_for_unmatched_signature_only(renderer):
    """Built-in variants stay built-in; a reordered CSG8 list is compiled."""
    f = scenes.config("C3", 96, 64)
    n0 = jit_count(renderer)
    gpu(renderer, f)                         # built-in variant 3
    assert jit_count(renderer) == n0
    g = f.copy()
    g.scene.prims[1], g.scene.prims[2] = g.scene.prims[2], g.scene.prims[1]
    a, sa = gpu(renderer, g)
    assert jit_count(renderer) == n0 + 1
    u = g.copy()
    u.params.dispatch = abi.DISPATCH_UNCULLED
    u.params.precision = g.params.precision = abi.PRECISION_EXACT
    a, sa = gpu(renderer, g)
    b, sb = gpu(renderer, u)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(sa, sb)


def test_jit_disabled_falls_back_to_generic(renderer):
    rng = np.random.default_rng(7)
    f = custom_scene(rng, 3)
    f.scene.prims[1].kind = abi.PRIM_CYLINDER      # a signature of its own
    f.scene.prims[2].kind = abi.PRIM_CYLINDER
    f.params.precision = abi.PRECISION_EXACT
    os.environ["SDF3D_JIT"] = "0"
    try:
        n0 = jit_count(renderer)
        a, sa = gpu(renderer, f)
        assert jit_count(renderer) == n0
    finally:
        del os.environ["SDF3D_JIT"]
    b, sb = gpu(renderer, f)                   # now specialised
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(sa, sb)


def test_jit_tiles_output(renderer):
    """The specialised kernel's TILES instantiation round-trips losslessly."""
    import torch
    rng = np.random.default_rng(11)
    f = custom_scene(rng, 4, 120, 72)
    ref, _ = gpu(renderer, f, steps=False)
    t = f.copy()
    t.params.output_format = abi.FORMAT_TILES
    st, _ = renderer.render(t)
    out = renderer.tiles_decode(st, 1, st.numel(), 120, 72)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
