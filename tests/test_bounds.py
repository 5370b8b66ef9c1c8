"""Host-side culling bounds (no GPU): sdf_scene_bounds returns the bounding
spheres the fixed-scene kernels cull with (sdf_abi.cpp prepare_bounds).  Exact
culling is only exact if every primitive lies inside its own sphere and every
cullable primitive inside the cluster sphere; these tests restate each
kind's radius independently and check the containment, and that the cluster
sphere (a minimax centre since round 2) is never larger than the centroid
one it replaced (render_kernel.inc: the smaller it is, the more the culling
and the shadow march's lit tail skip)."""
import ctypes as C

import numpy as np
import pytest

from sdf3d_amd import abi, scenes

ABS, REL = 1e-4, 1e-5
SMOOTH = (abi.OP_SMOOTH_UNION,)


def bounds_of(scene):
    lib = abi.load_library()
    b = (C.c_float * (4 * abi.SDF_MAX_PRIMS))()
    c = (C.c_float * 4)()
    first = C.c_int32()
    rc = lib.sdf_scene_bounds(C.byref(scene), b, c, C.byref(first))
    return rc, np.array(b, dtype=np.float64).reshape(-1, 4), np.array(c, dtype=np.float64), first.value


def sphere_of(pr):
    """Centre and radius of a sphere containing the primitive (its own
    statement of the shapes in render_kernel.inc)."""
    p = np.array(pr.p, dtype=np.float64)
    c = p[0:3].copy()
    if pr.kind == abi.PRIM_SPHERE:
        r = p[3]
    elif pr.kind == abi.PRIM_BOX:
        r = np.linalg.norm(p[3:6])
    elif pr.kind == abi.PRIM_ROUND_BOX:       # the box b - r rounded by r
        r = np.linalg.norm(np.maximum(p[3:6] - p[6], 0.0)) + abs(p[6])
    elif pr.kind == abi.PRIM_TORUS:
        r = p[3] + p[4]
    elif pr.kind == abi.PRIM_CAPSULE:
        c = 0.5 * (p[0:3] + p[3:6])
        r = 0.5 * np.linalg.norm(p[3:6] - p[0:3]) + p[6]
    elif pr.kind == abi.PRIM_CYLINDER:
        r = np.hypot(p[3], p[4])
    else:
        r = 0.0
    return c, abs(r)


def random_scene(rng, n):
    f = scenes.config("C3", 64, 64)
    s = f.scene
    C.memset(C.addressof(s.prims), 0, C.sizeof(s.prims))
    s.count = n
    u = lambda a, b: float(rng.uniform(a, b))  # noqa: E731
    s.prims[0].kind, s.prims[0].op = abi.PRIM_PLANE, abi.OP_UNION
    s.prims[0].p[1] = 1.0
    kinds = [abi.PRIM_SPHERE, abi.PRIM_BOX, abi.PRIM_ROUND_BOX, abi.PRIM_TORUS,
             abi.PRIM_CAPSULE, abi.PRIM_CYLINDER]
    for i in range(1, n):
        pr = s.prims[i]
        pr.kind = kinds[int(rng.integers(len(kinds)))]
        pr.op = abi.OP_SMOOTH_UNION if rng.random() < 0.8 else abi.OP_UNION
        pr.k = u(1e-3, 0.5)
        for j in range(3):
            pr.p[j] = u(-3, 3)
        if pr.kind == abi.PRIM_CAPSULE:
            for j in range(3, 6):
                pr.p[j] = u(-3, 3)
            pr.p[6] = u(0.01, 0.5)
        else:
            for j in range(3, 6):
                pr.p[j] = u(0.01, 1.0)
            pr.p[6] = u(0.0, 0.05)
    return f.scene


def check_containment(scene):
    rc, b, cl, first = bounds_of(scene)
    assert rc == 0
    n = scene.count
    centres, radii, ks = [], [], []
    for i in range(n):
        pr = scene.prims[i]
        c, r = sphere_of(pr)
        k = pr.k if pr.op in SMOOTH else 0.0
        if i >= first:
            # the kernel's per-primitive bound: K_i >= (k + R + abs) / (1 - rel)
            assert np.allclose(b[i, :3], c, rtol=0, atol=1e-6 * (1 + np.abs(c))), i
            assert b[i, 3] >= (k + r + ABS) / (1 - REL) * (1 - 1e-6), i
            centres.append(c)
            radii.append(r)
            ks.append(k)
    if first >= n:
        return None
    centres, radii = np.array(centres), np.array(radii)
    kmax = max(ks)
    rc_cluster = cl[3] * (1 - REL) - ABS - kmax   # the radius the cluster bound encloses
    far = np.linalg.norm(centres - cl[:3], axis=1) + radii
    assert np.all(far <= rc_cluster * (1 + 1e-6) + 1e-9), (far.max(), rc_cluster)
    centroid = centres.mean(axis=0)
    rc_centroid = (np.linalg.norm(centres - centroid, axis=1) + radii).max()
    return rc_cluster, rc_centroid


def test_csg8_cluster_sphere():
    f = scenes.config("C4", 64, 64)
    rc_cluster, rc_centroid = check_containment(f.scene)
    assert abs(rc_centroid - 1.2088) < 2e-3       # the centroid sphere round 1 used (1.2219 with
                                                    # its looser round-box sphere)
    assert rc_cluster < 1.04                        # the minimax sphere: 1.033
    _, _, _, first = bounds_of(f.scene)
    assert first == 1                               # the plane heads the list, the rest is culled


@pytest.mark.parametrize("seed", range(40))
def test_random_scenes_contained_and_tighter(seed):
    rng = np.random.default_rng(seed)
    scene = random_scene(rng, int(rng.integers(2, abi.SDF_MAX_PRIMS + 1)))
    res = check_containment(scene)
    if res is not None:
        rc_cluster, rc_centroid = res
        # rc_cluster carries the bound's rounding margins (~1e-6 relative
        # and absolute, twice) and the fp32 rounding of the centre
        assert rc_cluster <= rc_centroid * (1 + 1e-5) + 1e-5


def test_bounds_cache_follows_the_scene():
    """The cluster search is cached per primitive list: alternating scenes
    must each get their own answer."""
    rng = np.random.default_rng(99)
    a, b = random_scene(rng, 6), random_scene(rng, 7)
    ra, rb = bounds_of(a), bounds_of(b)
    for _ in range(3):
        for s, ref in ((a, ra), (b, rb), (a, ra)):
            got = bounds_of(s)
            assert got[0] == ref[0] and got[3] == ref[3]
            assert np.array_equal(got[1], ref[1]) and np.array_equal(got[2], ref[2])


def test_bounds_refusals():
    f = scenes.config("C5", 64, 64)
    rc, *_ = bounds_of(f.scene)
    assert rc == abi.SDF_E_UNSUPPORTED
    g = scenes.config("C4", 64, 64)
    g.scene.prims[3].p[0] = float("nan")
    rc, *_ = bounds_of(g.scene)
    assert rc == abi.SDF_E_INVALID_ARG


@pytest.mark.parametrize("kind", [abi.PRIM_SPHERE, abi.PRIM_BOX, abi.PRIM_ROUND_BOX,
                                  abi.PRIM_TORUS, abi.PRIM_CAPSULE, abi.PRIM_CYLINDER])
def test_primitive_solid_lies_inside_its_sphere(kind):
    """Geometric check, independent of any radius formula: points
    where the ORACLE's own SDF of the primitive is <= 0 (the solid) must lie
    inside the bound the kernel culls with -- including rounded boxes whose
    rounding radius exceeds a half extent (r > b on some axes, the branch the
    round-box sphere |max(b - r, 0)| + r clamps)."""
    import oracle
    rng = np.random.default_rng(1000 + kind)
    checked = 0
    for trial in range(12):
        f = scenes.config("C3", 64, 64)
        s = f.scene
        C.memset(C.addressof(s.prims), 0, C.sizeof(s.prims))
        s.count = 2
        s.prims[0].kind, s.prims[0].op = abi.PRIM_PLANE, abi.OP_UNION
        s.prims[0].p[1], s.prims[0].p[3] = 1.0, 1e3      # far below: never the minimum
        pr = s.prims[1]
        pr.kind, pr.op, pr.k = kind, abi.OP_SMOOTH_UNION, 0.05
        for j in range(3):
            pr.p[j] = float(rng.uniform(-1, 1))
        if kind == abi.PRIM_CAPSULE:
            for j in range(3, 6):
                pr.p[j] = float(rng.uniform(-1, 1))
            pr.p[6] = float(rng.uniform(0.02, 0.4))
        else:
            for j in range(3, 6):
                pr.p[j] = float(rng.uniform(0.05, 0.6))
            if kind == abi.PRIM_ROUND_BOX:
                # r beyond the smallest half extent on alternate trials
                bmin = min(pr.p[3], pr.p[4], pr.p[5])
                pr.p[6] = float(rng.uniform(1.05, 2.0) * bmin if trial % 2 else
                                rng.uniform(0.0, 0.9) * bmin)
        rc, b, cl, first = bounds_of(s)
        assert rc == 0 and first == 1
        cen, K = b[1, :3], b[1, 3]
        R = K * (1 - REL) - ABS - pr.k          # the radius the bound encloses
        ext = 2.5
        pts = rng.uniform(-ext, ext, size=(6000, 3)) + np.array(pr.p[0:3])
        # the primitive alone: the plane term is 1e3 above every sample
        inside = [p for p in pts if oracle.scene_sdf(s, *map(float, p)) <= 0.0]
        for p in inside:
            assert np.linalg.norm(p - cen) <= R * (1 + 1e-6) + 1e-6, (kind, trial, p, R)
        checked += len(inside)
    assert checked > 100, checked
