"""Algorithmic cost model of the per-pixel hot path (SURVEY.md 8(d) counting rule).

Counting rule: add, sub, mul, min, max and compare = 1 flop each (an FMA would
be 2, but the algorithm is written with separate mul/add); negation and abs are
free (input modifiers); sqrt, div, pow, log = 1 SFU op each, reported
separately; uniform-only work (inverse(V_mat), camera.pos, the focal term,
dot(ba,ba) of a capsule, b - r of a rounded box, per-tap AO heights and
weights) is excluded; dead code (`reflect`, voxel_fragment.frag:202) is
excluded.  Step counts S_p (primary) and S_s (shadow) per pixel come from the
CPU oracle, never from the GPU.

Per pixel:
    flops = F_fixed + (9 + C) * S_p + (19 + C) * S_s
    sfu   = U_fixed + C_sfu * S_p + (3 + C_sfu) * S_s
with C / C_sfu the cost of one sceneSDF evaluation.  For the reference scene
(plane + sphere, hard min: C = 11, C_sfu = 1) the per-step terms are the
survey's 20 * S_p + 30 * S_s and 1 * S_p + 4 * S_s exactly; the fixed part
itemised below is 191 flops / 31 SFU (the survey quotes ~183 / 32 without an
itemisation; the 8-flop gap is the vec3 offsets p +- DX, counted here as the
three subtractions GLSL writes).
"""
from __future__ import annotations

from dataclasses import dataclass

from . import abi

# (flops, sfu) per primitive evaluation, as written in DESIGN.md "Scene spec"
PRIM_COST = {
    abi.PRIM_SPHERE: (9, 1),      # p - c (3), dot (5), sqrt, - r (1)
    abi.PRIM_BOX: (18, 1),        # p-c (3), |.|-b (3), max0 x3 (3), length (5, sqrt), inside (3), + (1)
    abi.PRIM_ROUND_BOX: (19, 1),  # box + final - r
    abi.PRIM_TORUS: (11, 2),      # p-c (3), xz len (3, sqrt), - R (1), len (3, sqrt), - r (1)
    abi.PRIM_CAPSULE: (22, 2),    # pa (3), dot (5), div, clamp (2), ba*h (3), pa- (3), len (5, sqrt), -r (1)
    abi.PRIM_CYLINDER: (16, 2),   # p-c (3), xz len (3, sqrt), -r (1), |y|-hh (1), in (2), max0 x2 (2), len (3, sqrt), + (1)
}
OP_COST = {
    abi.OP_UNION: (1, 0), abi.OP_SUBTRACT: (1, 0), abi.OP_INTERSECT: (1, 0),
    # smin: a-b, k-|.|, max, /k (SFU), min, h*h, *k, *0.25, sub
    abi.OP_SMOOTH_UNION: (8, 1), abi.OP_SMOOTH_SUBTRACT: (8, 1), abi.OP_SMOOTH_INTERSECT: (8, 1),
}


def plane_cost(p) -> tuple[int, int]:
    """planeSDF is p.y in the reference (voxel_fragment.frag:68): 0 flops.  An
    axis-aligned unit normal costs 0 (+1 for a nonzero offset); a general
    normal is dot(p, n) + h = 6."""
    n = [p[0], p[1], p[2]]
    axis = sorted(abs(v) for v in n) == [0.0, 0.0, 1.0]
    if axis:
        return (0 if p[3] == 0.0 else 1, 0)
    return (6, 0)


def scene_eval_cost(scene: abi.sdf_scene) -> tuple[int, int]:
    """(flops, sfu) of one sceneSDF evaluation of a primitive scene."""
    if scene.kind != abi.SCENE_PRIMITIVES:
        raise ValueError("data-dependent cost (Mandelbulb iterations): no static model")
    f = u = 0
    for i in range(scene.count):
        pr = scene.prims[i]
        pf, pu = plane_cost(pr.p) if pr.kind == abi.PRIM_PLANE else PRIM_COST[pr.kind]
        of, ou = OP_COST[pr.op]
        f += pf + of
        u += pu + ou
    return f, u


@dataclass
class Coefficients:
    fixed_flops: int
    primary_flops: int
    shadow_flops: int
    fixed_sfu: int
    primary_sfu: int
    shadow_sfu: int

    def flops(self, sum_pixels, sum_sp, sum_ss) -> float:
        return (self.fixed_flops * float(sum_pixels) + self.primary_flops * float(sum_sp)
                + self.shadow_flops * float(sum_ss))

    def sfu(self, sum_pixels, sum_sp, sum_ss) -> float:
        return (self.fixed_sfu * float(sum_pixels) + self.primary_sfu * float(sum_sp)
                + self.shadow_sfu * float(sum_ss))


def coefficients(frame) -> Coefficients:
    """Per-pixel cost coefficients of `frame` (sdf3d_amd.scenes.Frame)."""
    p = frame.params
    c, cu = scene_eval_cost(frame.scene)
    taps = 4 if p.normal_mode == abi.NORMAL_TETRA else 6
    ff, fu = 0, 0
    ff += 32; fu += 8                   # ray: qx*AR, normalize, inverse(V)*(r,0), normalize
    ff += 6                             # P = cam + d*ray
    ff += 26 + taps * c; fu += 4 + taps * cu   # normal offsets/differences, normalize
    ff += 30; fu += 13                  # view, incident, halfway (normalize x3), dot/max, pow
    ff += 8                             # clamp(dot(N, L)) * shadow
    ff += 12                            # dif*M.dif + spec*M.ref + sums
    shadow = bool(p.flags & abi.FLAG_SHADOW)
    if shadow:
        ff += 11                        # origin P + N*2*eps (9), final clamp (2)
    if (p.flags & abi.FLAG_AO) and p.ao_taps > 0:
        ff += p.ao_taps * (9 + c) + 7   # P + N*h (6), occ update (3); 1 - s*occ, clamp, amb*ao
        fu += p.ao_taps * cu
    return Coefficients(ff, 9 + c, (19 + c) if shadow else 0, fu, cu, (3 + cu) if shadow else 0)
