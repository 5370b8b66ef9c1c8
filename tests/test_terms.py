"""The shading terms that SDF_FORMAT_SHADE32F renders and the TILES wire
carries (include/sdf_abi.h; sdf3d_amd/csrc/shade.h), on the CPU oracle.

The colour is la * amb * ao + dif * mat.dif + pow(x, shininess) * mat.ref
(voxel_fragment.frag:204-210 plus the AO extension): made from the oracle's
own terms in the restatement's operation order, it must be the oracle's
colour bit for bit -- the formula shade.h's exact precision restates (the
GPU tests check the kernel's terms against these, tests/test_gpu_tiles.py).
"""
import numpy as np
import pytest

import oracle
from sdf3d_amd import abi, scenes


@pytest.mark.parametrize("cfg,pose", [("REF", 0), ("C1", 1), ("C2", 2), ("C3", 0), ("C3", 3),
                                      ("C5", 1)])
def test_colour_from_terms_is_the_oracle_colour(cfg, pose):
    f = scenes.config(cfg, 96, 54, pose=pose, precision=abi.PRECISION_EXACT)
    rgba, _ = oracle.render(f)
    terms = oracle.render_terms(f)
    assert np.all(terms[..., 3] == 1.0)
    col = oracle.colour_from_terms(f, terms)
    assert np.array_equal(col.view(np.uint32), rgba.view(np.uint32))


@pytest.mark.parametrize("flags", [0, abi.FLAG_SHADOW, abi.FLAG_AO, abi.FLAG_SHADOW | abi.FLAG_AO])
def test_terms_follow_the_feature_flags(flags):
    """ao is 1 without AO; without a shadow dif is clamp(N.L, 0, 1) alone, so
    turning the shadow off can only raise it; the specular term ignores both."""
    f = scenes.config("C3", 64, 40, pose=1, precision=abi.PRECISION_EXACT)
    f.params.flags = flags
    t = oracle.render_terms(f)
    g = f.copy()
    g.params.flags = flags & ~abi.FLAG_SHADOW
    t_lit = oracle.render_terms(g)
    if not flags & abi.FLAG_AO:
        assert np.all(t[..., 0] == 1.0)
    assert np.all(t[..., 1] <= t_lit[..., 1])
    assert np.array_equal(t[..., 2], t_lit[..., 2])
    assert np.all((t[..., 2] >= 0) & (t[..., 1] >= 0) & (t[..., 1] <= 1))
