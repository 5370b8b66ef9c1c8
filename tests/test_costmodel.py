"""Algorithmic cost model (SURVEY.md 8(d) counting rule)."""
import numpy as np
import pytest

from sdf3d_amd import abi, costmodel, scenes


def test_reference_scene_matches_survey_per_step_terms():
    c = costmodel.coefficients(scenes.reference())
    # 20 * S_p + 30 * S_s flops, 1 * S_p + 4 * S_s SFU
    assert (c.primary_flops, c.shadow_flops) == (20, 30)
    assert (c.primary_sfu, c.shadow_sfu) == (1, 4)
    assert c.fixed_flops == 191 and c.fixed_sfu == 31   # survey: ~183 / 32 (see module doc)


def test_csg8_eval_cost():
    s = scenes.config("C4").scene
    f, u = costmodel.scene_eval_cost(s)
    prims = 0 + 9 + 18 + 11 + 22 + 16 + 19 + 9
    ops = 1 + 7 * 8
    assert f == prims + ops
    assert u == (0 + 1 + 1 + 2 + 2 + 2 + 1 + 1) + 7


def test_primary_only_has_no_shadow_terms():
    c = costmodel.coefficients(scenes.config("C2"))
    assert c.shadow_flops == 0 and c.shadow_sfu == 0
    assert c.fixed_flops == 191 - 11


def test_c4_flops_per_pixel_from_stats():
    f = scenes.config("C4")
    c = costmodel.coefficients(f)
    z = np.load("tests/golden/stats_C4_p0.npz")
    n = int(z["width"]) * int(z["height"])
    fl = c.flops(n, z["row_sp"].sum(), z["row_ss"].sum()) / n
    assert 8000 < fl < 12000


def test_mandelbulb_has_no_static_model():
    with pytest.raises(ValueError):
        costmodel.scene_eval_cost(scenes.config("C5").scene)
