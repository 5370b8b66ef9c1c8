"""The forced-step replay (oracle.replay, oracle_core.h march_limit) and the
parity policy built on it (tests/parity.py), on the CPU: the replay at the
oracle's own step counts IS the oracle; imposed break points are honoured;
a colour change the step counts do not explain stays undiagnosed; the
readings policy bounds the magnitude of undiagnosed pixels."""
import numpy as np
import pytest

import oracle
from parity import assert_parity, assert_parity_frame, compare, pixel_err, report
from sdf3d_amd import abi, scenes


@pytest.mark.parametrize("cfg,pose", [("REF", 0), ("C3", 1), ("C5", 0), ("C2", 2)])
def test_replay_at_own_steps_is_the_oracle(cfg, pose):
    f = scenes.config(cfg, 96, 54, pose=pose)
    ref, st = oracle.render(f)
    rp, rst = oracle.replay(f, st)
    assert np.array_equal(rp.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(rst, st)


def test_replay_imposes_break_points():
    f = scenes.config("C3", 64, 36, pose=1)
    _, st = oracle.render(f)
    forced = st.copy()
    forced[..., 0] = np.where(np.arange(64)[None, :] % 2 == 0, st[..., 0] + 3, st[..., 0] - 1)
    forced[..., 1] = 5
    _, rst = oracle.replay(f, forced)
    want = np.clip(forced, 0, f.params.max_steps)
    assert np.array_equal(rst[..., 0], want[..., 0])
    # the shadow march runs only where the frame has shadows on (always here)
    assert np.array_equal(rst[..., 1], want[..., 1])


def test_replay_mask_visits_only_masked_pixels():
    f = scenes.config("C3", 48, 24, pose=2)
    ref, st = oracle.render(f)
    m = np.zeros(st.shape[:2], bool)
    m[3, 5] = m[20, 40] = True
    rp, rst = oracle.replay(f, st, mask=m)
    assert np.array_equal(rp[m].view(np.uint32), ref[m].view(np.uint32))
    assert np.isnan(rp[~m]).all() and (rst[~m] == -1).all()


def test_replay_diagnoses_flips_not_colour_changes():
    """A frame computed with a march stopped one step early at some pixels
    (a branch flip) is fully diagnosed; the same step counts with a colour
    change on top (a 'kernel bug' that also moved a break point) are not."""
    f = scenes.config("C3", 96, 54, pose=1)
    ref, st = oracle.render(f)
    flipped = st.copy()
    sel = (st[..., 0] > 3) & (np.arange(96)[None, :] % 7 == 0)
    flipped[sel, 0] -= 1
    g, gst = oracle.replay(f, flipped)
    rep = compare(f, g, gst, ref, st)
    assert rep["outliers"] > 0 and rep["undiagnosed"] == 0, rep
    assert rep["replay_diagnosed"] == rep["outliers"]
    bug = g.copy()
    out = pixel_err(g, ref) > 1e-4
    y, x = np.argwhere(out)[0]
    bug[y, x, 1] += 0.01
    rep2 = compare(f, bug, gst, ref, st)
    assert rep2["undiagnosed"] == 1 and rep2["undiagnosed_max_err"] > 1e-4
    with pytest.raises(AssertionError):
        assert_parity(rep2)
    # equal step counts: never diagnosed, whatever the colour
    same = ref.copy()
    same[0, 0, 0] += 1e-3
    rep3 = compare(f, same, st, ref, st)
    assert rep3["outliers"] == 1 and rep3["undiagnosed"] == 1


def test_pair_comparison_needs_both_sides_explained():
    """Kernel-vs-kernel comparisons (culled vs unculled) diagnose an outlier
    only if the oracle replays reproduce both sides."""
    f = scenes.config("C3", 64, 36, pose=3)
    ref, st = oracle.render(f)
    a_st = st.copy()
    a_st[::5, ::3, 0] = np.maximum(a_st[::5, ::3, 0] - 1, 0)
    a, a_st = oracle.replay(f, a_st)
    rep = compare(f, a, a_st, ref, st, ref_is_oracle=False)
    assert rep["undiagnosed"] == 0
    b = ref.copy()
    b[1, 1, 2] += 0.02
    rep = compare(f, a, a_st, b, st, ref_is_oracle=False)
    assert rep["undiagnosed"] >= 1


def _rep(outliers, undiag, und_max, pixels=10**6, max_err=0.01):
    return {"pixels": pixels, "outliers": outliers, "undiagnosed": undiag,
            "undiagnosed_max_err": und_max, "max_err": max_err, "over_max_err": 0}


def test_readings_policy_counts_and_magnitude():
    strict_ok = {"twin": _rep(3, 0, 0.0), "fma": _rep(2, 0, 0.0)}
    assert assert_parity_frame(_rep(5, 0, 0.0), strict_ok) == "strict"
    with pytest.raises(AssertionError):
        assert_parity_frame(_rep(5, 1, 2e-4), strict_ok)
    ill = {"twin": _rep(400, 120, 0.08, max_err=0.3), "fma": _rep(380, 90, 0.05, max_err=0.2)}
    assert assert_parity_frame(_rep(700, 200, 0.07, max_err=0.5), ill) == "readings"
    with pytest.raises(AssertionError):       # an undiagnosed pixel beyond every reading's
        assert_parity_frame(_rep(700, 200, 0.09), ill)
    with pytest.raises(AssertionError):       # too many undiagnosed (2 x 120 + 3 sigma = 286)
        assert_parity_frame(_rep(700, 300, 0.01), ill)
    # readings without undiagnosed pixels allow none
    flips = {"twin": _rep(40, 0, 0.0, max_err=0.09), "fma": _rep(30, 0, 0.0, max_err=0.14)}
    assert assert_parity_frame(_rep(48, 0, 0.0, max_err=0.72), flips) == "readings"
    with pytest.raises(AssertionError):
        assert_parity_frame(_rep(48, 1, 2e-4), flips)


def test_twin_flips_at_the_reference_scene_are_replay_diagnosed():
    """The fp64 twin's outliers on the reference scene are branch flips the
    fp32 replay at the twin's own step counts reproduces."""
    f = scenes.config("REF", 400, 300, pose=2)
    ref, st = oracle.render(f)
    tw, tst = oracle.render(f, twin=True)
    rep = compare(f, tw, tst, ref, st)
    assert rep["undiagnosed"] == 0, rep


def test_report_without_diagnosis_counts_every_outlier():
    a = np.zeros((2, 2, 4), np.float32)
    b = a.copy()
    b[0, 0, 0] = 1.0
    rep = report(a, None, b, None)
    assert rep["outliers"] == 1 and rep["undiagnosed"] == 1 and rep["over_max_err_undiagnosed"] == 1
    assert abi.PRECISION_EXACT == 0


def test_full_size_conditioning_overrides_a_lucky_small_frame():
    """A small frame whose readings pass the strict policy by chance is still
    held to the readings' spread when its scene and pose fail it at full size
    (the counts scale with the full-size rates)."""
    full = {"strict_at_full_size": False,
            "twin": {"outlier_rate": 2e-4, "undiagnosed_rate": 1.6e-4, "undiagnosed_max_err": 0.4},
            "fma": {"outlier_rate": 1.7e-4, "undiagnosed_rate": 1.5e-4,
                    "undiagnosed_max_err": 0.1}}
    lucky = {"twin": _rep(0, 0, 0.0, pixels=5184), "fma": _rep(0, 0, 0.0, pixels=5184)}
    kern = _rep(1, 1, 1.02e-4, pixels=5184)
    with pytest.raises(AssertionError):
        assert_parity_frame(dict(kern), lucky)
    rep = dict(kern)
    assert assert_parity_frame(rep, lucky, full_size=full) == "readings"
    assert rep["readings_bound"]["undiagnosed_max_err"] == 0.4
    # a scene that passes at full size keeps the strict policy
    full_ok = dict(full, strict_at_full_size=True)
    with pytest.raises(AssertionError):
        assert_parity_frame(dict(kern), lucky, full_size=full_ok)


@pytest.mark.parametrize("cfg", ["C2", "C3", "C4", "C5"])
def test_conditioning_fixture_matches_the_presets(cfg):
    """tests/golden/conditioning.json covers every BASELINE config and pose,
    and its fingerprints are those of the current presets (a changed preset
    must be re-measured with make_conditioning.py)."""
    from parity import full_size_conditioning
    for pose in range(4):
        rec = full_size_conditioning(scenes.config(cfg, 64, 36, pose=pose,
                                                   precision=abi.PRECISION_FAST))
        assert rec is not None, (cfg, pose)
        assert rec["width"] == scenes.CONFIGS[cfg][0]


def test_conditioning_fixture_reproduces_c2():
    """The committed full-size measurement is what make_conditioning.py
    computes (C2 pose 1, 1920x1080, ~3 s)."""
    import json
    from pathlib import Path
    import sys
    here = Path(__file__).resolve().parent / "golden"
    sys.path.insert(0, str(here))
    from make_conditioning import measure
    want = json.loads((here / "conditioning.json").read_text())["C2_p1"]
    assert measure("C2", 1) == want


def test_readings_policy_bounds_pixels_over_max_err():
    """Round 4: replay-diagnosed pixels may exceed MAX_ERR only about as often
    as the readings' own (2x the worst reading's count + 3 sigma)."""
    def rep(over):
        r = _rep(700, 200, 0.07, max_err=0.5)
        r["over_max_err"] = over
        return r
    ill = {"twin": _rep(400, 120, 0.08, max_err=0.3), "fma": _rep(380, 90, 0.05, max_err=0.2)}
    ill["twin"]["over_max_err"], ill["fma"]["over_max_err"] = 3, 2
    r = rep(12)
    assert assert_parity_frame(r, ill) == "readings"          # 2 * 3 + 3 sqrt 6 = 13.3
    assert r["readings_bound"]["over_max_err"] == pytest.approx(6 + 3 * 6 ** 0.5)
    with pytest.raises(AssertionError):
        assert_parity_frame(rep(14), ill)
    # a full-size rate scales to the frame
    full = {"strict_at_full_size": False, "width": 1000, "height": 1000,
            "twin": {"outlier_rate": 4e-4, "undiagnosed_rate": 1.2e-4, "undiagnosed_max_err": 0.08,
                     "over_max_err": 30},
            "fma": {"outlier_rate": 4e-4, "undiagnosed_rate": 1.2e-4, "undiagnosed_max_err": 0.08,
                    "over_max_err": 10}}
    assert assert_parity_frame(rep(70), ill, full_size=full) == "readings"   # 60 + 3 sqrt 60


def test_fast_regression_bounds():
    """Full-size fast frames are held to the kernel's own last measurement
    (tests/golden/fast_regression.json), inside the readings' spread."""
    from parity import assert_regression, regression_bound
    b = regression_bound("C5_p0")
    m = b["measured"]
    assert b["undiagnosed_max_err"] < 0.482      # tighter than the readings' magnitude
    ok = {k: m[k] for k in ("outliers", "undiagnosed", "over_max_err", "undiagnosed_max_err",
                            "max_err")}
    assert assert_regression(dict(ok), "C5_p0") is not None
    for k, v in (("undiagnosed", 2 * m["undiagnosed"]), ("undiagnosed_max_err", 0.45),
                 ("over_max_err", 3 * m["over_max_err"] + 10)):
        bad = dict(ok)
        bad[k] = v
        with pytest.raises(AssertionError):
            assert_regression(bad, "C5_p0")
    assert regression_bound("nope_p9") is None
    for cfg in ("C2", "C3", "C4", "C5"):
        assert regression_bound(f"{cfg}_p0") is not None
