"""Parity policy between the HIP kernel and the CPU oracle.

A pixel's error is its largest per-channel |delta| over RGBA; an OUTLIER is a
pixel whose error exceeds `tol` (1e-4).

DIAGNOSIS is by forced-step REPLAY (round 3).  The
oracle is re-run on the outlier pixels with the kernel's own recorded
(primary, shadow) iteration counts imposed as the marches' break points
(oracle.replay, oracle_core.h march_limit; voxel_fragment.frag:86-103,
:105-132).  An outlier is DIAGNOSED only if that replay reproduces the
kernel's value within `tol`: the whole difference is then explained by
where a march stopped (a branch flip of the break tests :97-99 / :126), and
the kernel's arithmetic on either side of the flip agrees with the oracle's.
A pixel whose step counts equal the oracle's is never diagnosed (its replay
IS the oracle).  Neither the fp64 twin nor the contracted reading diagnoses
anything any more; their disagreement counts are reported only.  (Round 2's
rule -- "the step counts differ, or a reading disagrees there" -- would have
labelled a kernel bug that changed a step count and the colour a flip.)

The STRICT policy passes when
  * at least `min_frac` (99.99 %) of pixels are within `tol` -- on frames
    under 10^4 pixels, at most one pixel may be outside --
  * every outlier is replay-diagnosed, and
  * no pixel's error exceeds `max_err` (0.05).
Exact precision runs the oracle's fp32 operation sequence and is held to it
on every frame.

Some frames are fp32-ILL-CONDITIONED: the oracle's own alternative readings
of the shader (the fp64 twin; the contracted fp32 reading that GLSL 4.60
4.7.1 permits, oracle/Makefile) fail the strict policy against the fp32
oracle under the same replay diagnosis (measured at 3840x2160: C4 grazing
rays whose march ends a step apart are off by up to 0.7; the Mandelbulb's
12-iteration map amplifies ulps without any flip).  That is decided per frame
by measurement, never by scene kind: on the frame itself, and -- because a
small frame cannot estimate rates of 1e-4 -- at the BASELINE size of the
frame's own scene and pose (tests/golden/conditioning.json, measured on the
CPU by tests/golden/make_conditioning.py; matched by a fingerprint of the
scene, camera, light, material and march parameters).  For those frames
`assert_parity_frame` holds the kernel to the readings' own spread, each
reading's count taken as the larger of its count on the frame and its
full-size rate times the frame's pixels:
  * the kernel's outlier and undiagnosed counts are each at most
    READING_FACTOR times the worst reading's, plus a 3-sigma Poisson
    allowance (outliers floored at the strict budget; no allowance where the
    readings have none), and
  * MAGNITUDE: no undiagnosed kernel pixel is further off than the worst
    undiagnosed pixel of any reading on the frame or at full size (nor than
    `tol` if the readings have none) -- pixels beyond that must be
    replay-diagnosed, and
  * the kernel's count of pixels off by more than `max_err` (diagnosed or
    not) is at most READING_FACTOR times the worst reading's plus 3 sigma.
Full-size fast frames are also held to the kernel's own last measurement
(`assert_regression`, tests/golden/fast_regression.json), so a regression
inside the readings' spread still fails.
`report()` returns the numbers the tests print and assert on.
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np

TOL = 1e-4
MIN_FRAC = 0.9999
MAX_ERR = 0.05


def quantize(rgba, fmt):
    """Reference conversion of float RGBA to a framebuffer format (sdf_abi.h
    sdf_format): 0 rgba32f, 1 rgba16f (round to nearest even), 2 rgba8
    (trunc(min(max(c,0),1) * 255 + 0.5), NaN -> 0, fp32 mul then add),
    3 rgb32f (alpha dropped)."""
    a = np.asarray(rgba, dtype=np.float32)
    if fmt == 0:
        return a
    if fmt == 3:                       # RGB32F: alpha (always 1) dropped
        return np.ascontiguousarray(a[..., :3])
    if fmt == 1:
        return a.astype(np.float16)
    q = np.fmin(np.fmax(a, np.float32(0)), np.float32(1))   # fmax/fmin drop NaN -> 0
    q = np.nan_to_num(q, nan=0.0).astype(np.float32)
    return ((q * np.float32(255)).astype(np.float32) + np.float32(0.5)).astype(np.uint8)


def pixel_err(a, b):
    """Per-pixel max over RGBA of |a - b| (NaN in both: 0; NaN in one: inf)."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    d = np.where(both_nan, 0.0, np.abs(a.astype(np.float64) - b))
    return np.where(np.isnan(d), np.inf, d).max(axis=-1)


def replay_diagnosed(frame, rgba, steps, mask, t=None, tol=TOL):
    """Pixels of `mask` whose forced-step replay -- the fp32 oracle with the
    marches stopped at `steps` -- reproduces `rgba` within `tol`."""
    mask = np.asarray(mask, dtype=bool)
    if steps is None or not mask.any():
        return np.zeros_like(mask)
    import oracle   # test infrastructure (the checker), imported only when replaying
    rp, _ = oracle.replay(frame, steps, t, mask=mask)
    return mask & (pixel_err(rgba, rp) <= tol)


def report(rgba, steps, ref_rgba, ref_steps, diagnosed=None, twin_rgba=None, alt_rgba=(),
           tol=TOL):
    """Parity numbers of `rgba` against `ref_rgba`.  `diagnosed`: bool array
    of the pixels the replay explains (None: none).  `twin_rgba` /
    `alt_rgba` (alternative readings) are counted where they disagree with
    the reference, for the record only."""
    rgba = np.asarray(rgba, dtype=np.float32)
    ref_rgba = np.asarray(ref_rgba, dtype=np.float32)
    assert rgba.shape == ref_rgba.shape, (rgba.shape, ref_rgba.shape)
    err = pixel_err(rgba, ref_rgba)
    out = err > tol
    n = err.size
    diag = out & (np.asarray(diagnosed, dtype=bool) if diagnosed is not None
                  else np.zeros_like(out))
    und = out & ~diag
    step_mm = None
    if steps is not None and ref_steps is not None:
        step_mm = int(np.any(np.asarray(steps) != np.asarray(ref_steps), axis=-1).sum())
    twin_dis = None
    if twin_rgba is not None:
        twin_dis = int((pixel_err(twin_rgba, ref_rgba) > tol).sum())
    alt_dis = None
    if len(alt_rgba):
        alt = np.zeros_like(out)
        for a in alt_rgba:
            alt |= pixel_err(a, ref_rgba) > tol
        alt_dis = int(alt.sum())
    return {
        "pixels": int(n),
        "bit_exact": int(np.sum(np.all(rgba.view(np.uint32) == ref_rgba.view(np.uint32), axis=-1))),
        "within_tol_frac": float(1.0 - out.mean()) if n else 1.0,
        "outliers": int(out.sum()),
        "replay_diagnosed": int(diag.sum()),
        "undiagnosed": int(und.sum()),
        "max_err": float(err.max()) if n else 0.0,
        "undiagnosed_max_err": float(err[und].max()) if und.any() else 0.0,
        "step_mismatch": step_mm,
        "twin_disagree": twin_dis,
        "reading_disagree": alt_dis,
        "over_max_err": int(np.sum(err > MAX_ERR)),
        "over_max_err_undiagnosed": int(np.sum(und & (err > MAX_ERR))),
    }


def compare(frame, rgba, steps, ref_rgba, ref_steps, t=None, ref_is_oracle=True, twin_rgba=None,
            alt_rgba=(), tol=TOL):
    """report() with the replay diagnosis: `rgba` (kernel frame with its
    recorded `steps`) against `ref_rgba`.  If the reference is itself a
    kernel frame (`ref_is_oracle=False`, e.g. culled vs unculled), an
    outlier is diagnosed only if BOTH sides are reproduced by the oracle at
    their own step counts."""
    out = pixel_err(rgba, ref_rgba) > tol
    diag = replay_diagnosed(frame, rgba, steps, out, t, tol)
    if not ref_is_oracle:
        diag &= replay_diagnosed(frame, ref_rgba, ref_steps, out, t, tol)
    return report(rgba, steps, ref_rgba, ref_steps, diag, twin_rgba, alt_rgba, tol)


def outlier_budget(pixels, min_frac=MIN_FRAC):
    """>= min_frac of pixels within tol; on small frames that is an outlier
    budget of ceil((1 - min_frac) * pixels), at least one pixel."""
    return max(1, int(np.ceil((1.0 - min_frac) * pixels - 1e-9)))


def passes_strict(rep) -> bool:
    return (rep["outliers"] <= outlier_budget(rep["pixels"]) and rep["undiagnosed"] == 0
            and rep["max_err"] <= MAX_ERR)


def assert_parity(rep, what=""):
    """The strict policy of SURVEY.md 8(c), outliers replay-diagnosed."""
    assert rep["outliers"] <= outlier_budget(rep["pixels"]), (what, rep)
    assert rep["undiagnosed"] == 0, (what, rep)
    assert rep["max_err"] <= MAX_ERR, (what, rep)


READING_FACTOR = 2.0
CONDITIONING = Path(__file__).resolve().parent / "golden" / "conditioning.json"


def frame_fingerprint(frame) -> str:
    """SHA-256 (16 hex) of what a frame's conditioning depends on: scene,
    camera, light, material and the march parameters -- not its size,
    precision, dispatch or output format."""
    import ctypes as C
    p = type(frame.params)()
    C.memmove(C.addressof(p), C.addressof(frame.params), C.sizeof(p))
    p.width = p.height = p.precision = p.dispatch = p.output_format = 0
    h = hashlib.sha256()
    for s in (frame.scene, frame.camera, frame.light, frame.material, p):
        h.update(C.string_at(C.addressof(s), C.sizeof(s)))
    return h.hexdigest()[:16]


def full_size_conditioning(frame):
    """The full-size reading measurement of `frame`'s own scene and pose
    (tests/golden/conditioning.json), or None when the frame is not an
    unmodified configuration preset."""
    if not CONDITIONING.exists():
        return None
    key = f"{frame.name}_p{frame.meta.get('pose', 0)}"
    rec = json.loads(CONDITIONING.read_text()).get(key)
    if rec is None or rec.get("fingerprint") != frame_fingerprint(frame):
        return None
    return rec


def reading_spread(frame, ref, ref_steps, readings, t=None):
    """Each alternative reading against the fp32 oracle under the same
    replay diagnosis (the fp32 oracle stopped at the reading's own step
    counts): {name: report}.  `readings` maps name -> (rgba, steps)."""
    return {name: compare(frame, rgba, st, ref, ref_steps, t)
            for name, (rgba, st) in readings.items()}


def _allowance(worst):
    """READING_FACTOR x the worst reading's count + 3 sigma (Poisson); none
    where the readings have none."""
    return READING_FACTOR * worst + 3.0 * np.sqrt(READING_FACTOR * worst)


def assert_parity_frame(rep, spread, what="", full_size=None):
    """Strict policy when every alternative reading passes it against the
    oracle on this frame and (if `full_size`, the frame's
    full_size_conditioning record, is given) at the BASELINE size.
    Otherwise the frame is fp32-ill-conditioned and the kernel is held to the
    readings' spread (module docstring).  Returns "strict" or "readings"."""
    if all(passes_strict(r) for r in spread.values()) and (
            full_size is None or full_size["strict_at_full_size"]):
        assert_parity(rep, what)
        return "strict"
    px = rep["pixels"]
    worst = {}
    for k, rate in (("outliers", "outlier_rate"), ("undiagnosed", "undiagnosed_rate")):
        worst[k] = max(r[k] for r in spread.values())
        if full_size is not None:
            worst[k] = max(worst[k], max(full_size[n][rate] * px for n in ("twin", "fma")))
    # pixels off by more than MAX_ERR, diagnosed or not (round 4: the
    # magnitude clause alone let any number of replay-diagnosed pixels be off
    # by any amount)
    worst["over_max_err"] = max(r["over_max_err"] for r in spread.values())
    if full_size is not None:
        fpx = full_size.get("width", 0) * full_size.get("height", 0)
        if fpx:
            worst["over_max_err"] = max(worst["over_max_err"], max(
                full_size[n].get("over_max_err", 0) / fpx * px for n in ("twin", "fma")))
    bound = max(TOL, max(r["undiagnosed_max_err"] for r in spread.values()))
    if full_size is not None:
        bound = max(bound, max(full_size[n]["undiagnosed_max_err"] for n in ("twin", "fma")))
    rep["readings_bound"] = {"outliers": max(outlier_budget(px), _allowance(worst["outliers"])),
                             "undiagnosed": _allowance(worst["undiagnosed"]),
                             "over_max_err": _allowance(worst["over_max_err"]),
                             "undiagnosed_max_err": bound}
    assert rep["outliers"] <= rep["readings_bound"]["outliers"], (what, "outliers", rep, spread)
    assert rep["undiagnosed"] <= rep["readings_bound"]["undiagnosed"], \
        (what, "undiagnosed", rep, spread)
    assert rep["over_max_err"] <= rep["readings_bound"]["over_max_err"], \
        (what, "over max_err", rep, spread)
    assert rep["undiagnosed_max_err"] <= bound, (what, "magnitude", rep, spread)
    return "readings"


# Regression bounds of the fast kernel at the BASELINE sizes (round 4, VERDICT
# r03 "What's weak" 1): the readings' spread is a bound any valid fp32 reading
# meets, so a regression that doubled the kernel's own error would still pass
# it.  Each full-size fast frame is therefore also held to the kernel's last
# measured numbers (tests/golden/fast_regression.json, from the committed
# full-size survey), with a 15 % + 3-sigma count allowance and a 10 %
# magnitude allowance (C5: undiagnosed pixels at most 0.341 off, against the
# readings' 0.482).
FAST_REGRESSION = Path(__file__).resolve().parent / "golden" / "fast_regression.json"


def regression_bound(key):
    """{outliers, undiagnosed, over_max_err, undiagnosed_max_err, max_err}
    bounds of the full-size fast frame `key` (e.g. "C5_p0"), or None."""
    if not FAST_REGRESSION.exists():
        return None
    rec = json.loads(FAST_REGRESSION.read_text()).get(key)
    if rec is None:
        return None
    cnt = lambda n: 1.15 * n + 3.0 * np.sqrt(n)   # noqa: E731
    return {"outliers": max(cnt(rec["outliers"]), 1), "undiagnosed": cnt(rec["undiagnosed"]),
            "over_max_err": cnt(rec["over_max_err"]),
            "undiagnosed_max_err": max(TOL, 1.10 * rec["undiagnosed_max_err"]),
            # (a replay-diagnosed flip may move to another pixel: the largest
            # error is bounded only where it already exceeds MAX_ERR)
            "max_err": max(MAX_ERR, 1.10 * rec["max_err"]), "measured": rec}


def assert_regression(rep, key, what=""):
    """The full-size fast frame `key` within its regression bounds (if any)."""
    b = regression_bound(key)
    if b is None:
        return None
    rep["regression_bound"] = {k: v for k, v in b.items() if k != "measured"}
    for k in ("outliers", "undiagnosed", "over_max_err", "undiagnosed_max_err", "max_err"):
        assert rep[k] <= b[k], (what, "regression", k, rep[k], b)
    return b
