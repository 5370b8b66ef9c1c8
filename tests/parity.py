"""Parity policy between the HIP kernel and the CPU oracle.

A pixel's error is its largest per-channel |delta| over RGBA.  A comparison
passes when
  * at least `min_frac` (99.99 %) of pixels are within `tol` (1e-4), and
  * every pixel above `tol` is a DIAGNOSED branch flip: the kernel's primary
    or shadow iteration count differs from the oracle's, or (when the fp64
    twin is supplied) the fp64 twin disagrees with the fp32 oracle there, and
  * no pixel's error exceeds `max_err` (0.05 by default).
`report()` returns the numbers the tests print and assert on.
"""
from __future__ import annotations

import numpy as np

TOL = 1e-4
MIN_FRAC = 0.9999
MAX_ERR = 0.05


def report(rgba, steps, ref_rgba, ref_steps, twin_rgba=None, tol=TOL):
    rgba = np.asarray(rgba, dtype=np.float32)
    ref_rgba = np.asarray(ref_rgba, dtype=np.float32)
    assert rgba.shape == ref_rgba.shape, (rgba.shape, ref_rgba.shape)
    both_nan = np.isnan(rgba) & np.isnan(ref_rgba)
    d = np.where(both_nan, 0.0, np.abs(rgba.astype(np.float64) - ref_rgba))
    d = np.where(np.isnan(d), np.inf, d)
    err = d.max(axis=-1)
    out = err > tol
    n = err.size
    flip = np.zeros_like(out)
    if steps is not None and ref_steps is not None:
        flip |= np.any(np.asarray(steps) != np.asarray(ref_steps), axis=-1)
    if twin_rgba is not None:
        flip |= np.abs(np.asarray(twin_rgba, np.float64) - ref_rgba).max(axis=-1) > tol
    return {
        "pixels": int(n),
        "bit_exact": int(np.sum(np.all(rgba.view(np.uint32) == ref_rgba.view(np.uint32), axis=-1))),
        "within_tol_frac": float(1.0 - out.mean()),
        "outliers": int(out.sum()),
        "undiagnosed": int(np.sum(out & ~flip)),
        "max_err": float(err.max()) if n else 0.0,
        "step_mismatch": int(flip.sum()) if steps is not None else None,
    }


def assert_parity(rep, min_frac=MIN_FRAC, max_err=MAX_ERR, what=""):
    assert rep["within_tol_frac"] >= min_frac, (what, rep)
    assert rep["undiagnosed"] == 0, (what, rep)
    assert rep["max_err"] <= max_err, (what, rep)
