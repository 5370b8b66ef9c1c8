"""Measure how fp32-ill-conditioned each BASELINE configuration is, at its
full size, and freeze the result in tests/golden/conditioning.json.

For every config (C2, C3, C4, C5) and camera pose (0-3) this renders the frame
with the fp32 oracle and with its two alternative readings -- the fp64 twin
and the contracted fp32 reading (oracle/Makefile liboracle_fma.so) -- and
diagnoses every reading outlier by the forced-step replay (tests/parity.py:
the fp32 oracle stopped at the reading's own step counts).  The per-pixel
RATES of outliers and undiagnosed outliers, the largest undiagnosed error, and
whether each reading passes the strict policy at full size are written per
(config, pose).

Small test frames cannot estimate these rates (a 96x54 Mandelbulb frame
expects ~0.8 twin outliers at the 4K rate, so its readings pass the strict
policy by chance about half the time).  tests/parity.py uses the full-size
measurement of the frame's own scene and pose: the rates scale the readings'
counts to the frame's size, and a scene whose readings fail the strict policy
at full size is never held to it on a small frame.  CPU only (test
infrastructure; no GPU and no reference code involved):

    python tests/golden/make_conditioning.py [--threads N]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(HERE.parent))

import oracle  # noqa: E402  (test infrastructure)
from parity import compare, frame_fingerprint, passes_strict  # noqa: E402
from sdf3d_amd import scenes  # noqa: E402

OUT = HERE / "conditioning.json"
CONFIGS = ("C2", "C3", "C4", "C5")
POSES = (0, 1, 2, 3)


def measure(cfg: str, pose: int, nthreads: int | None = None) -> dict:
    f = scenes.config(cfg, pose=pose)
    ref, rst = oracle.render(f, nthreads=nthreads)
    out = {"width": f.params.width, "height": f.params.height,
           "fingerprint": frame_fingerprint(f)}
    for name, kw in (("twin", {"twin": True}), ("fma", {"variant": "fma"})):
        rgba, st = oracle.render(f, nthreads=nthreads, **kw)
        rep = compare(f, rgba, st, ref, rst)
        px = rep["pixels"]
        out[name] = {"outliers": rep["outliers"], "undiagnosed": rep["undiagnosed"],
                     "outlier_rate": rep["outliers"] / px,
                     "undiagnosed_rate": rep["undiagnosed"] / px,
                     "undiagnosed_max_err": rep["undiagnosed_max_err"],
                     "max_err": rep["max_err"], "over_max_err": rep["over_max_err"],
                     "strict": passes_strict(rep)}
    out["strict_at_full_size"] = out["twin"]["strict"] and out["fma"]["strict"]
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=None)
    a = ap.parse_args()
    res = {}
    for cfg in CONFIGS:
        for pose in POSES:
            t0 = time.perf_counter()
            res[f"{cfg}_p{pose}"] = measure(cfg, pose, a.threads)
            r = res[f"{cfg}_p{pose}"]
            print(f"{cfg}_p{pose} strict={r['strict_at_full_size']} "
                  f"twin {r['twin']['outliers']}/{r['twin']['undiagnosed']} "
                  f"fma {r['fma']['outliers']}/{r['fma']['undiagnosed']} "
                  f"({time.perf_counter() - t0:.1f} s)", flush=True)
    res["_generator"] = ("tests/golden/make_conditioning.py: fp64 twin and contracted fp32 "
                         "reading vs the fp32 oracle at full size, outliers diagnosed by the "
                         "forced-step replay (tests/parity.py)")
    OUT.write_text(json.dumps(res, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
