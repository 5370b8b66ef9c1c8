#!/usr/bin/env python3
"""Which fast-precision Mandelbulb form meets the strict parity policy, and at what cost.

Builds (here, --build) variants of libsdf3d.so whose fast translation unit
compiles the Mandelbulb with -DSDF_BULB_FORM=n (render_kernel.inc):
  0  the shipped fast form (complex squarings, factored k1/k4, FMA)
  1  the oracle's polynomial, contraction on, hardware rsq/sqrt/log
  2  the oracle's polynomial, contraction off
  3  2 + IEEE 1/sqrt for r
  4  3 + IEEE sqrt/log/division
  5  4 + IEEE division for the local coordinates
then (on the GPU box) renders C5 with each at 320x180 (poses 0-3), the golden
fixture size and 3840x2160 pose 0, reports the parity policy's numbers
against the oracle (step counts + fp64 twin diagnosis) and times the 4K
kernel (HIP events, median of interleaved rounds).

    python tools/bulb_forms.py --build            # CPU: variant libraries
    python tools/bulb_forms.py --out gpurun_out/bulb_forms.json   # GPU box
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
VDIR = ROOT / "tools" / "_variants"
FORMS = [0, 1, 2, 3, 4, 5]


def lib_path(form: int) -> Path:
    return VDIR / f"libsdf3d_bulb{form}.so"


def build():
    from sdf3d_amd import build as b
    b.build_library(verbose=False)
    VDIR.mkdir(parents=True, exist_ok=True)
    hipcc = b._hipcc()
    others = [b.OBJ / (Path(src).stem + ".o") for src, _ in b.UNITS if src != "render_fast.hip"]
    extra = dict(b.UNITS)["render_fast.hip"]
    for form in FORMS:
        o = VDIR / f"render_fast_bulb{form}.o"
        b._run([hipcc, *b.COMMON, *extra, f"-DSDF_BULB_FORM={form}", "-I", b.OBJ, "-c",
                b.CSRC / "render_fast.hip", "-o", o], True)
        b._run([hipcc, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", lib_path(form), o,
                *others, "-lhiprtc", "-ldl"], True)


def run(out_path: Path, rounds: int):
    import numpy as np
    import torch

    import oracle
    from golden.make_golden import frame_for
    from parity import assert_parity, report
    from sdf3d_amd import Renderer, abi, scenes

    cases = [("C5", 320, 180, p) for p in range(4)] + [("fixture", 96, 54, 0), ("C5", 3840, 2160, 0)]
    frames = {}
    for cfg, w, h, p in cases:
        if cfg == "fixture":
            f = frame_for("c5_96x54_p0")
        else:
            f = scenes.config(cfg, w, h, precision=abi.PRECISION_FAST, pose=p)
        f.params.precision = abi.PRECISION_FAST
        key = f"{cfg}_{w}x{h}_p{p}"
        ref, rst = oracle.render(f)
        frames[key] = (f, ref, rst, None)
        print("oracle", key, flush=True)
    rds = {}
    for form in FORMS:
        rd = Renderer("cuda:0")
        rd.lib = abi.load_library(lib_path(form))
        rds[form] = rd
    results = {}
    for form, rd in rds.items():
        res = {}
        for key, (f, ref, rst, twin) in frames.items():
            rgba, st = rd.render(f, steps=True)
            torch.cuda.synchronize()
            rgba, st = rgba.cpu().numpy(), st.cpu().numpy()
            rep = report(rgba, st, ref, rst)
            if rep["undiagnosed"]:
                if twin is None:
                    twin, _ = oracle.render(f, twin=True)
                    frames[key] = (f, ref, rst, twin)
                rep = report(rgba, st, ref, rst, twin)
            try:
                assert_parity(rep)
                rep["strict_pass"] = True
            except AssertionError:
                rep["strict_pass"] = False
            res[key] = rep
            print(form, key, json.dumps(rep), flush=True)
        results[form] = {"parity": res}
    # 4K kernel time, interleaved rounds
    f4 = frames["C5_3840x2160_p0"][0]
    times = {form: [] for form in FORMS}
    bufs = {form: rds[form].alloc(f4)[0] for form in FORMS}
    for _ in range(rounds):
        for form, rd in rds.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            for _ in range(2):
                rd.render(f4, out=bufs[form])
            ev[0].record()
            for _ in range(5):
                rd.render(f4, out=bufs[form])
            ev[1].record()
            torch.cuda.synchronize()
            times[form].append(ev[0].elapsed_time(ev[1]) / 5)
    for form in FORMS:
        results[form]["kernel_ms_4k"] = round(statistics.median(times[form]), 4)
        print(form, "kernel ms", results[form]["kernel_ms_4k"], flush=True)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    out_path.write_text(json.dumps(results, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--out", default="gpurun_out/bulb_forms.json")
    ap.add_argument("--rounds", type=int, default=10)
    a = ap.parse_args()
    if a.build:
        build()
    else:
        run(Path(a.out), a.rounds)


if __name__ == "__main__":
    main()
