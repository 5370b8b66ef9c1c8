#!/usr/bin/env python3
"""Wave-level event counts of the fast-precision render kernel, per stage.

Loads the debug library ``libsdf3d_stats.so`` (``sdf3d_amd.build.
build_stats_library``: the same sources with ``-DSDF_STATS``, see
render_kernel.inc), renders one frame and prints, per pipeline stage
(primary ray / normal+AO probes / shadow ray), the number of wave-level scene
evaluations and how each culling level resolved: cluster skipped on its
cached gap or after a fresh test, and per primitive of the cullable suffix
the cached skips, fresh tests and evaluations.  Per-wave averages guide
where the kernel's VALU issue cycles go.

    python tools/kernel_stats.py [--config C4] [--pose 0]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

STAGES = ["primary", "probes", "shadow"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--pose", type=int, default=0)
    ap.add_argument("--lib", default=None, help="a prebuilt -DSDF_STATS library (default: build "
                                               "sdf3d_amd/lib/libsdf3d_stats.so)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, build, scenes
    lib = abi.load_library(args.lib or build.build_stats_library(verbose=False))
    lib.sdf_debug_stats.restype = C.c_int
    lib.sdf_debug_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    rd = Renderer("cuda:0")
    rd.lib = lib
    f = scenes.config(args.config, precision=abi.PRECISION_FAST, pose=args.pose)
    rd.render(f)                       # warm-up (and lazy init)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 128)()
    lib.sdf_debug_stats(buf, 128, 1)   # reset
    rd.render(f)
    torch.cuda.synchronize()
    lib.sdf_debug_stats(buf, 128, 0)
    W, H = f.params.width, f.params.height
    waves = ((W + 7) // 8) * ((H + 7) // 8)
    out = {"config": args.config, "pose": args.pose, "waves": waves, "stages": {}}
    for s, name in enumerate(STAGES):
        v = [buf[s * 32 + e] / waves for e in range(32)]
        out["stages"][name] = {
            "evals_per_wave": round(v[0], 3),
            "cluster_cached_skip": round(v[1], 3),
            "cluster_fresh_test": round(v[2], 3),
            "cluster_fresh_skip": round(v[3], 3),
            "cluster_test_forgone": round(v[28], 3),
            "prim_cached_skip": [round(x, 3) for x in v[4:12]],
            "prim_fresh_test": [round(x, 3) for x in v[12:20]],
            "prim_evaluated": [round(x, 3) for x in v[20:28]],
            "prim_fresh_total": round(sum(v[12:20]), 3),
            "prim_evaluated_total": round(sum(v[20:28]), 3),
        }
    print(json.dumps(out, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
