#!/usr/bin/env python3
"""Exact precision on a scaled scene (test infrastructure: the CPU oracle is
the checker).  The C3/C4 CSG scene with every length -- primitive positions
and sizes, smooth-min k, light, eye, max_dist, eps, normal_eps, the AO
heights -- multiplied by S renders the same picture up to rounding; the
exact kernel must still equal the oracle bit for bit at every S (the
culling margins must hold at any coordinate magnitude in the working range).

    python tools/scale_exactness_probe.py [--scales 1,100,10000] [--size 480x270]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

# the primitive kinds' parameter slots that are lengths (sdf_abi.h): every
# slot but a plane's unit normal
PLANE = 1


def scaled(cfg: str, S: float, w: int, h: int, pose: int):
    from sdf3d_amd import abi, scenes
    f = scenes.config(cfg, w, h, precision=abi.PRECISION_EXACT, pose=pose)
    sc = f.scene
    for i in range(sc.count):
        pr = sc.prims[i]
        pr.k = pr.k * S
        if pr.kind == PLANE:
            pr.p[3] = pr.p[3] * S
        else:
            for j in range(12):
                pr.p[j] = pr.p[j] * S
    for j in range(3):
        f.camera.eye[j] = f.camera.eye[j] * S
        f.light.pos[j] = f.light.pos[j] * S
    p = f.params
    p.max_dist, p.eps, p.normal_eps = p.max_dist * S, p.eps * S, p.normal_eps * S
    p.ao_step, p.ao_base = p.ao_step * S, p.ao_base * S
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--scales", default="1,100,10000,1000000")
    ap.add_argument("--size", default="480x270")
    ap.add_argument("--poses", default="0,1")
    ap.add_argument("--out", default="gpurun_out/scale_exactness.jsonl")
    a = ap.parse_args()
    import numpy as np
    import torch
    import oracle
    from sdf3d_amd import Renderer, abi
    w, h = (int(v) for v in a.size.split("x"))
    rd = Renderer("cuda:0")
    rows = []
    for S in (float(s) for s in a.scales.split(",")):
        for pose in (int(p) for p in a.poses.split(",")):
            f = scaled(a.config, S, w, h, pose)
            rc = abi.load_library().sdf_validate(*(C_ref(x) for x in (f.scene, f.camera, f.light,
                                                                        f.material, f.params)), None)
            if rc != 0:
                row = {"scale": S, "pose": pose, "validate": rc}
            else:
                gpu, _ = rd.render(f)
                torch.cuda.synchronize()
                g = gpu.cpu().numpy()
                ref, _ = oracle.render(f)
                same = (g.view(np.uint32) == ref.view(np.uint32)).all(axis=-1)
                row = {"config": a.config, "scale": S, "pose": pose, "size": a.size,
                       "pixels": int(same.size), "bit_exact": int(same.sum())}
            rows.append(row)
            print(json.dumps(row), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in rows))


def C_ref(x):
    import ctypes as C
    return C.byref(x)


if __name__ == "__main__":
    main()
