"""Diagnose exact-mode step mismatches: print the mismatching pixels with the
kernel's, the fp32 oracle's and the fp64 twin's step counts and colours."""
import sys
from pathlib import Path
sys.path[:0] = [str(Path(__file__).resolve().parent.parent), str(Path(__file__).resolve().parent.parent / "tests")]
import numpy as np, torch
import oracle
from sdf3d_amd import Renderer, scenes, abi

rd = Renderer("cuda:0")
for cfg, w, h, pose in [("REF", 800, 600, 0), ("REF", 640, 360, 2), ("C5", 320, 180, 0)]:
    f = scenes.config(cfg, w, h, precision=abi.PRECISION_EXACT, pose=pose)
    g, gs = rd.render(f, steps=True); torch.cuda.synchronize()
    g, gs = g.cpu().numpy(), gs.cpu().numpy()
    o, os_ = oracle.render(f)
    t, ts = oracle.render(f, twin=True)
    bad = np.argwhere(np.any(gs != os_, axis=-1))
    print(cfg, w, h, pose, "mismatch", len(bad))
    for y, x in bad[:8]:
        print(f"  px({x},{y}) gpu={gs[y,x]} f32={os_[y,x]} f64={ts[y,x]} "
              f"gpu_rgb={g[y,x,:3]} f32_rgb={o[y,x,:3]} f64_rgb={t[y,x,:3]}")
