#!/usr/bin/env python3
"""Render preview images of each configuration (RGBA8) and the C4 step-count
heat maps into gpurun_out/snapshots/ (PNG, row 0 at the bottom flipped up)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np
import torch
from PIL import Image

from sdf3d_amd import Renderer, abi, scenes

out = ROOT / "gpurun_out" / "snapshots"
out.mkdir(parents=True, exist_ok=True)
rd = Renderer("cuda:0")
for cfg in ["REF", "C1", "C2", "C3", "C5"]:
    w, h = (960, 540) if cfg != "C1" else (512, 512)
    f = scenes.config(cfg, w, h, precision=abi.PRECISION_FAST, pose=1 if cfg == "C3" else 0)
    f.params.output_format = abi.FORMAT_RGBA8
    img, st = rd.render(f, steps=True)
    torch.cuda.synchronize()
    Image.fromarray(img.cpu().numpy()[::-1, :, :3]).save(out / f"{cfg}.png")
    if cfg in ("C3", "C5"):
        for which, name in [(0, "primary"), (1, "shadow")]:
            hm = rd.heatmap(st, which, f.params.max_steps)
            torch.cuda.synchronize()
            Image.fromarray(hm.cpu().numpy()[::-1, :, :3]).save(out / f"{cfg}_steps_{name}.png")
print("ok", sorted(p.name for p in out.iterdir()))
