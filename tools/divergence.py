#!/usr/bin/env python3
"""Lane utilisation of the two marches, from the per-pixel step counts.

A wave (one 8x8 tile) runs each march loop until its slowest lane is done, so
its cost follows the per-wave MAXIMUM step count while the useful work is the
MEAN.  This prints, per march (primary / shadow):

- ``lane_util``: sum of per-wave means / sum of per-wave maxima;
- ``wave_iters``: wave-level loop iterations per wave as launched;
- ``compact_iters``: the same if the workgroup's (4 waves, 256 lanes) live
  lanes were repacked into ceil(live / 64) waves before every iteration --
  the upper bound of what lane compaction could save.

The step counts come from sdf_render's `steps` output (every lane marches
the shadow ray when counts are requested; without them lanes with
dot(N, L) <= 0 skip it, so the shadow figures are an upper bound).

    python tools/divergence.py [--config C4] [--pose 0]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def analyse(s: np.ndarray) -> dict:
    """s: [H, W] step counts, H and W multiples of 8 (W of 32)."""
    H, W = s.shape
    tiles = s.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(H // 8, W // 8, 64)
    mx = tiles.max(axis=2)
    mean = tiles.mean(axis=2)
    groups = tiles.reshape(H // 8, W // 32, 256)
    gmax = groups.max(axis=2)
    compact = 0
    for k in range(1, int(gmax.max()) + 1):
        live = (groups >= k).sum(axis=2)
        compact += int(np.ceil(live / 64.0).sum())
    waves = mx.size
    return {
        "mean_steps": round(float(s.mean()), 3),
        "lane_util": round(float(mean.sum() / max(mx.sum(), 1)), 4),
        "wave_iters": round(float(mx.sum() / waves), 3),
        "compact_iters": round(compact / waves, 3),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--pose", type=int, default=0)
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    f = scenes.config(args.config, precision=abi.PRECISION_FAST, pose=args.pose)
    _, st = rd.render(f, steps=True)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    H, W = s.shape[:2]
    H8, W32 = H // 8 * 8, W // 32 * 32
    out = {"config": args.config, "pose": args.pose}
    for i, name in enumerate(["primary", "shadow"]):
        out[name] = analyse(s[:H8, :W32, i])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
