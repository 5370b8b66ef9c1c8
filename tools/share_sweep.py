#!/usr/bin/env python3
"""Kernel time of one rank's share of the frame for an N-way interleaved
tiling (N = 1, 2, 4, 8, 16): how the render kernel itself scales when each
launch holds 1/N of the waves.  Also prints the per-wave work spread from
the step counts (primary + shadow steps summed over a tile's 64 pixels'
maximum) of the whole frame.

    python tools/share_sweep.py [--config C4]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    f = scenes.config(args.config, precision=abi.PRECISION_FAST)
    out = {}
    for n in (1, 2, 4, 8, 16):
        t = R.tiling(1 % n, n, 8)
        buf, _ = rd.render(f, t)
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rd.render(f, t, out=buf)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[f"1/{n}"] = round(statistics.median(ts), 4)
    _, st = rd.render(f, steps=True)
    torch.cuda.synchronize()
    s = st.cpu().numpy()
    H, W = s.shape[:2]
    tiles = s.reshape(H // 8, 8, W // 8, 8, 2).transpose(0, 2, 1, 3, 4).reshape(-1, 64, 2)
    work = tiles[..., 0].max(axis=1) + tiles[..., 1].max(axis=1)   # wave iterations, roughly
    import numpy as np
    out["tile_work_steps"] = {"mean": float(work.mean()), "p50": float(np.percentile(work, 50)),
                              "p99": float(np.percentile(work, 99)), "max": int(work.max())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
