#!/usr/bin/env python3
"""Render C4 in the TILES format and decode it, N times each (for
rocprofv3 --kernel-trace --stats: per-kernel cost of the multi-device wire).

    python tools/tiles_prof.py [--config C4] [--world 8] [--n 20]
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--world", type=int, default=8, help="render rank 1's share of this tiling")
    ap.add_argument("--n", type=int, default=20)
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    f = scenes.config(args.config, precision=abi.PRECISION_FAST)
    f.params.output_format = abi.FORMAT_TILES
    W, H = f.params.width, f.params.height
    t = R.tiling(1 % args.world, args.world, 8)
    st, _ = rd.render(f, t)
    whole = scenes.config(args.config, precision=abi.PRECISION_FAST)
    whole.params.output_format = abi.FORMAT_TILES
    sw, _ = rd.render(whole)
    frame = torch.empty((H, W, 4), dtype=torch.float32, device=rd.device)
    plain = scenes.config(args.config, precision=abi.PRECISION_FAST)
    pb, _ = rd.render(plain, t)
    for _ in range(args.n):
        rd.render(plain, t, out=pb)      # the same share as RGBA32F (encoder cost)
    for _ in range(args.n):
        rd.render(f, t, out=st)
    for _ in range(args.n):
        rd.tiles_decode(sw, 1, sw.numel(), W, H, 8, out=frame)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
