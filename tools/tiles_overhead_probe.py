#!/usr/bin/env python3
"""The TILES wire's cost on a peer's share (measurement tooling): the same
rows rendered as RGBA32F, as SHADE32F (the terms the stream carries, no
colour) and as a TILES stream (render_tiles + the compaction), frames on 3
streams; per-kernel times come from a rocprofv3 --kernel-trace --stats run
of this script.

    python tools/tiles_overhead_probe.py --config C5 --precision exact [--world 8 --shares 1:7]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--precision", default="exact")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--shares", default="1:7")
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--formats", default="rgba32f,shade32f,tiles")
    a = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    f = scenes.config(a.config, precision=abi.PRECISION_EXACT if a.precision == "exact"
                      else abi.PRECISION_FAST)
    W, H = f.params.width, f.params.height
    sh = tuple(int(v) for v in a.shares.split(":"))
    t = R.tiling(1, a.world, 8, shares=sh)
    rows = R.owned_rows(H, t)
    out = {"config": a.config, "precision": a.precision, "world": a.world, "shares": a.shares,
           "rows": rows}
    NS = a.streams
    out["streams"] = NS
    streams = [torch.cuda.Stream() for _ in range(NS)]
    fmts = {"rgba32f": abi.FORMAT_RGBA32F, "shade32f": abi.FORMAT_SHADE32F,
            "tiles": abi.FORMAT_TILES}
    for name in a.formats.split(","):
        fmt = fmts[name]
        g = f.copy()
        g.params.output_format = fmt
        bufs = [rd.alloc(g, t)[0] for _ in range(NS)]
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.frames):
                rd.render(g, t, out=bufs[i % NS], stream=streams[i % NS])
            torch.cuda.synchronize()
            out[name + "_ms"] = round((time.perf_counter() - t0) / a.frames * 1e3, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
