#!/usr/bin/env python3
"""Cost of the TILES wire on the render side, on one MI355X: the same rows
rendered as RGBA32F and as a TILES stream (render with the encoder
epilogue + scan + move), serialised launches timed with HIP events after a
clock warm-up, for the whole frame and for the shares of N-rank frames.

    python tools/tiles_cost.py [--config C4] [--n 50]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--whole-only", action="store_true")
    ap.add_argument("--share", default=None,
                    help="WORLD:A:B -- time only rank 1's share of that tiling (e.g. 8:2:7)")
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    s = torch.cuda.current_stream()
    plain = scenes.config(args.config, precision=abi.PRECISION_FAST)
    tiles = plain.copy()
    tiles.params.output_format = abi.FORMAT_TILES
    out = {"config": args.config}

    def timed(fr, t, n):
        buf, _ = rd.alloc(fr, t)
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.3:
            for _ in range(5):
                rd.render(fr, t, out=buf, stream=s)
            torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(n):
            rd.render(fr, t, out=buf, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        return round(a.elapsed_time(b) / n, 4)

    for name, t in [("whole", None), ("half_of_2", R.tiling(1, 2, 8)),
                    ("share_3_of_7_N2", R.tiling(1, 2, 8, shares=(4, 3))),
                    ("quarter_of_4", R.tiling(1, 4, 8)),
                    ("share_2_of_15_N8", R.tiling(1, 8, 8, shares=(1, 2)))][:1 if args.whole_only else 5] \
            if not args.share else \
            [(f"share_{args.share}", R.tiling(1, int(args.share.split(":")[0]), 8,
                                              shares=tuple(int(v) for v in args.share.split(":")[1:])))]:
        p, q = timed(plain, t, args.n), timed(tiles, t, args.n)
        out[name] = {"rgba32f_ms": p, "tiles_ms": q, "overhead": round(q / p - 1, 4)}
        if t is None:
            st, _ = rd.render(tiles)
            torch.cuda.synchronize()
            W, H = plain.params.width, plain.params.height
            out[name]["stream_bytes_per_px"] = round(R.tiles_stream_bytes(st) / (W * H), 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
