#!/usr/bin/env python3
"""Persistent frame-sequence kernel (sdf_render_frames) against per-frame
launches, on one GPU: ms per frame of K frames of one config, median of
interleaved rounds, each frame into its own buffer (16 buffers).

  launches/1 stream   K sdf_render calls serialised on one stream
  launches/3 streams  K sdf_render calls alternating over 3 streams
  frames              sdf_render_frames(K cameras): K/16 persistent launches
  frames_static       (--sweep) the static schedule (no work queues)
  frames_qQ_cC        (--sweep) Q work queues, C tiles per request

Also checks the sequence's frames bit-exact against sdf_render.
    python tools/frames_probe.py --config C4 --frames 64 --rounds 7
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--precision", default="fast")
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--poses", default="0")
    ap.add_argument("--sweep", action="store_true", help="also the static schedule and "
                    "queue / chunk settings")
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    prec = abi.PRECISION_FAST if a.precision == "fast" else abi.PRECISION_EXACT
    res = {}
    for pose in [int(p) for p in a.poses.split(",")]:
        f = scenes.config(a.config, precision=prec, pose=pose)
        nb = 16
        bufs = [rd.alloc(f)[0] for _ in range(nb)]
        cams = [f.camera] * a.frames
        outs = [bufs[i % nb] for i in range(a.frames)]
        # exactness: one sequence of nb frames against single renders
        rd.render_frames(f, cams[:nb], bufs)
        ref, _ = rd.render(f)
        torch.cuda.synchronize()
        exact = all(torch.equal(b.view(torch.int32), ref.view(torch.int32)) for b in bufs)
        streams = [torch.cuda.Stream() for _ in range(3)]

        def launches(ns):
            for i in range(a.frames):
                rd.render(f, out=outs[i], stream=streams[i % ns])

        def frames(**env):
            for k, v in env.items():
                os.environ[k] = str(v)
            rd.render_frames(f, cams, outs)
            for k in env:
                os.environ.pop(k, None)

        modes = {"launches_1stream": lambda: launches(1), "launches_3streams": lambda: launches(3),
                 "frames": frames}
        if a.sweep:
            modes["frames_static"] = lambda: frames(SDF3D_FRAMES_SCHEDULE="static")
            for q in (1, 8, 32):
                for c in (1, 2, 4, 8):
                    modes[f"frames_q{q}_c{c}"] = (
                        lambda q=q, c=c: frames(SDF3D_FRAMES_QUEUES=q, SDF3D_FRAMES_CHUNK=c))
        t = {m: [] for m in modes}
        for _ in range(2):   # warm the clocks
            for fn in modes.values():
                fn()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for m, fn in modes.items():
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for s in streams:   # the loop starts after e0 ...
                    s.wait_stream(torch.cuda.current_stream())
                fn()
                for s in streams:   # ... and is done when every stream is
                    torch.cuda.current_stream().wait_stream(s)
                e1.record()
                torch.cuda.synchronize()
                t[m].append(e0.elapsed_time(e1) / a.frames)
        r = {m: round(statistics.median(v), 4) for m, v in t.items()}
        r["bit_exact_vs_sdf_render"] = exact
        r["fps_frames"] = round(1000.0 / r["frames"], 1)
        res[f"{a.config}_pose{pose}"] = r
        print(json.dumps({f"{a.config} pose {pose}": r}), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
