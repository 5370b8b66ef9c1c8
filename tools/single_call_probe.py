#!/usr/bin/env python3
"""The single-call path: one frame in flight, launches
serialised on one stream, HIP events around each -- sdf_render (host-ordered
8-row blocks, one wave per 8x8 tile) against sdf_render_frames with ONE
camera (the persistent kernel: per-XCD work queues hand out tiles, heavy
rows first is not needed, every wave takes the next tile) and against
sdf_render_scheduled (costliest blocks first, learnt).  ms per frame, median
of rounds; the frames are checked bit-exact against sdf_render.

    python tools/single_call_probe.py --config C3 --precision exact
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--precision", default="exact")
    ap.add_argument("--calls", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lib", default=None, help="another libsdf3d.so build (A/B)")
    ap.add_argument("--only", default=None, choices=["render", "frames1", "scheduled"],
                    help="run one leg only (for rocprofv3 counter passes)")
    ap.add_argument("--period", type=int, default=16,
                    help="the schedule measures block costs every `period` launches")
    a = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    if a.lib:
        rd.lib = abi.load_library(a.lib, any_version=True)
    f = scenes.config(a.config, precision=abi.PRECISION_EXACT if a.precision == "exact"
                      else abi.PRECISION_FAST)
    out = rd.alloc(f)[0]
    out2 = rd.alloc(f)[0]
    s = torch.cuda.current_stream()

    def timed(fn):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.calls)]
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        for e0, e1 in ev:
            e0.record(s)
            fn()
            e1.record(s)
        torch.cuda.synchronize()
        return statistics.median(e0.elapsed_time(e1) for e0, e1 in ev)

    sch = rd.schedule(f.params.height, period=a.period)
    out3 = rd.alloc(f)[0]
    legs = {"render": lambda: rd.render(f, out=out, stream=s),
            "frames1": lambda: rd.render_frames(f, [f.camera], [out2], stream=s),
            "scheduled": lambda: rd.render(f, out=out3, stream=s, schedule=sch)}
    if a.only:
        legs = {a.only: legs[a.only]}
    res = {k: [] for k in legs}
    for _ in range(a.rounds):
        for k, fn in legs.items():
            res[k].append(timed(fn))
    torch.cuda.synchronize()
    if a.only:
        print(json.dumps({"config": a.config, "precision": a.precision, "only": a.only,
                          a.only + "_ms": round(statistics.median(res[a.only]), 4)}), flush=True)
        return
    same = bool(torch.equal(out.view(torch.int32), out2.view(torch.int32)))
    same3 = bool(torch.equal(out.view(torch.int32), out3.view(torch.int32)))
    print(json.dumps({"config": a.config, "precision": a.precision, "calls": a.calls,
                      "lib": a.lib or "tree",
                      **{k + "_ms": round(statistics.median(v), 4) for k, v in res.items()},
                      "frames1_bit_exact": same, "scheduled_bit_exact": same3,
                      "schedule_period": a.period}), flush=True)


if __name__ == "__main__":
    main()
