#!/usr/bin/env python3
"""A/B of the render schedule (sdf_render_scheduled: row blocks dispatched
costliest first, learnt from the kernels' cycle counters) against launch
order, per configuration and precision: median kernel time of 5 serialised
launches (HIP events), rounds interleaved, bit-exactness checked.

    python tools/ab_schedule.py --configs C2,C3,C4,C5 --precisions fast,exact --out x.json
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
    ap.add_argument("--configs", default="C2,C3,C4,C5")
    ap.add_argument("--precisions", default="fast,exact")
    ap.add_argument("--poses", default="0")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    res = {}
    for cfg in a.configs.split(","):
        for prec_name in a.precisions.split(","):
            prec = abi.PRECISION_FAST if prec_name == "fast" else abi.PRECISION_EXACT
            for pose in [int(p) for p in a.poses.split(",")]:
                f = scenes.config(cfg, precision=prec, pose=pose)
                base, _ = rd.render(f)
                out = torch.empty_like(base)
                sch = rd.schedule(f.params.height, period=64)   # learnt from launch 0, then no copies
                for _ in range(4):   # the order is learnt from the first launches
                    rd.render(f, out=out, schedule=sch)
                    torch.cuda.synchronize()
                same = bool(torch.equal(out.view(torch.uint8), base.view(torch.uint8)))
                for _ in range(60):
                    rd.render(f, out=out)
                torch.cuda.synchronize()
                # and a schedule that measures every launch (its clock reads and
                # atomics on every wave: the measurement's own cost)
                sch1 = rd.schedule(f.params.height, period=1)
                for _ in range(4):
                    rd.render(f, out=out, schedule=sch1)
                    torch.cuda.synchronize()
                arms = {"launch_order": None, "scheduled": sch, "measured_every_launch": sch1}
                t = {k: [] for k in arms}
                for _ in range(a.rounds):
                    for k in t:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(5):
                            rd.render(f, out=out, schedule=arms[k])
                        e1.record()
                        torch.cuda.synchronize()
                        t[k].append(e0.elapsed_time(e1) / 5)
                r = {k: round(statistics.median(v), 4) for k, v in t.items()}
                r["gain"] = round(r["launch_order"] / r["scheduled"] - 1, 4)
                r["measure_cost"] = round(r["measured_every_launch"] / r["scheduled"] - 1, 4)
                r["bit_exact"] = same
                r["order_head"] = sch.order()[:12]
                key = f"{cfg}/{prec_name}/pose{pose}"
                res[key] = r
                print(json.dumps({key: r}), flush=True)
                sch.close()
                sch1.close()
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
