#!/usr/bin/env python3
"""In-process A/B timing of render-kernel builds (libsdf3d.so variants).

Each library is loaded side by side (tools/build_variant.sh builds one from a
git revision); the C4 frame (or --config) is rendered by each in turn,
rounds interleaved so clock drift hits all alike, and the median per-launch
kernel time (HIP events around 5 serialised launches) is printed per
library, with a bit-exactness check of each against the first.

    python tools/ab_kernel.py base=tools/_variants/libsdf3d_base.so new=sdf3d_amd/lib/libsdf3d.so
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
    ap.add_argument("libs", nargs="+", help="name=path")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--precision", default="fast")
    ap.add_argument("--format", default="rgba32f")
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--poses", default="0")
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, scenes
    rds = {}
    for spec in a.libs:
        name, path = spec.split("=", 1)
        rd = Renderer("cuda:0")
        rd.lib = abi.load_library(path, any_version=True)
        rds[name] = rd
    prec = abi.PRECISION_FAST if a.precision == "fast" else abi.PRECISION_EXACT
    res = {}
    for pose in [int(p) for p in a.poses.split(",")]:
        f = scenes.config(a.config, precision=prec, pose=pose)
        f.params.output_format = abi.FORMAT_NAMES[a.format]
        bufs = {n: rd.alloc(f)[0] for n, rd in rds.items()}
        first = None
        same = {}
        for n, rd in rds.items():
            rd.render(f, out=bufs[n])
            torch.cuda.synchronize()
            if first is None:
                first = bufs[n].clone()
            same[n] = bool(torch.equal(bufs[n].view(torch.uint8), first.view(torch.uint8)))
        t = {n: [] for n in rds}
        # warm the clocks
        for _ in range(100):
            for n, rd in rds.items():
                rd.render(f, out=bufs[n])
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for n, rd in rds.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                rd.render(f, out=bufs[n])
                e0.record()
                for _ in range(5):
                    rd.render(f, out=bufs[n])
                e1.record()
                torch.cuda.synchronize()
                t[n].append(e0.elapsed_time(e1) / 5)
        res[f"pose{pose}"] = {n: {"kernel_ms": round(statistics.median(v), 4),
                                  "bit_exact_vs_first": same[n]} for n, v in t.items()}
        print(json.dumps({f"{a.config} pose {pose}": res[f"pose{pose}"]}), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
