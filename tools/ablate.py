#!/usr/bin/env python3
"""In-process ablation of the render kernel's cost (one binary, one device).

Times the C4 frame with features toggled at run time (shadow, AO, normal
mode, precision, culled vs generic dispatch), interleaving the variants
round-robin so clock drift hits all of them alike (cdna_hip_programming.md
5.4 rule 24), and prints the median kernel time of each.

    python tools/ablate.py [--config C4] [--rounds 10]
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
    ap.add_argument("--config", default="C4")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")

    def variant(name, **kw):
        f = scenes.config(args.config, precision=abi.PRECISION_FAST)
        for k, v in kw.items():
            setattr(f.params, k, v)
        return name, f

    def jit_variant():
        # the CSG8 list with its first two primitives after the plane
        # swapped: no built-in variant matches, AUTO compiles one at run time
        f = scenes.config(args.config, precision=abi.PRECISION_FAST)
        f.scene.prims[1], f.scene.prims[2] = f.scene.prims[2], f.scene.prims[1]
        return "jit_reordered", f

    full = abi.FLAG_SHADOW | abi.FLAG_AO
    variants = [
        variant("full"),
        variant("no_ao", flags=abi.FLAG_SHADOW),
        variant("no_shadow", flags=abi.FLAG_AO),
        variant("primary+normal", flags=0),
        variant("central_normal", normal_mode=abi.NORMAL_CENTRAL),
        variant("exact", precision=abi.PRECISION_EXACT),
        variant("generic_culled", dispatch=abi.DISPATCH_GENERIC),
        variant("unculled", dispatch=abi.DISPATCH_UNCULLED),
        variant("max_steps_1", max_steps=1, flags=0),
        jit_variant(),
        variant("rgb32f_out", output_format=abi.FORMAT_RGB32F),
        variant("tiles_out", output_format=abi.FORMAT_TILES),
    ]
    _ = full
    out = {v[0]: [] for v in variants}
    bufs = {name: rd.alloc(f)[0] for name, f in variants}
    for _ in range(2):
        for name, f in variants:
            rd.render(f, out=bufs[name])
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for name, f in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                rd.render(f, out=bufs[name])
            e1.record()
            torch.cuda.synchronize()
            out[name].append(e0.elapsed_time(e1) / args.reps)
    # decode of the whole-frame TILES stream into RGBA32F (rank 0's side)
    ft = dict(variants)["tiles_out"]
    W, H = ft.params.width, ft.params.height
    frame = torch.empty((H, W, 4), dtype=torch.float32, device=rd.device)
    st = bufs["tiles_out"]
    dec = []
    for _ in range(args.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            rd.tiles_decode(st, 1, st.numel(), W, H, 8, out=frame)
        e1.record()
        torch.cuda.synchronize()
        dec.append(e0.elapsed_time(e1) / args.reps)
    out["tiles_decode"] = dec
    from sdf3d_amd import renderer as R
    out["tiles_bytes_per_px"] = [R.tiles_stream_bytes(st) / (W * H)]
    res = {k: round(statistics.median(v), 4) for k, v in out.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
