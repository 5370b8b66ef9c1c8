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
    ap.add_argument("--precision", default="fast", choices=["fast", "exact"])
    ap.add_argument("--no-normal-lib", default=None,
                    help="a -DSDF_ABLATE_NO_NORMAL=1 build (tools/flag_variant.py): adds the "
                         "primary-march-only variant, so the frame splits into primary, normal, "
                         "AO and shadow")
    ap.add_argument("--stages-only", action="store_true")
    ap.add_argument("--out")
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    prec = abi.PRECISION_FAST if args.precision == "fast" else abi.PRECISION_EXACT
    rd_nn = None
    if args.no_normal_lib:
        rd_nn = Renderer("cuda:0")
        rd_nn.lib = abi.load_library(args.no_normal_lib, any_version=True)

    def variant(name, **kw):
        f = scenes.config(args.config, precision=prec)
        for k, v in kw.items():
            setattr(f.params, k, v)
        return name, f

    def jit_variant():
        # the CSG8 list with its first two primitives after the plane
        # swapped: no built-in variant matches, AUTO compiles one at run time
        f = scenes.config(args.config, precision=prec)
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
    if args.stages_only or args.config == "C5":
        keep = {"full", "no_ao", "no_shadow", "primary+normal", "central_normal"}
        variants = [v for v in variants if v[0] in keep]
    rds = {name: rd for name, _ in variants}
    if rd_nn is not None:
        variants.append(variant("primary_only", flags=0))
        rds["primary_only"] = rd_nn
    out = {v[0]: [] for v in variants}
    bufs = {name: rd.alloc(f)[0] for name, f in variants}
    for _ in range(2):
        for name, f in variants:
            rds[name].render(f, out=bufs[name])
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for name, f in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                rds[name].render(f, out=bufs[name])
            e1.record()
            torch.cuda.synchronize()
            out[name].append(e0.elapsed_time(e1) / args.reps)
    res = {k: round(statistics.median(v), 4) for k, v in out.items()}
    if "primary_only" in res:
        # the frame split by stage (ms of the kernel): the differences of
        # the toggled variants
        res["stages_ms"] = {
            "primary": res["primary_only"],
            "normal": round(res["primary+normal"] - res["primary_only"], 4),
            "ao": round(res["full"] - res["no_ao"], 4),
            "shadow": round(res["full"] - res["no_shadow"], 4),
            "rest (shading, store, AO-shadow overlap)": round(
                res["full"] - res["primary+normal"] - (res["full"] - res["no_ao"])
                - (res["full"] - res["no_shadow"]), 4)}
    res["config"], res["precision"] = args.config, args.precision
    if "tiles_out" not in dict(variants):
        print(json.dumps(res, indent=1))
        if args.out:
            Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
        return
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
    from sdf3d_amd import renderer as R
    res["tiles_decode"] = round(statistics.median(dec), 4)
    res["tiles_bytes_per_px"] = round(R.tiles_stream_bytes(st) / (W * H), 4)
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
