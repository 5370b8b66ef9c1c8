#!/usr/bin/env python3
"""Rank 0's per-frame GPU work in an N-rank TILES frame, on one MI355X.

At N ranks the root renders its own rows straight into the frame
(SDF_TILING_FRAME_ROWS) on alternating streams and decodes the N - 1 peer
streams into the same frame (the frame driver: on the frame's own render
stream, root_serial below); a peer renders its share as TILES.  Without N GPUs the peers' streams are rendered once up front and the
root's loop is timed alone (the RCCL transfer itself is not included), so the
frame period at N is bounded below by max(root, peer):

    root_render    the root's rows only, frames on 3 streams
    decode         the N - 1 decodes only, back to back on one stream
    root_both      both, decode on the side stream as the frame driver does
    root_serial    both on one stream (no overlap)
    peer_tiles     one peer's share as TILES, frames on 3 streams
    peer_plain     the same share as plain RGBA32F (the TILES wire's cost is
                   peer_tiles - peer_plain)

    python tools/root_probe.py [--world 8] [--shares 1:3] [--config C4] [--frames 200]
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
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--precision", default="fast", choices=["fast", "exact"])
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--shares", default="1:1", help="rank 0 : other ranks, blocks per period")
    ap.add_argument("--streams", type=int, default=3, help="alternating streams / buffers")
    ap.add_argument("--lib", default=None, help="another libsdf3d.so build (A/B)")
    ap.add_argument("--skip-root-part", action="store_true",
                    help="decode only the peers' parts (rank 0's empty part not launched)")
    ap.add_argument("--only", choices=["decode", "root", "peer", "peer_plain"], default=None,
                    help="time one leg only (for rocprofv3 counter passes)")
    args = ap.parse_args()
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    if args.lib:
        rd.lib = abi.load_library(args.lib, any_version=True)
    N, K = args.world, args.frames
    f = scenes.config(args.config, precision=abi.PRECISION_FAST if args.precision == "fast"
                      else abi.PRECISION_EXACT)
    W, H = f.params.width, f.params.height
    ft = f.copy()
    ft.params.output_format = abi.FORMAT_TILES
    shares = tuple(int(v) for v in args.shares.split(":"))
    tilings = [R.tiling(r, N, 8, shares=shares) for r in range(N)]
    stride = max(R.tiles_bytes(W, R.owned_rows(H, t)) for t in tilings)
    parts = torch.zeros(N * stride, dtype=torch.uint8, device=rd.device)
    for r in range(1, N):
        rd.render(ft, tilings[r], out=parts[r * stride:(r + 1) * stride])
    NS = args.streams
    frames = [torch.empty((H, W, 4), dtype=torch.float32, device=rd.device) for _ in range(NS)]
    streams = [torch.cuda.Stream() for _ in range(NS)]
    side = torch.cuda.Stream()
    t0_tiling = R.tiling(0, N, 8, frame_rows=True, shares=shares)
    # the busiest peer: the most rows
    busiest = max(range(1, N), key=lambda r: R.owned_rows(H, tilings[r])) if N > 1 else 0
    peer_bufs = [torch.empty(stride, dtype=torch.uint8, device=rd.device) for _ in range(NS)]
    prow = R.owned_rows(H, tilings[busiest])
    peer_plain = [torch.empty((prow, W, 4), dtype=torch.float32, device=rd.device) for _ in range(NS)]

    # the parts the decode is given: all N (rank 0's empty: its header says
    # ntiles = 0) or, with --skip-root-part, the N - 1 peers' only
    first = 1 if args.skip_root_part else 0
    dparts, dN, dtilings = parts[first * stride:], N - first, tilings[first:]

    def run(render=True, decode=True, serial=False, peer=False, plain=False):
        pf = f if plain else ft
        for b in range(NS):
            if peer:
                rd.render(pf, tilings[busiest], out=peer_plain[b] if plain else peer_bufs[b],
                          stream=streams[b])
            if render:
                rd.render(f, t0_tiling, out=frames[b], stream=streams[b])
            if decode:
                rd.tiles_decode(dparts, dN, stride, W, H, 8, tilings=dtilings, out=frames[b],
                                stream=streams[b] if serial else side)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            b = i % NS
            s = streams[b]
            if peer:
                rd.render(pf, tilings[busiest], out=peer_plain[b] if plain else peer_bufs[b],
                          stream=s)
                continue
            if render:
                rd.render(f, t0_tiling, out=frames[b], stream=s)
            if decode:
                rd.tiles_decode(dparts, dN, stride, W, H, 8, tilings=dtilings, out=frames[b],
                                stream=s if serial else side)
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / K * 1e3, 4)

    def fill():
        for i in range(K):
            frames[i % NS].fill_(1.0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            frames[i % NS].fill_(1.0)
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / K * 1e3, 4)

    out = {"config": args.config, "precision": args.precision, "world": N, "shares": args.shares, "frames": K, "streams": NS}
    if args.only:
        leg = {"decode": dict(render=False), "root": dict(), "peer": dict(render=False,
               decode=False, peer=True),
               "peer_plain": dict(render=False, decode=False, peer=True, plain=True)}[args.only]
        for _ in range(2):   # the second pass (warm clocks) is the reported one
            out[args.only + "_ms"] = run(**leg)
        print(json.dumps(out))
        return
    out["frame_fill_ms"] = fill()   # the write floor of one RGBA32F frame
    for _ in range(2):   # second pass is the reported one
        out["root_render_ms"] = run(decode=False)
        out["decode_ms"] = run(render=False)
        out["root_both_ms"] = run()
        out["root_serial_ms"] = run(serial=True)
        out["peer_tiles_ms"] = run(render=False, decode=False, peer=True)
        out["peer_plain_ms"] = run(render=False, decode=False, peer=True, plain=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
