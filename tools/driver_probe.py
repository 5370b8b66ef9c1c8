#!/usr/bin/env python3
"""Host cost of the N > 1 frame driver, measured with one rank on one MI355X.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so the
multi-rank loop cannot be rehearsed on a one-GPU box.  This runs the N > 1
code path of FrameDriver with a one-rank RCCL process group instead
(collectives_at_world1): every frame renders a peer's share of the N-rank
frame as a TILES stream, all-reduces its size, gathers it (to itself) and
decodes it into the frame -- the same calls, in the same order, as a rank
of the N-rank job makes.

    per_call      host time of each call the loop makes, queue not backed up
    loop          ms per frame of the whole driver loop, per (lag, nbuf),
                  against the GPU-only time of the same renders
    host_bound    the same loop on a 64x64 frame with one march step per
                  pixel and no shadow / AO: GPU time ~0, so this is the
                  host's own cost per frame
    native        the same measurements for the C++ driver (sdf_driver_*)

    torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/driver_probe.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8, help="the N whose peer share is rendered")
    ap.add_argument("--shares", default="1:2")
    ap.add_argument("--config", default="C4")
    ap.add_argument("--frames", type=int, default=300)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    from sdf3d_amd.multigpu import FrameDriver

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    rd = Renderer(dev)
    shares = tuple(int(v) for v in args.shares.split(":"))
    tl = R.tiling(1, args.world, 8, shares=shares)      # a peer's share
    out = {"world": args.world, "shares": args.shares, "config": args.config}

    def per_call(fn, n=500):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        el = time.perf_counter() - t0
        torch.cuda.synchronize()
        return round(el / n * 1e6, 2)

    # ---- per-call host costs (small frame: the GPU never backs up) ----------
    fs = scenes.config(args.config, 64, 64, precision=abi.PRECISION_FAST)
    fs.params.output_format = abi.FORMAT_TILES
    tb, _ = rd.render(fs)
    frame = torch.empty((64, 64, 4), dtype=torch.float32, device=dev)
    s = torch.cuda.Stream()
    i32 = tb[:4].view(torch.int32)
    pin = torch.zeros((4,), dtype=torch.int32, pin_memory=True)
    ev = torch.cuda.Event()
    glist = [torch.empty_like(tb)]
    pc = {}
    pc["render_tiles"] = per_call(lambda: rd.render(fs, out=tb, stream=s))
    pc["tiles_decode"] = per_call(lambda: rd.tiles_decode(tb, 1, tb.numel(), 64, 64, 8,
                                                          out=frame, stream=s, tilings=[R.tiling()]))

    def allreduce():
        with torch.cuda.stream(s):
            w = dist.all_reduce(i32, op=dist.ReduceOp.MAX, async_op=True)
            w.wait()
    pc["all_reduce+wait"] = per_call(allreduce)

    def gather():
        with torch.cuda.stream(s):
            w = dist.gather(tb, gather_list=glist, dst=0, async_op=True)
            w.wait()
    pc["gather+wait"] = per_call(gather)

    def item():
        with torch.cuda.stream(s):
            return int(i32.item())
    pc["item_roundtrip"] = per_call(item)

    def pinned():
        with torch.cuda.stream(s):
            pin[:1].copy_(i32, non_blocking=True)
            ev.record(s)
        ev.synchronize()
        return int(pin[0])
    pc["pinned_roundtrip"] = per_call(pinned)
    pc["stream_ctx"] = per_call(lambda: torch.cuda.stream(s).__enter__())
    out["per_call_us"] = pc

    # ---- the driver loop -----------------------------------------------------
    def loop(fr, lag, nbuf, frames):
        W, H = fr.params.width, fr.params.height
        ft = fr.copy()
        ft.params.output_format = abi.FORMAT_TILES

        def render_fn(o, stream):
            rd.render(ft, tl, out=o, stream=stream)

        def decode_fn(parts, nparts, pitch, w, h, b, o, stream, shares=None):
            rd.tiles_decode(parts, nparts, pitch, w, h, b, out=o, stream=stream, tilings=[tl])

        drv = FrameDriver(W, H, 0, 1, dev, render_fn, decode_fn, dist=dist, wire="tiles",
                          nbuf=nbuf, lag=lag, collectives_at_world1=True,
                          wire_bytes=R.tiles_bytes(W, R.owned_rows(H, tl)))
        from sdf3d_amd.multigpu import tiles_data_offset
        drv.data_off = tiles_data_offset(W, R.owned_rows(H, tl))   # the share's header
        for i in range(10):
            drv.step(i)
        drv.drain()
        t0 = time.perf_counter()
        for i in range(10, 10 + frames):
            drv.step(i)
        drv.drain()
        el = time.perf_counter() - t0
        return round(el / frames * 1e3, 4)

    def gpu_only(fr, nbuf, frames):
        ft = fr.copy()
        ft.params.output_format = abi.FORMAT_TILES
        bufs = [rd.alloc(ft, tl)[0] for _ in range(nbuf)]
        strs = [torch.cuda.Stream() for _ in range(nbuf)]
        for i in range(10):
            rd.render(ft, tl, out=bufs[i % nbuf], stream=strs[i % nbuf])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(frames):
            rd.render(ft, tl, out=bufs[i % nbuf], stream=strs[i % nbuf])
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / frames * 1e3, 4)

    f = scenes.config(args.config, precision=abi.PRECISION_FAST)
    # host-bound loops: a frame the GPU finishes in microseconds (one march
    # step per pixel, no shadow / AO), so the loop time is the host's cost
    small = scenes.config(args.config, 64, 64, precision=abi.PRECISION_FAST)
    small.params.max_steps = 1
    small.params.flags = 0
    res = {"gpu_only_render_ms": gpu_only(f, 3, args.frames)}
    for lag, nbuf in ((1, 3), (2, 3), (2, 4), (3, 4)):
        res[f"loop_ms_lag{lag}_nbuf{nbuf}"] = loop(f, lag, nbuf, args.frames)
        res[f"host_bound_ms_lag{lag}_nbuf{nbuf}"] = loop(small, lag, nbuf, args.frames)
    out["loop"] = res

    # ---- the native driver (sdf_driver_*): rank 0 ships its whole frame to
    # itself as TILES (ROOT_AS_PEER), the N > 1 sequence of calls ------------
    from sdf3d_amd.driver import NativeFrameDriver

    def native(fr, lag, nbuf, frames, peer=True):
        drv = NativeFrameDriver(fr, 0, 1, dev, nbuf=nbuf, lag=lag, dist=dist, root_as_peer=peer)
        for _ in range(10):
            drv.step()
        drv.drain()
        t0 = time.perf_counter()
        for _ in range(frames):
            drv.step()
        drv.drain()
        el = time.perf_counter() - t0
        st = drv.stats()
        drv.close()
        return {"ms_per_frame": round(el / frames * 1e3, 4),
                "host_us_per_frame": st["host_us_per_frame"],
                "enqueue_us_per_frame": st["enqueue_us_per_frame"]}

    nat = {}
    for lag, nbuf in ((1, 3), (2, 4)):
        nat[f"host_bound_ms_lag{lag}_nbuf{nbuf}"] = native(small, lag, nbuf, args.frames)
        nat[f"loop_full_frame_ms_lag{lag}_nbuf{nbuf}"] = native(f, lag, nbuf, 100)
    nat["local_full_frame_ms_nbuf3"] = native(f, 1, 3, 100, peer=False)
    nat["local_host_bound_ms_nbuf3"] = native(small, 1, 3, args.frames, peer=False)
    out["native"] = nat
    print(json.dumps(out, indent=1), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
