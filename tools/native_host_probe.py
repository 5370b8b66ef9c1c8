#!/usr/bin/env python3
"""Host cost per frame of the native frame driver's N > 1 path (sdf_driver_*,
csrc/driver.cpp) over REAL RCCL, on one MI355X: a one-rank RCCL world with
SDF_DRIVER_ROOT_AS_PEER, so every frame takes the multi-rank route (TILES
render + compaction, RCCL length all-gather, RCCL send/recv group to rank 0
= itself, decode).  For each ship batch (frames per all-gather and per
send/recv group) it reports the driver's own host microseconds per frame
(waits excluded) and their split by call, on the 4K C4 frame and on a
host-bound frame (64x64, one march step, no shadow/AO: GPU time ~0).

At N ranks rank 0's group holds N - 1 receives per frame instead of one
here; `recv_us` (the group's cost per extra receive, measured by issuing
the one-rank group's receive several times: --extra-recvs) extrapolates it.

    torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/native_host_probe.py
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
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--batches", default="1,2,4")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from sdf3d_amd import abi, scenes
    from sdf3d_amd.driver import NativeFrameDriver
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out = {"method": __doc__.split("\n\n")[0].replace("\n", " ")}
    frames = {"C4_4k": scenes.config("C4", precision=abi.PRECISION_FAST)}
    tiny = scenes.config("C2", 64, 64, precision=abi.PRECISION_FAST)
    tiny.params.max_steps = 1
    tiny.params.flags = 0
    frames["host_bound_64x64"] = tiny
    for name, f in frames.items():
        for b in [int(x) for x in args.batches.split(",")]:
            nbuf = max(4, 2 * b)
            drv = NativeFrameDriver(f, 0, 1, dev, nbuf=nbuf, lag=min(2, nbuf - b), dist=dist,
                                    root_as_peer=True, batch=b)
            for _ in range(3 * nbuf):
                drv.step()
            drv.drain()
            torch.cuda.synchronize()
            s0 = drv.stats()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                drv.step()
            drv.drain()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            s1 = drv.stats()
            n = s1["frames"] - s0["frames"]
            host = (s1["call_s"] - s1["wait_s"]) - (s0["call_s"] - s0["wait_s"])
            out[f"{name}_batch{b}"] = {
                "nbuf": nbuf, "frames": n, "ms_per_frame": round(el / n * 1e3, 4),
                "host_us_per_frame": round(host / n * 1e6, 2),
                "enqueue_us_per_frame_cumulative": s1["enqueue_us_per_frame"]}
            print(json.dumps({f"{name}_batch{b}": out[f"{name}_batch{b}"]}), flush=True)
            drv.close()
    print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
