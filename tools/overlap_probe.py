#!/usr/bin/env python3
"""Frame period of one rank's share (1/1 and 1/8 of the 4K C4 frame) when
consecutive frames render on 1, 2 or 3 alternating streams, for the RGBA32F
and the TILES output: how much of a launch's tail (its slowest tiles) the
next frame hides, and what the TILES encoder costs per frame.

    python tools/overlap_probe.py
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    res = {}
    for fmt in (abi.FORMAT_RGBA32F, abi.FORMAT_TILES):
        f = scenes.config("C4", precision=abi.PRECISION_FAST)
        f.params.output_format = fmt
        for n in (1, 8):
            t = R.tiling(1 % n, n, 8)
            bufs = [rd.render(f, t)[0] for _ in range(3)]
            streams = [torch.cuda.Stream() for _ in range(3)]
            for ns in (1, 2, 3):
                for _ in range(2):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    K = 100
                    for i in range(K):
                        b = i % ns
                        rd.render(f, t, out=bufs[b], stream=streams[b])
                    torch.cuda.synchronize()
                    el = (time.perf_counter() - t0) / K * 1e3
                name = "tiles" if fmt == abi.FORMAT_TILES else "rgba32f"
                res[f"{name} share 1/{n}, {ns} streams ms/frame"] = round(el, 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
