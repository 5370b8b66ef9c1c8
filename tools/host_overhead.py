#!/usr/bin/env python3
"""Host (CPU) time of the per-frame calls the frame driver makes: one
Renderer.render enqueue, one tiles_decode enqueue, a torch event record and
an empty-ish torch op, measured without waiting for the GPU (small frames,
so the queue never backs up).

    python tools/host_overhead.py
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def per_call(fn, n=2000):
    import torch
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    el = time.perf_counter() - t0
    torch.cuda.synchronize()
    return round(el / n * 1e6, 2)


def main():
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    f = scenes.config("C1", 64, 64, precision=abi.PRECISION_FAST)
    buf, _ = rd.render(f)
    s = torch.cuda.Stream()
    ft = f.copy()
    ft.params.output_format = abi.FORMAT_TILES
    tb, _ = rd.render(ft)
    frame = torch.empty((64, 64, 4), dtype=torch.float32, device=rd.device)
    ev = torch.cuda.Event()
    x = torch.zeros(1, device=rd.device)
    out = {
        "render_us": per_call(lambda: rd.render(f, out=buf, stream=s)),
        "render_tiles_us": per_call(lambda: rd.render(ft, out=tb, stream=s)),
        "tiles_decode_us": per_call(lambda: rd.tiles_decode(tb, 1, tb.numel(), 64, 64, 8,
                                                            out=frame, stream=s)),
        "event_record_us": per_call(lambda: ev.record(s)),
        "torch_add_us": per_call(lambda: x.add_(1)),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
