#!/usr/bin/env python3
"""Statistics of a rendered TILES stream (the 4K C4 frame by default): bytes
per pixel, base bits per tile, and how many tiles / channels escape -- what
the decoder's per-tile paths cost (tiles.hip decode_body)."""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    args = ap.parse_args()
    import numpy as np
    import torch
    from sdf3d_amd import Renderer, abi, renderer as R, scenes
    rd = Renderer("cuda:0")
    f = scenes.config(args.config, precision=abi.PRECISION_FAST)
    f.params.output_format = abi.FORMAT_TILES
    st, _ = rd.render(f)
    torch.cuda.synchronize()
    b = st.cpu().numpy()
    used, nt = np.frombuffer(b[:8].tobytes(), dtype=np.uint32)
    head = (abi.TILES_HEADER_BYTES + 4 * int(nt) + 15) // 16 * 16
    h = np.frombuffer(b[head:head + 16 * int(nt)].tobytes(), dtype=np.uint32).reshape(-1, 4)[:, 0]
    bw = np.stack([h & 63, (h >> 6) & 63, (h >> 12) & 63], 1)
    esc = (h >> 26) & 7
    q = (h >> 18) & 255
    px = f.params.width * f.params.height
    out = {"config": args.config, "tiles": int(nt), "bytes_per_pixel": round(R.tiles_stream_bytes(st) / px, 3),
           "base_bits_mean": [round(float(x), 2) for x in bw.mean(0)],
           "B_over_64_frac": round(float((bw.sum(1) > 64).mean()), 4),
           "escaped_tile_frac": round(float((esc != 0).mean()), 4),
           "escaped_channel_frac": [round(float(((esc >> c) & 1).mean()), 4) for c in range(3)],
           "qwords_mean": round(float(q.mean()), 2), "qwords_over_64_frac": round(float((q > 64).mean()), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
