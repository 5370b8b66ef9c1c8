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
    # the residual widths w per tile and channel (tests/tiles_ref.py's
    # encoder steps on the SHADE32F terms): how often channel pairs fit one
    # 32-bit word of the encoder's transpose
    sys.path.insert(0, str(ROOT / "tests"))
    import tiles_ref as T
    f.params.output_format = abi.FORMAT_SHADE32F
    sh, _ = rd.render(f)
    torch.cuda.synchronize()
    terms = sh.cpu().numpy()
    rows, width = terms.shape[:2]
    n = T.tiles_shape(width, rows)[0] * T.tiles_shape(width, rows)[1]
    ws = []
    for c in range(3):
        u = T.ordered(np.ascontiguousarray(terms[..., c]).view(np.uint32))
        t = T._tiles(u, rows, width).astype(np.uint64)
        L = np.zeros_like(t); L[:, :, 1:] = t[:, :, :-1]
        U = np.zeros_like(t); U[:, 1:, :] = t[:, :-1, :]
        UL = np.zeros_like(t); UL[:, 1:, 1:] = t[:, :-1, :-1]
        r = ((t - L - U + UL) & np.uint64(0xFFFFFFFF)).astype(np.int64)
        r = np.where(r >= 2 ** 31, r - 2 ** 32, r)
        z = np.where(r >= 0, 2 * r, -2 * r - 1).astype(np.uint64).reshape(n, 64)
        z[:, 0] = 0
        ws.append(np.ceil(np.log2(z.max(axis=1).astype(np.float64) + 1)).astype(int))
    w0, w1, w2 = ws
    out["w_mean"] = [round(float(w.mean()), 2) for w in ws]
    out["w_le16"] = [round(float((w <= 16).mean()), 4) for w in ws]
    out["w0_w2_le16"] = round(float(((w0 <= 16) & (w2 <= 16)).mean()), 4)
    out["w0_plus_w2_le32"] = round(float((w0 + w2 <= 32).mean()), 4)
    out["w1_plus_w2_le32"] = round(float((w1 + w2 <= 32).mean()), 4)
    out["w_sum_le64"] = round(float((w0 + w1 + w2 <= 64).mean()), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
