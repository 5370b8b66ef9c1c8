#!/usr/bin/env python3
"""Exact precision at full size over the four standard poses (test
infrastructure: the CPU oracle is the checker).  For each configuration and
pose, the GPU's exact frame (`sdf_render`, no steps buffer: the bench's path)
is compared bit for bit with the fp32 oracle's frame of the same inputs.  One
JSON object per (config, pose) on stdout and in --out.

    python tools/fullsize_exact_poses.py [--configs C2,C3,C4,C5] [--poses 0,1,2,3]
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
    ap.add_argument("--configs", default="C2,C3,C4,C5")
    ap.add_argument("--poses", default="0,1,2,3")
    ap.add_argument("--out", default="gpurun_out/fullsize_exact_poses.jsonl")
    a = ap.parse_args()
    import numpy as np
    import torch
    import oracle
    from sdf3d_amd import Renderer, abi, scenes
    rd = Renderer("cuda:0")
    kid = abi.load_library().sdf_kernel_id(abi.PRECISION_EXACT).decode()
    rows = []
    for cfg in a.configs.split(","):
        for pose in (int(p) for p in a.poses.split(",")):
            f = scenes.config(cfg, precision=abi.PRECISION_EXACT, pose=pose)
            gpu, _ = rd.render(f)
            torch.cuda.synchronize()
            g = gpu.cpu().numpy()
            t0 = time.time()
            ref, _ = oracle.render(f)
            cpu_s = time.time() - t0
            same = (g.view(np.uint32) == ref.view(np.uint32)).all(axis=-1)
            err = np.abs(g.astype(np.float64) - ref.astype(np.float64)).max(axis=-1)
            row = {"config": cfg, "pose": pose, "precision": "exact", "kernel_id": kid,
                   "pixels": int(same.size), "bit_exact": int(same.sum()),
                   "max_err": float(np.nan_to_num(err, nan=np.inf).max()),
                   "oracle_s": round(cpu_s, 2)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text("".join(json.dumps(r) + "\n" for r in rows))


if __name__ == "__main__":
    main()
