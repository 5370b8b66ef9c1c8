"""Full-resolution oracle step-count statistics for roofline accounting.

For each bench workload this renders the whole frame with the CPU oracle and
stores, per frame row, the pixel count and the sums of the primary and shadow
iteration counts (S_p, S_s).  bench.py turns these into algorithmic flops per
launch with sdf3d_amd.costmodel (step counts come from the
oracle, not from the GPU).  The GPU tests check the kernel's own counts
against these sums.

    python tests/golden/make_stats.py [CONFIG ...]     # default: C4 C3 C2
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402  (test infrastructure)
from sdf3d_amd import scenes  # noqa: E402


def stats_path(cfg: str, pose: int = 0) -> Path:
    return HERE / f"stats_{cfg}_p{pose}.npz"


def make(cfg: str, pose: int = 0) -> dict:
    f = scenes.config(cfg, pose=pose)
    t0 = time.time()
    _, steps = oracle.render(f)
    dt = time.time() - t0
    sp = steps[..., 0].astype(np.int64).sum(axis=1)
    ss = steps[..., 1].astype(np.int64).sum(axis=1)
    np.savez_compressed(stats_path(cfg, pose), row_sp=sp, row_ss=ss,
                        width=f.params.width, height=f.params.height)
    info = {"config": cfg, "pose": pose, "width": f.params.width, "height": f.params.height,
            "mean_sp": float(sp.sum() / steps[..., 0].size),
            "mean_ss": float(ss.sum() / steps[..., 0].size),
            "exhausted_frac": float((steps[..., 0] == f.params.max_steps).mean()),
            "oracle_seconds": round(dt, 2), "threads": oracle.default_threads()}
    print(json.dumps(info))
    return info


if __name__ == "__main__":
    for c in (sys.argv[1:] or ["C4", "C3", "C2"]):
        make(c)
