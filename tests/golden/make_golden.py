"""Generate the golden fixtures in tests/golden/ from the CPU oracle.

The reference (GLSL, ezorzin/SDF3D voxel_fragment.frag) cannot run here and
ships no tests or images, so these fixtures are renders of the oracle
restatement (oracle/oracle_core.h), frozen with SHA-256 in MANIFEST.json.
They pin the oracle against regressions (CPU test) and are the parity target
for the HIP kernel on the GPU box (GPU test).

    python tests/golden/make_golden.py          # (re)write fixtures + manifest
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402  (test infrastructure)
from sdf3d_amd import scenes  # noqa: E402

# name: (config, width, height, pose)
FIXTURES = {
    "ref_64x36_p0": ("REF", 64, 36, 0),
    "ref_64x36_p1": ("REF", 64, 36, 1),
    "ref_64x36_p2": ("REF", 64, 36, 2),
    "ref_64x36_p3": ("REF", 64, 36, 3),
    "ref_160x90_p0": ("REF", 160, 90, 0),
    "ref_37x23_p1": ("REF", 37, 23, 1),
    "c1_64x64_p0": ("C1", 64, 64, 0),
    "c2_160x90_p0": ("C2", 160, 90, 0),
    "c2_128x72_p2": ("C2", 128, 72, 2),
    "c3_160x90_p0": ("C3", 160, 90, 0),
    "c3_128x72_p1": ("C3", 128, 72, 1),
    "c5_96x54_p0": ("C5", 96, 54, 0),
}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def frame_for(name: str):
    cfg, w, h, pose = FIXTURES[name]
    return scenes.config(cfg, w, h, pose=pose)


def main() -> None:
    manifest = {}
    for name, (cfg, w, h, pose) in FIXTURES.items():
        f = frame_for(name)
        rgba, steps = oracle.render(f, nthreads=1)
        np.savez_compressed(HERE / f"{name}.npz", rgba=rgba, steps=steps)
        manifest[name] = {
            "config": cfg, "width": w, "height": h, "pose": pose,
            "sha256_rgba": sha(rgba), "sha256_steps": sha(steps),
            "mean_primary_steps": float(steps[..., 0].mean()),
            "mean_shadow_steps": float(steps[..., 1].mean()),
        }
        print(name, manifest[name]["sha256_rgba"][:16])
    manifest["_generator"] = "tests/golden/make_golden.py (CPU oracle, oracle/oracle_core.h)"
    (HERE / "MANIFEST.json").write_text(json.dumps(manifest, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
