#!/usr/bin/env python3
"""TILES stream bytes per pixel of a frame's colours against its shading
terms (ao, dif, max(N.H, 0)), both encoded by the NumPy restatement of the
codec (tests/tiles_ref.py), on the CPU oracle's frame (tools/terms_probe.c).
MEASUREMENT TOOL: why the wire carries terms (TILES).

    python tools/terms_cost.py [--config C4] [--pose 0]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--pose", type=int, default=0)
    a = ap.parse_args()
    from sdf3d_amd import scenes
    import tiles_ref
    f = scenes.config(a.config, pose=a.pose)
    W, H = f.params.width, f.params.height
    with tempfile.TemporaryDirectory() as d:
        exe, fr, out = (os.path.join(d, n) for n in ("probe", "frame.bin", "out.bin"))
        subprocess.check_call(["gcc", "-O2", "-fopenmp", "-I", str(ROOT / "include"),
                               str(ROOT / "tools" / "terms_probe.c"), "-o", exe, "-lm"])
        with open(fr, "wb") as fh:
            for s in (f.scene, f.camera, f.light, f.material, f.params):
                fh.write(C.string_at(C.addressof(s), C.sizeof(s)))
        subprocess.check_call([exe, str(W), str(H), fr, out])
        v = np.fromfile(out, dtype=np.float32)
    res = {"config": a.config, "pose": a.pose, "width": W, "height": H}
    for name, img in (("colour", v[:W * H * 3]), ("terms", v[W * H * 3:])):
        img = img.reshape(H, W, 3)
        res[name + "_bytes_per_px"] = round(tiles_ref.stream_bytes(tiles_ref.encode(img)) / (W * H), 4)
        per = []
        for c in range(3):
            one = np.zeros_like(img)
            one[..., c] = img[..., c]
            per.append(round(tiles_ref.stream_bytes(tiles_ref.encode(one)) / (W * H), 4))
        res[name + "_per_channel"] = per
    print(json.dumps(res))


if __name__ == "__main__":
    main()
