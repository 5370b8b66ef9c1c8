#!/usr/bin/env python3
"""Rank 0's N-rank frame loop on one MI355X with the streams moved by real
RCCL (tools/root_rccl_probe.cpp): builds the probe, writes
the frame description (the C4 frame, `--sets` cameras: the peers' streams of
that many distinct frames, rotated so every decode reads streams the
previous frames did not), and runs it per (world, shares, batch).  One JSON
line per run, and with --out all of them.

    python tools/root_rccl_probe.py --worlds 8:2:7,4:3:4,2:1:1 --batches 1,2 --out x.json
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
SRC = ROOT / "tools" / "root_rccl_probe.cpp"
EXE = ROOT / "tools" / "root_rccl_probe.bin"


def build() -> Path:
    from sdf3d_amd import build as b
    lib = b.build_library(verbose=False)
    deps = [SRC, ROOT / "include" / "sdf_abi.h", b.CSRC / "kernel_args.h", lib]
    if not EXE.exists() or any(d.stat().st_mtime > EXE.stat().st_mtime for d in deps):
        subprocess.run([b._hipcc(), "-O2", "-std=c++17", f"--offload-arch={b.ARCH}",
                        str(SRC), "-I", str(ROOT / "include"), "-L", str(b.LIB_DIR), "-lsdf3d",
                        "-ldl", f"-Wl,-rpath,{b.LIB_DIR}", "-Wl,-rpath,$ORIGIN/../sdf3d_amd/lib",
                        "-o", str(EXE)], check=True)
    return EXE


def write_frame(path: Path, cfg: str, world: int, a: int, b: int, sets: int,
                precision: str = "fast") -> None:
    import numpy as np
    from sdf3d_amd import abi, scenes
    prec = abi.PRECISION_FAST if precision == "fast" else abi.PRECISION_EXACT
    f = scenes.config(cfg, precision=prec)
    cams = []
    for s in range(sets):
        g = scenes.config(cfg, precision=prec, pose=s % len(scenes.POSES))
        if s >= len(scenes.POSES):   # more sets than poses: small extra yaw
            m = lambda v: np.asarray(v, dtype=np.float64).reshape(4, 4, order="F")  # noqa: E731
            v = m(scenes.orbit_view(*scenes.POSES[s % len(scenes.POSES)])) @ m(
                scenes.orbit_view(3.0 * (s // len(scenes.POSES)), 0.0))
            scenes.set_view(g, v.astype(np.float32).reshape(16, order="F"))
        cams.append(bytes(g.camera))
    blob = (bytes(f.scene) + bytes(f.light) + bytes(f.material) + bytes(f.params)
            + bytes((C.c_int32 * 4)(world, a, b, sets)) + b"".join(cams))
    path.write_bytes(blob)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--precision", default="fast", choices=["fast", "exact"])
    ap.add_argument("--worlds", default="8:2:7", help="world:a:b,...")
    ap.add_argument("--batches", default="2")
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--modes", default="full",
                    help="full,norccl,rccl,decode,render (root_rccl_probe.cpp)")
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--out")
    args = ap.parse_args()
    exe = build()
    if args.build_only:
        print(exe)
        return
    from sdf3d_amd.driver import loaded_rccl_path
    import torch  # noqa: F401  (maps PyTorch's librccl for loaded_rccl_path)
    rccl = loaded_rccl_path()
    res = []
    out_dir = ROOT / "gpurun_out"
    out_dir.mkdir(exist_ok=True)
    for spec in args.worlds.split(","):
        world, a, b = (int(v) for v in spec.split(":"))
        fb = out_dir / f"rccl_probe_{world}.bin"
        write_frame(fb, args.config, world, a, b, args.sets, args.precision)
        for batch, mode in [(int(v), m) for v in args.batches.split(",")
                            for m in args.modes.split(",")]:
            r = subprocess.run([str(exe), str(fb), rccl, str(args.frames), str(args.warmup),
                                str(batch), "4", mode], capture_output=True, text=True,
                               timeout=300)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            d = json.loads(line[-1]) if line else {"error": r.stderr[-2000:]}
            d["rc"] = r.returncode
            d["config"] = args.config
            d["precision"] = args.precision
            res.append(d)
            print(json.dumps(d), flush=True)
            if r.returncode != 0:
                break
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
    sys.exit(0 if all(d["rc"] == 0 for d in res) else 1)


if __name__ == "__main__":
    main()
