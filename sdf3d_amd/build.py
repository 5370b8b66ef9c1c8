"""Build the HIP C-ABI library ``sdf3d_amd/lib/libsdf3d.so`` for gfx950.

Explicit ``hipcc`` invocations (no JIT, no torch extension cache) so the built
library lives in-tree and travels to the GPU box with the repository snapshot.

Translation units:
  render_exact.hip  -- render kernel, -ffp-contract=off, IEEE div/sqrt
  render_fast.hip   -- render kernel, FMA contraction, hardware sqrt/rcp
  deinterleave.hip  -- multi-device row-block scatter
  sdf_abi.cpp       -- the extern "C" entry points of include/sdf_abi.h

Run ``python -m sdf3d_amd.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB_DIR = PKG / "lib"
LIB = LIB_DIR / "libsdf3d.so"
ARCH = os.environ.get("SDF3D_ARCH", "gfx950")

COMMON = ["-O3", "-fPIC", "-std=c++17", "-Wall", f"--offload-arch={ARCH}"]
UNITS = [
    # -fno-slp-vectorize: on gfx950 v_pk_*_f32 issue at twice the cycles of
    # their scalar forms (tools/valu_rates.hip) and cannot take abs modifiers,
    # so SLP packing only adds shuffles and v_and masks (and SGPRs)
    ("render_exact.hip", ["-ffp-contract=off", "-fno-slp-vectorize"]),
    ("render_fast.hip", ["-ffp-contract=fast", "-fno-slp-vectorize"]),
    ("deinterleave.hip", []),
    ("heatmap.hip", []),
    ("tiles.hip", []),
    ("sdf_abi.cpp", ["-ffp-contract=off", "-x", "hip"]),
]
HEADERS = [CSRC / "kernel_args.h", CSRC / "render_kernel.inc", ROOT / "include" / "sdf_abi.h"]


def _hipcc() -> str:
    exe = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(exe).exists():
        raise RuntimeError("hipcc not found: the HIP library cannot be built")
    return exe


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True)


def build_library(force: bool = False, verbose: bool = True) -> Path:
    hipcc = _hipcc()
    OBJ.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    objs = []
    for src, extra in UNITS:
        s = CSRC / src
        o = OBJ / (s.stem + ".o")
        objs.append(o)
        if force or _stale(o, [s, *HEADERS, Path(__file__)]):
            _run([hipcc, *COMMON, *extra, "-c", s, "-o", o], verbose)
    if force or _stale(LIB, objs):
        tmp = LIB.with_suffix(".so.tmp")
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs], verbose)
        os.replace(tmp, LIB)
    return LIB


STATS_LIB = LIB_DIR / "libsdf3d_stats.so"


def build_stats_library(force: bool = False, verbose: bool = True) -> Path:
    """Debug variant of the library whose fast-precision kernel counts
    wave-level culling / evaluation events (render_kernel.inc SDF_STATS;
    read with sdf_debug_stats, tools/kernel_stats.py).  Not used by the
    product path."""
    hipcc = _hipcc()
    odir = OBJ / "stats"
    odir.mkdir(parents=True, exist_ok=True)
    objs = []
    for src, extra in UNITS:
        s = CSRC / src
        o = odir / (s.stem + ".o")
        objs.append(o)
        flags = [*extra, "-DSDF_STATS=1"] if src == "render_fast.hip" else extra
        if force or _stale(o, [s, *HEADERS, Path(__file__)]):
            _run([hipcc, *COMMON, *flags, "-c", s, "-o", o], verbose)
    if force or _stale(STATS_LIB, objs):
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", STATS_LIB, *objs], verbose)
    return STATS_LIB


BIN_DIR = PKG / "bin"
EXAMPLE = ROOT / "examples" / "sdf_main.cpp"


def build_example(force: bool = False, verbose: bool = True) -> Path:
    """The headless C++ host program over include/sdf3d.hpp (links libsdf3d.so)."""
    BIN_DIR.mkdir(parents=True, exist_ok=True)
    exe = BIN_DIR / "sdf_main"
    deps = [EXAMPLE, ROOT / "include" / "sdf3d.hpp", ROOT / "include" / "sdf_abi.h", LIB]
    if force or _stale(exe, deps):
        _run([_hipcc(), "-O2", "-std=c++17", f"--offload-arch={ARCH}", "-I", ROOT / "include",
              EXAMPLE, "-L", LIB_DIR, "-lsdf3d", "-Wl,-rpath,$ORIGIN/../lib", "-o", exe], verbose)
    return exe


def build_oracle(verbose: bool = True) -> Path:
    """Compile the CPU oracle (test infrastructure) with its own Makefile."""
    _run(["make", "-s", "-C", ROOT / "oracle"], verbose)
    return ROOT / "oracle" / "build" / "liboracle.so"


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
    build_example(force="--force" in sys.argv)
    build_oracle()
