#!/usr/bin/env python3
"""Build libsdf3d.so variants of the WORKING TREE with extra preprocessor
flags on the render translation units (kernel A/B experiments), side by side
for tools/ab_kernel.py:

    python tools/flag_variant.py NAME [--sched=default] [--units=tiles] [-DFLAG=1 ...]
        -> tools/_variants/libsdf3d_NAME.so

The units whose names start with one of --units (default: render_, the
render units) are compiled with the flags into tools/_variants/NAME/; every other object is the in-tree build's
(sdf3d_amd/build/*.o, built first).  Variants of several names build in
parallel when run as separate processes.
"""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    flags = ["-DSDF_EXPERIMENT=1", *flags]   # unlocks the experiment-only knobs (tiles.hip)
    prefixes = ("render_",)
    # --sched=NAME (after NAME): the render units' scheduler strategy
    # (max-ilp, iterative-ilp, ..., or default: none)
    sched = None
    if len(flags) > 1 and flags[1].startswith("--sched="):
        sched = flags[1].split("=", 1)[1]
        flags = [flags[0], *flags[2:]]
    if len(flags) > 1 and flags[1].startswith("--units="):
        prefixes = tuple(flags[1].split("=", 1)[1].split(","))
        flags = [flags[0], *flags[2:]]
    from sdf3d_amd import build as b
    b.build_library(verbose=False)
    out = ROOT / "tools" / "_variants" / name
    out.mkdir(parents=True, exist_ok=True)
    objs = []
    for src, extra in b.UNITS:
        if src.startswith(prefixes):
            o = out / (Path(src).stem + ".o")
            if sched is not None:   # replace the unit's scheduler strategy
                ex = []
                it = iter(extra)
                for f in it:
                    if f == "-mllvm":
                        g = next(it)
                        if g.startswith("-amdgpu-sched-strategy="):
                            continue
                        ex += [f, g]
                    else:
                        ex.append(f)
                extra = ex + ([] if sched == "default" else
                              ["-mllvm", f"-amdgpu-sched-strategy={sched}"])
            subprocess.run([b._hipcc(), *b.COMMON, *extra, *flags, "-I", str(b.OBJ), "-c",
                            str(b.CSRC / src), "-o", str(o)], check=True)
        else:
            o = b.OBJ / (Path(src).stem + ".o")
        objs.append(str(o))
    lib = ROOT / "tools" / "_variants" / f"libsdf3d_{name}.so"
    subprocess.run([b._hipcc(), f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", str(lib),
                    *objs, "-lhiprtc", "-ldl"], check=True)
    print(lib)


if __name__ == "__main__":
    main()
