#!/usr/bin/env python3
"""Collect rocprofv3 PMC counters for the bench's render kernel.

Runs bench.py under rocprofv3 once per counter pass (one --pmc set per run, no
tracing domains besides the counters themselves), averages each counter over
the render-kernel dispatches, and writes profiles/pmc_<cfg>_<precision>.json:

  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
      FETCH_SIZE / WRITE_SIZE are kB; on gfx950 FETCH_SIZE reports half the
      bytes of a wide coalesced read, so it is doubled (MI355X_MICROARCH.md
      "HBM"); WRITE_SIZE is exact for 16-B-per-lane stores (our float4 stores).
  valu_lane_util = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)   (when available)
  executed_flops_per_launch = 64 x (ADD + MUL + TRANS + 2 FMA) wave-instructions
      x valu_lane_util: the flops of the lanes that were active (the counters
      count a wave-instruction whatever its EXEC mask)
  kernel_id = sdf_kernel_id(precision) of the library profiled (sdf_abi.h):
      bench.py applies these counters only to a kernel with the same id

    python tools/pmc_traffic.py [--config C4] [--precision fast] [--out DIR]

This script never touches the GPU itself: every profiled run is a child
process started by rocprofv3.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES",
     "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
    ["SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
     "SQ_WAIT_ANY"],
    ["SQ_INSTS_VALU_FLOPS_FP32", "SQ_INSTS_VALU_FLOPS_FP32_TRANS", "SQ_INSTS_VALU_TRANS_F32",
     "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_ADD_F32"],
    ["SQ_INSTS", "SQ_INSTS_BRANCH", "SQ_IFETCH", "SQ_INST_CYCLES_SALU", "SQ_ACTIVE_INST_SCA",
     "SQ_ACTIVE_INST_MISC"],
    ["SQ_LEVEL_WAVES", "SQ_CYCLES", "SQ_BUSY_CU_CYCLES", "SQ_INSTS_VSKIPPED",
     "SQ_ACTIVE_INST_VMEM", "SQ_INST_LEVEL_SMEM"],
]
# --f64: the fp64 VALU mix (C5's exact bulb runs its map in f64)
F64_PASS = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
            "SQ_INSTS_VALU_TRANS_F64"]


def run_pass(counters, cfg, prec, outdir, steps):
    d = outdir / ("pmc_" + "_".join(c.lower() for c in counters)[:60])
    # each pass under its own kill timer (a counter request the hardware
    # cannot serve makes rocprofv3 hang)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", str(d), "-o", "run",
           "--", sys.executable, str(ROOT / "bench.py"), "--config", cfg, "--precision", prec,
           "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline", "--no-display", "--no-exact",
           "--streams", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    files = list(d.rglob("*counter_collection*.csv"))
    if r.returncode != 0 or not files:
        return None, (r.stderr or "")[-800:]
    vals = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "render" not in row.get("Kernel_Name", ""):
                    continue
                vals[(row["Counter_Name"], row.get("Dispatch_Id"))].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (name, _), v in vals.items():
        per[name].append(sum(v))           # sum over dimensions (XCDs / SEs) per dispatch
    return {k: sum(v) / len(v) for k, v in per.items()}, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--precision", default="fast")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/pmc")
    ap.add_argument("--f64", action="store_true", help="add the fp64 VALU pass")
    args = ap.parse_args()
    outdir = ROOT / args.out
    outdir.mkdir(parents=True, exist_ok=True)
    res, errors = {}, {}
    for counters in PASSES + ([F64_PASS] if args.f64 else []):
        v, err = run_pass(counters, args.config, args.precision, outdir, args.steps)
        if v is None:
            errors[",".join(counters)] = err
            print("pass failed:", counters, err[-300:] if err else "", flush=True)
            continue
        res.update(v)
        print("pass ok:", counters, {k: v[k] for k in v}, flush=True)
    sys.path.insert(0, str(ROOT))
    from sdf3d_amd import abi, scenes
    f = scenes.config(args.config)
    prec = abi.PRECISION_FAST if args.precision == "fast" else abi.PRECISION_EXACT
    kid = abi.load_library().sdf_kernel_id(prec)
    algo_bytes = f.params.width * f.params.height * 16
    out = {"config": args.config, "precision": args.precision, "counters": res,
           "kernel_id": kid.decode() if kid else None,
           "algorithmic_bytes_per_launch": algo_bytes, "errors": errors,
           "method": "rocprofv3 --pmc, one pass per counter set, mean over render dispatches; "
                     "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)"}
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        out["fetch_bytes_per_launch"] = 2 * res["FETCH_SIZE"] * 1024
        out["write_bytes_per_launch"] = res["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = out["fetch_bytes_per_launch"] + out["write_bytes_per_launch"]
    if all(k in res for k in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
                              "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32")):
        # hardware-counted fp32 work the (culled) kernel executed, Omniperf's VALU
        # FLOPs formula: 64 lanes x (ADD + MUL + TRANS + 2 FMA) wave-instructions.
        # min/max/compare are not counted by these counters (the algorithmic
        # count does count them), so this is a lower bound on executed flops.
        out["executed_flops_all_lanes_per_launch"] = 64.0 * (
            res["SQ_INSTS_VALU_ADD_F32"] + res["SQ_INSTS_VALU_MUL_F32"]
            + res["SQ_INSTS_VALU_TRANS_F32"] + 2.0 * res["SQ_INSTS_VALU_FMA_F32"])
        if res.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in res:
            # only the lanes the EXEC mask enabled did the work
            lanes = res["SQ_THREAD_CYCLES_VALU"] / (64 * res["SQ_ACTIVE_INST_VALU"])
            out["executed_flops_per_launch"] = out["executed_flops_all_lanes_per_launch"] * lanes
    need = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
            "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32", "SQ_WAVES", "GRBM_GUI_ACTIVE")
    if all(k in res for k in need):
        # instruction mix per wave: full-rate add/mul/FMA, transcendentals, and
        # the remainder (min/max/cmp/cndmask/mov/logic, not split by counters)
        full = res["SQ_INSTS_VALU_ADD_F32"] + res["SQ_INSTS_VALU_MUL_F32"] + res["SQ_INSTS_VALU_FMA_F32"]
        trans = res["SQ_INSTS_VALU_TRANS_F32"]
        other = res["SQ_INSTS_VALU"] - full - trans
        out["valu_mix_per_wave"] = {"full_rate": full / res["SQ_WAVES"],
                                    "transcendental": trans / res["SQ_WAVES"],
                                    "other": other / res["SQ_WAVES"],
                                    "total": res["SQ_INSTS_VALU"] / res["SQ_WAVES"]}
    f64 = [k for k in F64_PASS if k in res]
    if f64 and "SQ_WAVES" in res:
        out["valu_f64_per_wave"] = {k[len("SQ_INSTS_VALU_"):]: res[k] / res["SQ_WAVES"] for k in f64}
    calib = ROOT / "profiles" / "r02_valu_busy_calib.json"
    if res.get("SQ_ACTIVE_INST_VALU") and res.get("GRBM_GUI_ACTIVE") and calib.exists():
        # counter-based VALU busy, gfx950 normalisation calibrated on pure
        # full-rate VALU chains (tools/valu_busy_calib.py): SIMD cycles per
        # SQ_ACTIVE_INST_VALU unit over 1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs
        cpu = json.loads(calib.read_text())["cycles_per_unit"]
        out["valu_busy"] = cpu * res["SQ_ACTIVE_INST_VALU"] / (1024 * res["GRBM_GUI_ACTIVE"] / 8)
        out["valu_busy_method"] = (f"{cpu} cycles/unit x SQ_ACTIVE_INST_VALU / (1024 SIMDs x "
                                   "GRBM_GUI_ACTIVE / 8); a lower bound (half-rate "
                                   "min/max/cmp count one unit)")
    if res.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in res:
        out["valu_lane_util"] = res["SQ_THREAD_CYCLES_VALU"] / (64 * res["SQ_ACTIVE_INST_VALU"])
    p = outdir / f"pmc_{args.config}_{args.precision}.json"   # copy into profiles/ to commit
    p.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
