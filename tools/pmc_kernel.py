#!/usr/bin/env python3
"""Hardware counters of one kernel, averaged over its dispatches.

Runs `cmd` under rocprofv3 once per counter set (--pmc only, no tracing
domains: MI355X_MICROARCH.md / the pool's rules), keeps the dispatches whose
kernel name contains --kernel, and prints the per-dispatch mean of every
counter plus derived figures:

  valu_per_wave, lds_per_wave, smem_per_wave      instructions per wave
  valu_busy            SQ_ACTIVE_INST_VALU / (SQ_BUSY_CYCLES * 4 SIMDs) (approx.)
  write_bytes, fetch_bytes                         TCC_EA0_WRREQ*64, 2*TCC_EA0_RDREQ*64
                       (the guide's gfx950 corrections for 16-B-per-lane
                       streaming accesses; other widths uncalibrated)

    python tools/pmc_kernel.py --kernel decode_tiles -- python3 tools/root_probe.py --only decode
"""
from __future__ import annotations

import argparse
import csv
import json
import subprocess
import sys
from pathlib import Path

SETS = [
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_SALU",
     "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
    ["SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_WAIT_INST_ANY",
     "SQ_WAVE_CYCLES"],
    ["TCC_EA0_WRREQ_sum", "TCC_EA0_RDREQ_sum", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD"],
]


def run_set(cmd, counters, outdir: Path, kernel: str):
    d = outdir / ("pmc_" + "_".join(c.lower() for c in counters)[:48])
    full = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", str(d), "-o",
            "run", "--", *cmd]
    r = subprocess.run(full, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-3000:])
        raise SystemExit(f"rocprofv3 failed ({r.returncode}) for {counters}")
    files = sorted(d.rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                key = (row.get("Dispatch_Id"), row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    sums, counts = {}, {}
    for (_, name), v in per.items():
        sums[name] = sums.get(name, 0.0) + v
        counts[name] = counts.get(name, 0) + 1
    return {k: sums[k] / counts[k] for k in sums}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--out", default="gpurun_out/pmc_kernel")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    cmd = args.cmd[1:] if args.cmd and args.cmd[0] == "--" else args.cmd
    res = {}
    for cs in SETS:
        res.update(run_set(cmd, cs, Path(args.out), args.kernel))
    w = res.get("SQ_WAVES") or 1.0
    out = {"kernel": args.kernel, "counters": {k: round(v, 1) for k, v in sorted(res.items())}}
    out["valu_per_wave"] = round(res.get("SQ_INSTS_VALU", 0) / w, 1)
    out["lds_per_wave"] = round(res.get("SQ_INSTS_LDS", 0) / w, 1)
    out["smem_per_wave"] = round(res.get("SQ_INSTS_SMEM", 0) / w, 1)
    calib = Path(__file__).resolve().parent.parent / "profiles" / "r02_valu_busy_calib.json"
    if res.get("SQ_ACTIVE_INST_VALU") and res.get("GRBM_GUI_ACTIVE") and calib.exists():
        # tools/pmc_traffic.py's calibrated form (a lower bound)
        cpu = json.loads(calib.read_text())["cycles_per_unit"]
        out["valu_busy_calibrated"] = round(
            cpu * res["SQ_ACTIVE_INST_VALU"] / (1024 * res["GRBM_GUI_ACTIVE"] / 8), 4)
    if "TCC_EA0_WRREQ_sum" in res:
        out["write_bytes"] = res["TCC_EA0_WRREQ_sum"] * 64
        out["fetch_bytes"] = res["TCC_EA0_RDREQ_sum"] * 64 * 2
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
