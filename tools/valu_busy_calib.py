#!/usr/bin/env python3
"""Calibrate a counter-based VALU-busy for gfx950 on kernels of known issue rate.

ROCm 7.2 ships no gfx950 formula for VALUBusy (MI355X_MICROARCH.md, PMC
slots); the gfx94x one, 100 * SQ_ACTIVE_INST_VALU * 4 / SIMD_NUM /
GRBM_GUI_ACTIVE, assumes 4-cycle VALU issue.  This runs
tools/valu_rates.bin (8 waves per SIMD on every CU, 8 independent chains of
one instruction class per lane, so each kernel is VALU-issue-bound by
construction) under `rocprofv3 --pmc` and reports per class:
  * units = SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU (counter units per wave-instruction),
  * raw   = SQ_ACTIVE_INST_VALU / (SIMDs * GRBM_GUI_ACTIVE / XCDs)
          (counter units per SIMD-cycle; GRBM_GUI_ACTIVE is summed over the 8 XCDs).
A pure full-rate chain (v_fma_f32 / v_add_f32) keeps its SIMD's VALU issue
busy, so cycles_per_unit = 1 / raw there is the gfx950 normalisation:
  VALU_busy = cycles_per_unit * SQ_ACTIVE_INST_VALU / (SIMDs * GRBM_GUI_ACTIVE / XCDs).

    hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates.bin
    python tools/valu_busy_calib.py --out gpurun_out/valu_busy_calib.json
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SIMDS, XCDS = 1024, 8
KINDS = ["v_fma_f32", "v_pk_fma_f32", "v_add_f32", "v_pk_add_f32", "v_sqrt_f32", "v_min_f32",
         "v_cmp+v_cndmask", "sqrt+3fma", "v_mul_f32", "fma_dependent_chain"]
COUNTERS = ["SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_BUSY_CYCLES",
            "GRBM_GUI_ACTIVE"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bin", default=str(ROOT / "tools" / "valu_rates.bin"))
    ap.add_argument("--out", default="gpurun_out/valu_busy_calib.json")
    a = ap.parse_args()
    d = Path("gpurun_out/pmc_valu_calib")
    r = subprocess.run(["rocprofv3", "--pmc", *COUNTERS, "--output-format", "csv", "-d", str(d),
                        "-o", "run", "--", a.bin], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-3000:])
        raise SystemExit(r.returncode)
    rates = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    per = {}
    for f in sorted(d.rglob("*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                m = re.search(r"bench<(\d+)>|benchILi(\d+)E", row["Kernel_Name"])
                if not m:
                    continue
                kind = int(m.group(1) or m.group(2))
                key = (kind, row["Dispatch_Id"])
                per.setdefault(key, {}).setdefault(row["Counter_Name"], 0.0)
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    out = {"method": __doc__.split("\n\n")[0], "kinds": {}}
    for kind, name in enumerate(KINDS):
        ds = [v for (k, _), v in per.items() if k == kind]
        if not ds:
            continue
        ds = ds[1:] or ds           # first launch warms the clocks
        mean = {c: sum(x.get(c, 0.0) for x in ds) / len(ds) for c in COUNTERS}
        units = mean["SQ_ACTIVE_INST_VALU"] / max(mean["SQ_INSTS_VALU"], 1.0)
        raw = mean["SQ_ACTIVE_INST_VALU"] / (SIMDS * mean["GRBM_GUI_ACTIVE"] / XCDS)
        out["kinds"][name] = {"units_per_inst": round(units, 4), "raw_units_per_simd_cycle":
                              round(raw, 4), "cycles_per_wave_inst": rates["rates"][name][
                                  "cycles_per_wave_inst"], "counters": mean}
    full = [out["kinds"][k]["raw_units_per_simd_cycle"] for k in ("v_fma_f32", "v_add_f32")
            if k in out["kinds"]]
    if full:
        out["cycles_per_unit"] = round(len(full) / sum(full), 4)
    print(json.dumps(out, indent=1))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
