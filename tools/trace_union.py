#!/usr/bin/env python3
"""GPU-busy time per frame of the pipelined bench loop, from a rocprofv3 kernel trace.

bench.py's frame loop puts frames on 3 alternating HIP streams, so one
frame's render launch overlaps the previous frame's tail: a launch's own
duration (`kernel_ms`, rocprof's average) can exceed the loop's time per
frame (`ms_per_step`).  This reads the `*kernel_trace.csv` of

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- \
        python3 bench.py --steps K --warmup W --no-cpu-baseline --no-display

takes the last K dispatches of the render kernel (the timed frames: with
--no-display the timed loop issues the run's last render launches), and
reports per frame:
  * the mean launch duration (what rocprof's stats average),
  * the UNION of the launches' busy intervals (the GPU time the frames
    really occupy; <= the loop's ms_per_step when nothing else runs),
  * the span from the first start to the last end, and the mean overlap
    between consecutive launches.

    python tools/trace_union.py DIR [--kernel render] [--frames K] [--out file.json]
"""
from __future__ import annotations

import argparse
import csv
import json
from pathlib import Path


def load(trace_dir: Path, kernel: str):
    files = sorted(Path(trace_dir).rglob("*kernel_trace.csv"))
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {trace_dir}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if kernel in name and "render_tiles" not in name:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name,
                                 r.get("Queue_Id"), r.get("Stream_Id")))
    rows.sort()
    return rows


def union_ns(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--kernel", default="render")
    ap.add_argument("--frames", type=int, default=50)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(Path(a.trace_dir), a.kernel)
    sel = rows[-a.frames:]
    k = len(sel)
    iv = [(s, e) for s, e, *_ in sel]
    dur = [(e - s) / 1e6 for s, e in iv]
    overl = [max(0, iv[i][1] - iv[i + 1][0]) / 1e6 for i in range(k - 1)]
    res = {
        "frames": k,
        "dispatches_in_trace": len(rows),
        "queues": sorted({str(q) for *_, q, _ in sel}),
        "mean_launch_ms": round(sum(dur) / k, 4),
        "union_busy_ms_per_frame": round(union_ns(iv) / 1e6 / k, 4),
        "span_ms_per_frame": round((iv[-1][1] - iv[0][0]) / 1e6 / k, 4),
        "mean_overlap_with_next_ms": round(sum(overl) / max(1, len(overl)), 4),
        "kernel": sel[-1][2],
    }
    print(json.dumps(res, indent=1))
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
