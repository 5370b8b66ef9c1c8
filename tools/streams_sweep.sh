#!/bin/bash
# N = 1 frame rate against the number of render streams (frames in flight),
# two alternating rounds, exact C4 and C5 by default -> gpurun_out/
# streams_sweep.jsonl (one bench.py line per run, no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/streams_sweep.jsonl
for round in 1 2; do
  for cfg in ${CFGS:-C4 C5}; do
    for s in ${STREAMS:-2 3 4 6}; do
      timeout -k 10 200 python bench.py --config $cfg --streams $s --steps 60 --warmup 5 \
        --no-cpu-baseline --no-display --no-other >> gpurun_out/streams_sweep.jsonl \
        2>> gpurun_out/streams_sweep.log || { echo "rc=$? $cfg $s"; exit 1; }
      echo "$round $cfg $s done"
    done
  done
done
