#!/bin/bash
# N default bench runs back to back (no CPU baseline): run-to-run spread of
# the headline number -> gpurun_out/bench_repeats.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/bench_repeats.jsonl
for i in $(seq ${N:-5}); do
  timeout -k 10 300 python bench.py --no-cpu-baseline >> gpurun_out/bench_repeats.jsonl 2>> gpurun_out/bench_repeats.log
  rc=$?; echo "bench $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python - <<'PY'
import json
v = [json.loads(l) for l in open("gpurun_out/bench_repeats.jsonl")]
print([round(x["fps"], 1) for x in v], [x["ms_per_step"] for x in v])
PY
