#!/bin/bash
# End-of-round measurement session: every configuration with its CPU
# baseline (tools/gpu_configs.sh), the default bench REPEATS times, and the
# rocprofv3 kernel-trace summary of the headline bench (tools/gpu_round.sh
# prof).  Outputs under gpurun_out/ (configs.jsonl, bench_repeats.jsonl,
# prof/).  Each step has its own time limit; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_configs.sh || exit $?
: > gpurun_out/bench_repeats.jsonl
for i in $(seq ${REPEATS:-3}); do
  timeout -k 10 400 python bench.py >> gpurun_out/bench_repeats.jsonl 2>> gpurun_out/bench_repeats.log
  rc=$?; echo "bench $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
STEPS=prof bash tools/gpu_round.sh
