#!/bin/bash
# Round-6 re-measurement at the final kernels: PMC of every configuration,
# the rocprof kernel stats, the default bench three times and C5 exact three
# times (each GPU step under its own limit; the first failure ends it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS="pmc prof repeats" PMC_SPECS="C4:exact C5:exact:f64 C4:fast C5:fast C3:exact C3:fast C2:exact C2:fast C1:exact C1:fast" \
  bash tools/gpu_final_r6.sh || exit $?
: > gpurun_out/bench_C5_repeats.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config C5 >> gpurun_out/bench_C5_repeats.jsonl 2>> gpurun_out/bench_C5_repeats.log
  rc=$?; echo "C5 bench $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
