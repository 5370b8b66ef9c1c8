#!/bin/bash
# Bench every configuration once (N=1), each with its CPU baseline beside it
# (BASELINE.md:57-58): whole frames for C1/C2/C3, every 2nd 8-row block for
# C4 and every 4th for C5 (the sample is stated in each line's
# cpu_baseline.sample).  One JSON line per run in gpurun_out/configs.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/configs.jsonl
SPECS=${SPECS:-"C4:fast:2 C4:exact:2 C3:fast:1 C3:exact:1 C2:fast:1 C5:exact:4 C5:fast:4 C1:fast:1"}
for spec in $SPECS; do
  IFS=: read -r cfg prec stride <<< "$spec"
  cpu="--cpu-sample-stride $stride --cpu-frames 3"
  [ "${NO_CPU:-0}" = 1 ] && cpu="--no-cpu-baseline"
  timeout -k 10 400 python bench.py --config $cfg --precision $prec --steps 30 --warmup 3 \
    --no-display --no-exact $cpu ${BENCH_EXTRA:-} >> gpurun_out/configs.jsonl 2>> gpurun_out/configs.log
  rc=$?; echo "$spec rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
