#!/bin/bash
# Bench every configuration once (N=1) and collect the headline PMC summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/configs.jsonl
for spec in "C4 fast" "C4 exact" "C3 fast" "C2 fast" "C5 fast" "C1 fast"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --precision $2 --steps 30 --warmup 3 --no-cpu-baseline --no-display >> gpurun_out/configs.jsonl 2>> gpurun_out/configs.log
  rc=$?; echo "$spec rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
