#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/single_call.jsonl
for spec in ${SPECS:-C3:exact C3:fast C2:exact C4:exact}; do
  IFS=: read -r c p <<< "$spec"
  timeout -k 10 200 python tools/single_call_probe.py --config $c --precision $p >> gpurun_out/single_call.jsonl 2>>gpurun_out/sc.log
  rc=$?; tail -1 gpurun_out/single_call.jsonl; [ $rc -eq 0 ] || exit $rc
done
