#!/bin/bash
# Counter listing + PMC passes for the bench kernel (no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
timeout -k 10 900 python tools/pmc_traffic.py ${PMC_ARGS:-} > gpurun_out/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -40 gpurun_out/pmc.log
exit $rc
