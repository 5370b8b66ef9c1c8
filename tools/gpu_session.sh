#!/bin/bash
# One GPU-box session of chained steps, each with its own time limit; the
# first failing step ends the call (never retried).  Steps (STEPS, in order):
#   tests:<pytest args>   python -m pytest <args> -m gpu (log gpurun_out/pytest_<n>.log)
#   ab:<SPECS>            tools/gpu_ab_flags.sh with SPECS (comma-free spec list, ';'-separated)
#   cmd:<command>         any command (log gpurun_out/cmd_<n>.log)
# e.g. STEPS='tests:tests/test_gpu_tiles.py|ab:C5:exact:0:base,new' (| separates steps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra ST <<< "$STEPS"
n=0
for s in "${ST[@]}"; do
  n=$((n + 1))
  kind=${s%%:*}; arg=${s#*:}
  case $kind in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $arg -m gpu -x -q -rf --timeout 300 \
        --timeout-method thread > gpurun_out/pytest_$n.log 2>&1
      rc=$?; echo "step $n tests rc=$rc"; tail -4 gpurun_out/pytest_$n.log ;;
    ab)
      SPECS="${arg//;/ }" bash tools/gpu_ab_flags.sh; rc=$?; echo "step $n ab rc=$rc" ;;
    cmd)
      timeout -k 10 ${CMD_TIMEOUT:-600} bash -c "$arg" > gpurun_out/cmd_$n.log 2>&1
      rc=$?; echo "step $n cmd rc=$rc"; tail -5 gpurun_out/cmd_$n.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  [ $rc -ne 0 ] && exit $rc
done
exit 0
