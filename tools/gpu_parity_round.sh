#!/bin/bash
# GPU parity session: the -m gpu suite (replay-diagnosed policy), smoke, and
# the full-size replay survey (tools/fullsize_parity.py).  Each GPU step has
# its own time limit; the first failing step ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests smoke survey}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=30 --timeout 300 --timeout-method thread \
        ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc ;;
    survey)
      timeout -k 10 600 python tools/fullsize_parity.py --configs ${SURVEY_CONFIGS:-C4,C3,C2,C5} \
        --out gpurun_out/fullsize_parity.json > gpurun_out/fullsize_parity.log 2>&1
      rc=$?; echo "survey rc=$rc"; tail -12 gpurun_out/fullsize_parity.log; [ $rc -ne 0 ] && exit $rc ;;
  esac
done
exit 0
