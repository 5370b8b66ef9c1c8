#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; the script stops at the first step
# that crashes, aborts or times out (exit 124/134/137/139) and never retries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests smoke bench prof}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
      fatal $rc && exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
      fatal $rc && exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.log
      rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.log
      fatal $rc && exit $rc ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-display --no-exact --streams 1 ${PROF_ARGS:-} > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; find gpurun_out/prof -name '*stats*' | head
      fatal $rc && exit $rc ;;
  esac
done
exit 0
