#!/bin/bash
# Round-6 final measurement session, at the final kernel ids.  STEPS (default
# all, in this order):
#   pmc      PMC summaries (tools/pmc_traffic.py, one rocprofv3 --pmc pass per
#            counter set, no tracing) for PMC_SPECS -> gpurun_out/pmc/
#   prof     rocprofv3 --kernel-trace --stats of the headline bench, one
#            render stream -> gpurun_out/prof/
#   configs  every configuration with its CPU baseline (tools/gpu_configs.sh)
#            -> gpurun_out/configs.jsonl
#   repeats  the default bench REPEATS times -> gpurun_out/bench_repeats.jsonl
# Every GPU step runs under its own limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 0) return 1;; *) return 0;; esac; }
for s in ${STEPS:-pmc prof configs repeats}; do
  case $s in
    pmc)
      SPECS="${PMC_SPECS:-C4:exact C5:exact:f64 C4:fast C5:fast C3:exact C2:exact C1:exact}" \
        bash tools/gpu_pmc_configs.sh
      rc=$?; echo "pmc rc=$rc"; fatal $rc && exit $rc ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-display --no-exact --streams 1 \
        > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; fatal $rc && exit $rc ;;
    configs)
      SPECS="${CFG_SPECS:-C4:exact:2 C4:fast:2 C5:exact:4 C5:fast:4 C3:exact:1 C3:fast:1 C2:exact:1 C2:fast:1 C1:exact:1 C1:fast:1}" \
        bash tools/gpu_configs.sh
      rc=$?; echo "configs rc=$rc"; fatal $rc && exit $rc ;;
    repeats)
      : > gpurun_out/bench_repeats.jsonl
      for i in $(seq ${REPEATS:-3}); do
        timeout -k 10 400 python bench.py >> gpurun_out/bench_repeats.jsonl 2>> gpurun_out/bench_repeats.log
        rc=$?; echo "bench $i rc=$rc"; fatal $rc && exit $rc
      done ;;
  esac
done
exit 0
