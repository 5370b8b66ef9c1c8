#!/bin/bash
# The round's measurement session on one MI355X, in order:
#   1. PMC counter passes of the render kernel for C4, C5, C2 (fast), copied
#      into profiles/ on the box so that bench.py's roofline reads this
#      kernel's counters (copy gpurun_out/pmc/pmc_*.json into profiles/ here);
#   2. every configuration benched once (gpurun_out/configs.jsonl);
#   3. the default bench (gpurun_out/bench.json);
#   4. rocprofv3 --kernel-trace --stats of the serialised bench (--streams 1)
#      and a kernel trace of the 3-stream loop (tools/trace_union.py).
# Each GPU step has its own time limit; the first failing step ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-pmc configs bench prof trace}
for s in $STEPS; do
  case $s in
    pmc)
      for spec in ${PMC_SPECS:-C4:fast C4:exact C5:fast C5:exact C2:fast}; do
        c=${spec%%:*}; p=${spec##*:}
        timeout -k 10 400 python tools/pmc_traffic.py --config $c --precision $p \
          --out gpurun_out/pmc > gpurun_out/pmc_${c}_$p.log 2>&1
        rc=$?; echo "pmc $c $p rc=$rc"; [ $rc -ne 0 ] && exit $rc
        cp gpurun_out/pmc/pmc_${c}_$p.json profiles/
      done ;;
    configs)
      : > gpurun_out/configs.jsonl
      for spec in ${CONFIG_SPECS:-"C4 fast" "C4 exact" "C3 fast" "C3 exact" "C2 fast" "C5 fast" "C5 exact" "C1 fast"}; do
        set -- $spec
        timeout -k 10 300 python bench.py --config $1 --precision $2 --steps 30 --warmup 3 \
          --no-cpu-baseline --no-display --no-exact >> gpurun_out/configs.jsonl 2>> gpurun_out/configs.log
        rc=$?; echo "$spec rc=$rc"; [ $rc -ne 0 ] && exit $rc
      done ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log
      rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -ne 0 ] && exit $rc ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
        -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-display \
        --no-exact --streams 1 > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    trace)
      rm -rf gpurun_out/trace3
      timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace3 \
        -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-display --no-exact \
        > gpurun_out/trace3.log 2>&1
      rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
      python tools/trace_union.py gpurun_out/trace3 --frames 50 \
        --out gpurun_out/trace_union_C4_3streams.json ;;
  esac
done
exit 0
