#!/bin/bash
# Round-6 GPU session: tests (full GPU suite), block counts of the C4 exact
# kernel (tools/block_counts.py), bench.  Every GPU step has its own limit;
# the script stops at the first step that crashes or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-tests blocks bench}
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
      fatal $rc && exit $rc ;;
    blocks)
      timeout -k 10 300 python tools/block_counts.py run --config ${BCFG:-C4} --precision exact > gpurun_out/blocks_run.log 2>&1
      rc=$?; echo "blocks rc=$rc"; tail -1 gpurun_out/blocks_run.log
      fatal $rc && exit $rc ;;
    blocks5)
      timeout -k 10 300 python tools/block_counts.py run --tag blocks_bulb --config C5 --precision exact > gpurun_out/blocks5_run.log 2>&1
      rc=$?; echo "blocks5 rc=$rc"; tail -1 gpurun_out/blocks5_run.log
      fatal $rc && exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.log
      rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/bench.json')); f=d.get('fast') or {}
print('value', d['value'], 'fps', d['fps'], 'kernel_ms', d['kernel_ms'], 'same_run', d['parity'].get('same_run',{}).get('bit_exact'), 'fast fps', f.get('fps'), f.get('kernel_ms'))"
      fatal $rc && exit $rc ;;
  esac
done
exit 0
