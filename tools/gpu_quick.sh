#!/bin/bash
# Quick round-6 check: the full GPU test suite, then the default bench (C4
# exact) and C5 exact without CPU baselines -> gpurun_out/{pytest_gpu.log,
# bench_C4.json, bench_C5.json}.  Every GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for c in ${CFGS:-C4 C5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.log
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && { tail -3 gpurun_out/bench_$c.log; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_$c.json')); f=d.get('fast') or {}
print('$c value', d['value'], 'fps', d['fps'], 'kernel_ms', d['kernel_ms'], 'same_run', d['parity'].get('same_run',{}).get('bit_exact'), 'fast fps', f.get('fps'), f.get('kernel_ms'))"
done
exit 0
