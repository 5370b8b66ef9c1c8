#!/bin/bash
# bench.py at N = 1 over render-stream counts (frames in flight)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/streams.jsonl
for cfg in ${CFGS:-C5 C4}; do for ns in ${NSS:-3 4 6 8}; do
  timeout -k 10 300 python bench.py --config $cfg --streams $ns --steps 60 --no-cpu-baseline --no-display --no-exact \
    >> gpurun_out/streams.jsonl 2>>gpurun_out/streams.log
  rc=$?; python -c "
import json; d=[json.loads(l) for l in open('gpurun_out/streams.jsonl')][-1]
print('$cfg', $ns, d['fps'], d['ms_per_step'], d['kernel_ms'])"; [ $rc -eq 0 ] || exit $rc
done; done
