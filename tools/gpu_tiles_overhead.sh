#!/bin/bash
# The TILES wire's cost on a peer's share: RGBA32F / SHADE32F / TILES frames
# of the N = 8, 1:7 peer rows, 3-8 render streams (tools/tiles_overhead_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/tiles_overhead.jsonl
for c in ${CFGS:-C5 C4}; do for ns in ${NSS:-3 4 6 8}; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python tools/tiles_overhead_probe.py --config $c --streams $ns \
    >> gpurun_out/tiles_overhead.jsonl 2>>gpurun_out/tp.log
  rc=$?; tail -1 gpurun_out/tiles_overhead.jsonl; [ $rc -eq 0 ] || exit $rc
done; done
