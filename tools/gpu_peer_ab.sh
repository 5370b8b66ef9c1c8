#!/bin/bash
# Busiest-peer A/B at N = 8, shares 2:7 (tools/root_probe.py --only peer):
# this build's TILES tests first (unless NOTESTS), then the variants in VARS
# (tools/_variants/libsdf3d_<name>.so), alternated, REPS times, plus the
# plain RGBA32F render of the same rows; the stream's width statistics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
out=gpurun_out/peer_ab.jsonl
if [ -z "$NOTESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_tiles.py tests/test_gpu_multi.py > gpurun_out/peer_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/peer_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python tools/tiles_stats.py >> $out 2>> gpurun_out/peer_ab.log || { echo "stats rc=$?"; exit 1; }
probe() {   # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python tools/root_probe.py --world 8 --frames 400 --streams ${STREAMS:-4} "$@" \
    | sed "s/^{/{\"tag\": \"$tag\", /" >> $out 2>> gpurun_out/peer_ab.log || { echo "$tag rc=$?"; exit 1; }
}
for rep in $(seq ${REPS:-2}); do
  for v in ${VARS:-main narrow}; do
    probe $v --shares 2:7 --only peer --lib tools/_variants/libsdf3d_$v.so
  done
  probe plain --shares 2:7 --only peer_plain
done
cat $out
