#!/bin/bash
# Round 4 decode / compaction A/B session: the TILES and driver tests, then
#  - rank 0's decode (2:7 at N = 8) for this build and the variants in VARS;
#  - the busiest peer: compaction on the render stream with this build and
#    with $OLD (four-wave compaction workgroups), on a stream of its own
#    (normal / high priority), and the plain render.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
out=gpurun_out/split_probe.jsonl
if [ -z "$NOTESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_tiles.py tests/test_gpu_multi.py tests/test_gpu_driver.py > gpurun_out/split_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/split_tests.log; [ $rc -eq 0 ] || exit $rc
fi
probe() {   # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python tools/root_probe.py --world 8 --frames 400 "$@" \
    | sed "s/^{/{\"tag\": \"$tag\", /" >> $out 2>> gpurun_out/split_probe.log || { echo "$tag rc=$?"; exit 1; }
}
OLD=${OLD:-tools/_variants/libsdf3d_olddec.so}
for rep in 1 2; do
  probe main --shares 2:7 --only decode
  for v in ${VARS:-olddec dec64 decnt dec64nt}; do
    probe $v --shares 2:7 --only decode --lib tools/_variants/libsdf3d_$v.so
  done
done
for rep in 1 2; do
  probe main --shares 2:7 --only peer
  probe old --shares 2:7 --only peer --lib $OLD
  probe split --shares 2:7 --only peer_split
  probe split_hi --shares 2:7 --only peer_split --cs-priority -1
  probe plain --shares 2:7 --only peer_plain
done
cat $out
