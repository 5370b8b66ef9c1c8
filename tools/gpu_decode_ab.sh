#!/bin/bash
# Decoder A/B (tools/root_probe.py --only decode, rank 0's 49/51 of the 4K C4
# frame): this build's TILES tests first, then the variants in VARS
# (tools/_variants/libsdf3d_<name>.so), alternated, REPS times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
out=gpurun_out/decode_ab.jsonl
if [ -z "$NOTESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_tiles.py tests/test_gpu_multi.py > gpurun_out/decode_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/decode_tests.log; [ $rc -eq 0 ] || exit $rc
fi
probe() {   # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python tools/root_probe.py --world 8 --frames 400 "$@" \
    | sed "s/^{/{\"tag\": \"$tag\", /" >> $out 2>> gpurun_out/decode_ab.log || { echo "$tag rc=$?"; exit 1; }
}
for rep in $(seq ${REPS:-3}); do
  for v in ${VARS:-main esc escvm}; do
    probe $v --shares 2:7 --only decode --lib tools/_variants/libsdf3d_$v.so
  done
done
cat $out
