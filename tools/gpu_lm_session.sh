#!/bin/bash
# Lane-major TILES: the TILES / multi-device / driver GPU tests, then rank 0's
# decode and the busiest peer at N = 8 (2:7) for the plane-major build (main)
# and this one (lm), alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
out=gpurun_out/lm_ab.jsonl; : > $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_tiles.py tests/test_gpu_multi.py tests/test_gpu_driver.py > gpurun_out/lm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lm_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main lm; do
    for m in decode peer; do
      timeout -k 10 120 python tools/root_probe.py --world 8 --shares 2:7 --frames 400 --streams 4 --only $m \
        --lib tools/_variants/libsdf3d_$v.so | sed "s/^{/{\"tag\": \"$v\", /" >> $out || { echo "$v $m failed"; exit 1; }
    done
  done
done
cat $out
