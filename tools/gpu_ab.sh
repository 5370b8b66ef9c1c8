#!/bin/bash
# One GPU-box session for a kernel change: GPU tests, then an in-process A/B
# of the working-tree library against tools/_variants/libsdf3d_base.so
# (tools/build_variant.sh <rev> base), then culling event counts of both
# (tools/_variants/libsdf3d_base_stats.so, sdf3d_amd/lib/libsdf3d_stats.so).
# Each GPU step has its own time limit; the first failing step ends the call.
#   TESTS="tests/test_gpu_parity.py" POSES=0,1,2,3 CONFIGS="C4 C3" bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
POSES=${POSES:-0,1,2,3}
CONFIGS=${CONFIGS:-C4}
# name=path pairs; bit-exactness is reported against the first
LIBS=${LIBS:-base=tools/_variants/libsdf3d_base.so new=sdf3d_amd/lib/libsdf3d.so}
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 300 \
    --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/ab_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
for c in $CONFIGS; do
  timeout -k 10 300 python tools/ab_kernel.py $LIBS --config $c --poses $POSES --out gpurun_out/ab_$c.json \
    > gpurun_out/ab_$c.log 2>&1
  rc=$?; echo "ab $c rc=$rc"; cat gpurun_out/ab_$c.log | grep '^{'
  [ $rc -ne 0 ] && exit $rc
done
if [ -f tools/_variants/libsdf3d_base_stats.so ] && [ -f sdf3d_amd/lib/libsdf3d_stats.so ]; then
  for v in base new; do
    lib=tools/_variants/libsdf3d_base_stats.so
    [ $v = new ] && lib=sdf3d_amd/lib/libsdf3d_stats.so
    timeout -k 10 120 python tools/kernel_stats.py --lib $lib --out gpurun_out/stats_$v.json \
      > gpurun_out/stats_$v.log 2>&1
    rc=$?; echo "stats $v rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
fi
exit 0
