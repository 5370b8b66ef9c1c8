#!/bin/bash
# tools/gpu_ab.sh, then the same A/B in exact precision (bit-exactness of the
# working tree's exact kernels against the base library's)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_ab.sh || exit $?
LIBS=${LIBS:-base=tools/_variants/libsdf3d_base.so new=sdf3d_amd/lib/libsdf3d.so}
for c in ${CONFIGS:-C4}; do
  timeout -k 10 300 python tools/ab_kernel.py $LIBS --config $c --precision exact \
    --poses ${POSES:-0,1,2,3} --out gpurun_out/ab_${c}_exact.json > gpurun_out/ab_${c}_exact.log 2>&1
  rc=$?; echo "ab exact $c rc=$rc"; grep '^{' gpurun_out/ab_${c}_exact.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
