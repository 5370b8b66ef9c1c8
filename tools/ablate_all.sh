#!/bin/bash
# Stage ablations (tools/ablate.py, the frame split into primary, normal, AO
# and shadow) for SPECS = "config:precision ..." -> gpurun_out/<TAG>_ablate_
# <config>_<precision>.json; needs tools/_variants/libsdf3d_nonormal.so
# (python tools/flag_variant.py nonormal -DSDF_ABLATE_NO_NORMAL=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for spec in ${SPECS:-C4:exact C4:fast C5:exact C5:fast}; do
  IFS=: read -r c p <<< "$spec"
  timeout -k 10 240 python tools/ablate.py --config $c --precision $p --stages-only \
    --no-normal-lib tools/_variants/libsdf3d_nonormal.so \
    --out gpurun_out/${TAG:-r05}_ablate_${c}_$p.json > gpurun_out/ablate_${c}_$p.log 2>&1
  rc=$?; echo "ablate $c $p rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/ablate_${c}_$p.log; exit $rc; }
done
exit 0
