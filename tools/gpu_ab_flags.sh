#!/bin/bash
# In-process A/B of working-tree flag variants (tools/flag_variant.py) of the
# render kernels: `SPECS` = "config:precision:poses:lib1,lib2,..." entries,
# each lib tools/_variants/libsdf3d_<name>.so (base first); one JSON per spec
# in gpurun_out/ab_<config>_<precision>.json.  Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in $SPECS; do
  IFS=: read -r cfg prec poses libs <<< "$spec"
  L=""
  for n in ${libs//,/ }; do L="$L $n=tools/_variants/libsdf3d_$n.so"; done
  timeout -k 10 300 python tools/ab_kernel.py $L --config $cfg --precision $prec --poses $poses \
    --rounds ${ROUNDS:-9} --out gpurun_out/ab_${cfg}_$prec.json > gpurun_out/ab_${cfg}_$prec.log 2>&1
  rc=$?; echo "$cfg $prec rc=$rc"; grep '^{' gpurun_out/ab_${cfg}_$prec.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
