#!/bin/bash
# PMC summaries (tools/pmc_traffic.py: one rocprofv3 --pmc pass per counter
# set, no tracing domains) for SPECS = "config:precision ..." ->
# gpurun_out/pmc/pmc_<cfg>_<prec>.json (copy into profiles/ to commit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${SPECS:-C4:exact C4:fast}; do
  IFS=: read -r c p x <<< "$spec"
  # a third field "f64" adds the fp64 VALU pass
  timeout -k 10 600 python tools/pmc_traffic.py --config $c --precision $p --out gpurun_out/pmc \
    ${x:+--$x} \
    > gpurun_out/pmc_${c}_$p.log 2>&1
  rc=$?; echo "pmc $c $p rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${c}_$p.log; exit $rc; }
done
exit 0
