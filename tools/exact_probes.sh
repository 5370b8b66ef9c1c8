#!/bin/bash
# The N = 8 frame bound at exact precision: rank 0's
# loop with real RCCL transfers (tools/root_rccl_probe.py) and the busiest
# peer's share (tools/root_probe.py), for SHARES ("a:b ..."), C4 by default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
CFG=${CFG:-C4}
SH=${SHARES:-"2:7 1:7 1:4"}
W=""
for s in $SH; do W="$W,8:$s"; done
timeout -k 10 400 python tools/root_rccl_probe.py --config $CFG --precision exact --worlds ${W#,} \
  --modes full,norccl --out gpurun_out/r05_root_rccl_probe_exact_$CFG.json \
  > gpurun_out/rccl_probe_exact.log 2>&1
rc=$?; echo "rccl probe rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/rccl_probe_exact.log; exit $rc; }
for s in $SH; do
  timeout -k 10 300 python tools/root_probe.py --config $CFG --precision exact --world 8 --shares $s \
    > gpurun_out/r05_root_probe_exact_${CFG}_${s/:/-}.json 2> gpurun_out/root_probe_exact.log
  rc=$?; echo "root probe $s rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/root_probe_exact.log; exit $rc; }
done
exit 0
