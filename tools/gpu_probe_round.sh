#!/bin/bash
# Feature ablation of C4 and C5 (tools/ablate.py), then the N = 2, 4, 8 root /
# peer probes (tools/gpu_root_probes.sh) for the shares chosen by
# multigpu.choose_shares.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C4 C5; do
  timeout -k 10 300 python tools/ablate.py --config $c > gpurun_out/ablate_$c.json 2> gpurun_out/ablate_$c.log
  rc=$?; echo "ablate $c rc=$rc"; cat gpurun_out/ablate_$c.json; [ $rc -ne 0 ] && exit $rc
done
bash tools/gpu_root_probes.sh
