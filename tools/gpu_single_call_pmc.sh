#!/bin/bash
# Per-variant counters of the single-call path: for each leg
# of tools/single_call_probe.py (render / frames1 / scheduled), C3 exact, the
# render kernels' counters (tools/pmc_kernel.py: one rocprofv3 --pmc pass
# per set, each under its own kill timer) -> gpurun_out/single_call_pmc_<leg>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for leg in render frames1 scheduled; do
  env ${LEG_ENV:-X=0} timeout -k 10 500 python tools/pmc_kernel.py --kernel render --out gpurun_out/pmc_sc_$leg -- \
    python3 tools/single_call_probe.py --config ${CFG:-C3} --precision exact --rounds 1 --calls 50 --only $leg \
    > gpurun_out/single_call_pmc_$leg.json 2> gpurun_out/single_call_pmc_$leg.log
  rc=$?; echo "$leg rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/single_call_pmc_$leg.log; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/single_call_pmc_$leg.json')); print('$leg', d.get('valu_busy_calibrated'), d['valu_per_wave'])"
done
