#!/bin/bash
# N = 8 bounds at exact precision, 1:7 shares: rank 0's
# loop with the receive side only (recvcopy), with both RCCL ends (full),
# without transfer (norccl), decode only; the busiest peer's TILES render
# and its plain render; the one-GPU frame (bench) -- for C4 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-C4 C5}; do
  timeout -k 10 400 python tools/root_rccl_probe.py --config $cfg --precision exact --worlds 8:1:7 \
    --batches 2 --modes ${MODES:-recvkernel,recvcopy,full,norccl,decode} --frames ${FRAMES:-400} \
    --out gpurun_out/n8_rccl_$cfg.json > gpurun_out/n8_rccl_$cfg.log 2>&1
  rc=$?; echo "rccl probe $cfg rc=$rc"; grep -o '"mode": "[a-z]*"\|"ms_per_frame": [0-9.]*' gpurun_out/n8_rccl_$cfg.log | paste - - 
  case $rc in 0) ;; *) exit $rc;; esac
  for leg in peer peer_plain; do
    timeout -k 10 200 python tools/root_probe.py --world 8 --shares 1:7 --config $cfg --precision exact \
      --frames ${FRAMES:-400} --only $leg > gpurun_out/n8_${leg}_$cfg.json 2>> gpurun_out/n8_probe.log
    rc=$?; echo "$leg $cfg rc=$rc $(cat gpurun_out/n8_${leg}_$cfg.json)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
exit 0
