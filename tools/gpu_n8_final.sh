#!/bin/bash
# N = 8 bound probes at the bench's N > 1 settings (exact, 1:7, batch 2):
# C4 with 4 buffer sets / peer streams, C5 with 8; 12 hardware queues.
# -> gpurun_out/n8f_rccl_<cfg>.json, gpurun_out/n8f_peer.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp GPU_MAX_HW_QUEUES=12
: > gpurun_out/n8f_peer.jsonl
for spec in C4:4 C5:8; do
  IFS=: read -r cfg ns <<< "$spec"
  timeout -k 10 400 python tools/root_rccl_probe.py --config $cfg --precision exact --worlds 8:1:7 \
    --batches 2 --sets $ns --modes recvkernel,norccl,decode --frames 300 \
    --out gpurun_out/n8f_rccl_$cfg.json > gpurun_out/n8f_rccl_$cfg.log 2>&1
  rc=$?; echo "rccl $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep -o '"mode": "[a-z]*"\|"ms_per_frame": [0-9.]*' gpurun_out/n8f_rccl_$cfg.log | paste - -
  for leg in peer peer_plain; do
    out=$(timeout -k 10 200 python tools/root_probe.py --world 8 --shares 1:7 --config $cfg --precision exact \
      --frames 300 --streams $ns --only $leg 2>> gpurun_out/n8f_probe.log) || exit 1
    echo "{\"streams\": $ns, \"result\": $out}" >> gpurun_out/n8f_peer.jsonl; echo "$cfg $leg $out"
  done
done
