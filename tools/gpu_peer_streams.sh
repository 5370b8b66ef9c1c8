#!/bin/bash
# The busiest peer's TILES share at N = 8 (1:7 shares, exact) over render
# stream counts, with HQ hardware queues -> gpurun_out/peer_streams.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/peer_streams.jsonl
for cfg in ${CFGS:-C4 C5}; do for ns in ${NSS:-3 4 6 8}; do for leg in ${LEGS:-peer}; do
  out=$(GPU_MAX_HW_QUEUES=${HQ:-12} timeout -k 10 200 python tools/root_probe.py --world 8 --shares 1:7 --config $cfg \
    --precision exact --frames ${FRAMES:-300} --streams $ns --only $leg 2>> gpurun_out/peer_streams.log) || exit 1
  echo "{\"streams\": $ns, \"hw_queues\": ${HQ:-12}, \"result\": $out}" >> gpurun_out/peer_streams.jsonl
  echo "$cfg $ns $leg $out"
done; done; done
