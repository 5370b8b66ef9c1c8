#!/bin/bash
# Decoder launch-shape A/B (tiles per wave, waves per workgroup) and the
# busiest peer's stream count / serial costs (tools/root_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
out=gpurun_out/decode_ab.jsonl
probe() {   # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python tools/root_probe.py --world 8 --frames 400 "$@" \
    | sed "s/^{/{\"tag\": \"$tag\", /" >> $out 2>> gpurun_out/decode_ab.log || { echo "$tag rc=$?"; exit 1; }
}
for rep in 1 2; do
  for v in ${VARS:-main t2 t8 t4w8 t4w2}; do
    probe $v --shares 2:7 --only decode --lib tools/_variants/libsdf3d_$v.so
  done
done
for ns in 1 3 4; do
  probe "peer_s$ns" --shares 2:7 --only peer --streams $ns
  probe "plain_s$ns" --shares 2:7 --only peer_plain --streams $ns
done
cat $out
