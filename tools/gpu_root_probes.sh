#!/bin/bash
# Rank 0 / busiest-peer GPU work per frame at N = 2, 4, 8 for the candidate
# row shares (tools/root_probe.py), one JSON per run in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
# SPECS: "N,a:b ..." (default: the candidate shares at N = 8, 4, 2)
for spec in ${SPECS:-8,1:2 8,1:3 8,1:4 8,2:7 4,1:1 4,3:4 4,2:3 2,1:1 2,4:3}; do
  set -- ${spec/,/ }
  out="gpurun_out/rp$1_${2/:/-}.json"
  timeout -k 10 200 python tools/root_probe.py --world $1 --shares $2 --frames 400 > "$out" 2>> gpurun_out/rp.log
  rc=$?; [ $rc -eq 0 ] || { echo "N=$1 $2 rc=$rc"; exit $rc; }
  python - "$out" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["world"], d["shares"], {k: d[k] for k in ("root_render_ms", "decode_ms", "root_serial_ms",
                                                  "peer_tiles_ms")})
EOF
done
exit 0
