#!/bin/bash
# Decode-only A/B (tools/root_probe.py --only decode) of the in-tree library
# ("tree") against tools/_variants/libsdf3d_<name>.so for LIBS = "name ...",
# PRECS (default "exact"), world 8, SHARES (default 1:7), ROUNDS alternating
# rounds -> gpurun_out/decode_libs.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/decode_libs.jsonl
for round in $(seq ${ROUNDS:-2}); do
  for prec in ${PRECS:-exact}; do
    for lib in tree $LIBS; do
      L=""; [ $lib != tree ] && L="--lib tools/_variants/libsdf3d_$lib.so"
      out=$(timeout -k 10 200 python tools/root_probe.py --precision $prec --world 8 --shares ${SHARES:-1:7} \
        --only decode $L 2> gpurun_out/decode_libs.log) || { echo "rc=$? $prec $lib"; tail -3 gpurun_out/decode_libs.log; exit 1; }
      echo "{\"round\": $round, \"lib\": \"$lib\", \"result\": $out}" | tr -d '\n' >> gpurun_out/decode_libs.jsonl
      echo >> gpurun_out/decode_libs.jsonl
    done
  done
done
cat gpurun_out/decode_libs.jsonl
