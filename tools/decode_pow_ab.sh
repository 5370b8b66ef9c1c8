#!/bin/bash
# A/B of the TILES decoder's specular pow (tiles.hip SDF_SHADE_LIBRARY_POW):
# the in-tree build (repeated squaring) against tools/_variants/
# libsdf3d_tpow1.so (library pow), decode only, fast and exact streams, two
# alternating rounds -> gpurun_out/decode_pow_ab.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/decode_pow_ab.jsonl
for round in 1 2; do
  for prec in fast exact; do
    for lib in tree tpow1; do
      L=""; [ $lib = tpow1 ] && L="--lib tools/_variants/libsdf3d_tpow1.so"
      out=$(timeout -k 10 200 python tools/root_probe.py --precision $prec --world 8 --shares 2:7 \
        --only decode $L 2> gpurun_out/decode_pow_ab.log) || { echo "rc=$? $prec $lib"; tail -3 gpurun_out/decode_pow_ab.log; exit 1; }
      echo "{\"round\": $round, \"lib\": \"$lib\", \"result\": $out}" | tr -d '\n' >> gpurun_out/decode_pow_ab.jsonl
      echo >> gpurun_out/decode_pow_ab.jsonl
    done
  done
done
cat gpurun_out/decode_pow_ab.jsonl
