#!/bin/bash
# Instruction counts of the busiest N = 8 peer's TILES render (encoder
# epilogue + compaction) against the plain render of the same rows: one
# rocprofv3 counter pass each (SQ_* only), per-dispatch CSV.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ppmc
export TMPDIR=/tmp
R=$PWD
for m in peer peer_plain; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY \
    --output-format csv -d $R/gpurun_out/ppmc/$m -o run -- python3 $R/tools/root_probe.py --world 8 --shares 2:7 \
    --frames 20 --streams 1 --only $m > $R/gpurun_out/ppmc/$m.log 2>&1 || { echo "$m rc=$?"; exit 1; }
done
find gpurun_out/ppmc -name '*.csv' | head
