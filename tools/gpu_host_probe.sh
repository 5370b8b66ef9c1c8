#!/bin/bash
# Rank 0's host time per frame of the native frame driver at world N (default
# 8) with all ranks on this one GPU over the stand-in communications library
# (tests/shmcomm, asynchronous), for several ship batches: bench.py's
# driver_host_us_per_frame (the driver's own calls, waits excluded).  One
# JSON line per batch in gpurun_out/host_probe.jsonl.
#   BATCHES="1 2 4" WORLD=8 CONFIG=C4 STEPS=60 bash tools/gpu_host_probe.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
WORLD=${WORLD:-8}; CONFIG=${CONFIG:-C4}; STEPS=${STEPS:-60}
: > gpurun_out/host_probe.jsonl
for b in ${BATCHES:-1 2 4}; do
  streams=4; [ "$b" -gt 2 ] && streams=$((2 * b))
  port=$((23000 + RANDOM % 5000))
  SHMCOMM_TIMEOUT_MS=60000 GPU_MAX_HW_QUEUES=8 SHMCOMM_REQUIRE_ASYNC=1 \
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $WORLD \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $WORLD --steps $STEPS \
    --warmup 4 --backend gloo --comm-lib tests/shmcomm/libshmcomm.so --driver native \
    --config $CONFIG --no-display --clock-warm-s 0 --batch $b --streams $streams \
    > gpurun_out/host_probe_b$b.json 2> gpurun_out/host_probe_b$b.log
  rc=$?; echo "batch $b rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python - "$b" <<'PY' >> gpurun_out/host_probe.jsonl
import json, sys
b = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/host_probe_b{b}.json") if l.startswith("{")][-1])
print(json.dumps({"batch": int(b), "world": d["n_gpus"], "config": d["config"]["workload"][:3],
                  "streams": d["config"]["streams"], "lag": d["config"]["lag"],
                  "driver_host_us_per_frame": d["driver_host_us_per_frame"],
                  "driver_enqueue_us_per_frame": d.get("driver_enqueue_us_per_frame"),
                  "ms_per_step": d["ms_per_step"], "frame_verified": d["frame_verified"]}))
PY
  tail -1 gpurun_out/host_probe.jsonl
done
exit 0
