#!/bin/bash
# Single-call sdf_render_frames (one camera) under the frames kernel's
# measurement overrides (frames.cpp SDF3D_FRAMES_*): C3 exact
# -> gpurun_out/frames1_env.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/frames1_env.jsonl
for env in "X=0" "SDF3D_FRAMES_SCHEDULE=static" "SDF3D_FRAMES_QUEUES=32" "SDF3D_FRAMES_CHUNK=1" "SDF3D_FRAMES_CHUNK=8" "SDF3D_FRAMES_QUEUES=1 SDF3D_FRAMES_CHUNK=8"; do
  out=$(env $env timeout -k 10 200 python tools/single_call_probe.py --config ${CFG:-C3} --precision exact --rounds 3 2>>gpurun_out/sc.log) || exit 1
  echo "{\"env\": \"$env\", \"result\": $out}" >> gpurun_out/frames1_env.jsonl
done
cat gpurun_out/frames1_env.jsonl
