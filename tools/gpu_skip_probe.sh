cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out; out=gpurun_out/skip_probe.jsonl; : > $out
export GPU_MAX_HW_QUEUES=8
for rep in 1 2 3; do
  for sk in "" "--skip-root-part"; do
    timeout -k 10 120 python tools/root_probe.py --world 8 --shares 2:7 --frames 400 --only decode $sk | sed "s/^{/{\"skip\": \"$sk\", /" >> $out || exit 1
  done
done
for sk in "" "--skip-root-part"; do
  timeout -k 10 120 python tools/root_probe.py --world 8 --shares 2:7 --frames 400 --only root $sk | sed "s/^{/{\"skip\": \"$sk\", /" >> $out || exit 1
done
cat $out
