cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out/pp
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in peer peer_plain decode; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pp/$m -o $m -- python3 $R/tools/root_probe.py --world 8 --shares 2:7 --frames 400 --only $m > $R/gpurun_out/pp/$m.json 2>> $R/gpurun_out/pp/log.txt || { echo "$m rc=$?"; exit 1; }
done
find $R/gpurun_out/pp -name '*stats.csv' | head -20
