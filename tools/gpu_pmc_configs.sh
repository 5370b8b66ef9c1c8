cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in C4 C5 C2; do
  timeout -k 10 400 python tools/pmc_traffic.py --config $c --precision fast --out gpurun_out/pmc > gpurun_out/pmc_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; exit 1; }
  echo "pmc $c ok"
done
