#!/bin/bash
# Register / occupancy report of the fast render kernels from the compiler's
# kernel-resource-usage remarks:  tools/resource_usage.sh [grep pattern]
#   one line per kernel: name  SGPRs  VGPRs  scratch  waves/SIMD
root=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=fast-honor-pragmas -fno-slp-vectorize \
  -I "$root/sdf3d_amd/build" -c "$root/sdf3d_amd/csrc/render_fast.hip" -o /tmp/_ru.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n -e 's/.*remark: *//' -e 's/ \[-Rpass.*//p' |
  awk '/^Function Name:/ {if (n) print n, s, v, sc, o; n=$3} /^TotalSGPRs:/ {s=$2} /^VGPRs:/ {v=$2}
       /^ScratchSize/ {sc=$NF} /^Occupancy/ {o=$NF} END {if (n) print n, s, v, sc, o}' |
  c++filt | grep -e "${1:-.}"
