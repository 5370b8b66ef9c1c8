#!/bin/bash
# Build libsdf3d.so of another git revision (for in-process A/B timing with
# tools/ab_kernel.py):  tools/build_variant.sh <rev> <name> [stats]
#   -> tools/_variants/libsdf3d_<name>.so   (with "stats": the -DSDF_STATS
#      debug library of tools/kernel_stats.py instead)
set -euo pipefail
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/sdfvar.XXXXXX)
git -C "$root" archive "$rev" sdf3d_amd include | tar -x -C "$tmp"
what=build_library; lib=libsdf3d.so
if [ "${3:-}" = stats ]; then what=build_stats_library; lib=libsdf3d_stats.so; fi
(cd "$tmp" && python -c "import sys; sys.path.insert(0, '.'); from sdf3d_amd import build; build.OBJ.mkdir(parents=True, exist_ok=True); build.LIB_DIR.mkdir(parents=True, exist_ok=True); build.write_rtc_sources(); build.$what(verbose=False)")
mkdir -p "$root/tools/_variants"
cp "$tmp/sdf3d_amd/lib/$lib" "$root/tools/_variants/libsdf3d_$name.so"
rm -rf "$tmp"
echo "tools/_variants/libsdf3d_$name.so"
