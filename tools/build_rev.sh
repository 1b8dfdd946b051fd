#!/bin/bash
# A/B builds: the library of git revision <rev> as sacmi/libsacmi_<name>.so of this tree
# (select with SACMI_LIB_PATH; tools/gpu_variants.sh runs several in one GPU call).
#   tools/build_rev.sh <rev> <name> ["-DKNOB=..."]
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
rev=$1; name=$2; flags=${3:-}
tmp=$(mktemp -d /tmp/sacmi_rev.XXXXXX)
git -C "$REPO" archive "$rev" humanoid-walking-with-sac_amd include | tar -x -C "$tmp"
PKG=$tmp/humanoid-walking-with-sac_amd
objs=""
for src in sacmi kernels replay per; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
    -fno-gpu-rdc $flags -c "$PKG/csrc/$src.hip" -o "$tmp/$src.o" &
  objs="$objs $tmp/$src.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$REPO/humanoid-walking-with-sac_amd/sacmi/libsacmi_$name.so" $objs
rm -rf "$tmp"
echo "$REPO/humanoid-walking-with-sac_amd/sacmi/libsacmi_$name.so"
