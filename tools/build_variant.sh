#!/bin/bash
# Tuning / diagnostic builds: every source with extra -D knobs (they may change shared
# layouts, e.g. SACMI_DIAG_PHASES the timeline words), as sacmi/libsacmi_<name>.so
# (select with SACMI_LIB_PATH).
#   tools/build_variant.sh <name> "-DSACMI_FWD_KS=2 ..."
set -e
PKG=$(cd "$(dirname "$0")/../humanoid-walking-with-sac_amd" && pwd)
name=$1; shift
mkdir -p "$PKG/build"
objs=""
for src in sacmi kernels replay per; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
    -fno-gpu-rdc $1 -c "$PKG/csrc/$src.hip" -o "$PKG/build/${src}_$name.o" &
  objs="$objs $PKG/build/${src}_$name.o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$PKG/sacmi/libsacmi_$name.so" $objs
echo "$PKG/sacmi/libsacmi_$name.so"
