#!/bin/bash
# Tuning builds: kernels.hip with extra -D knobs, linked against the main build's other
# objects, as sacmi/libsacmi_<name>.so (select with SACMI_LIB_PATH).
#   tools/build_variant.sh <name> "-DSACMI_FWD_KS=2 ..."
set -e
PKG=$(cd "$(dirname "$0")/../humanoid-walking-with-sac_amd" && pwd)
name=$1; shift
make -s -C "$PKG" >/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result \
  -fno-gpu-rdc $1 -c "$PKG/csrc/kernels.hip" -o "$PKG/build/kernels_$name.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$PKG/sacmi/libsacmi_$name.so" \
  "$PKG/build/sacmi.o" "$PKG/build/kernels_$name.o" "$PKG/build/replay.o" "$PKG/build/per.o"
echo "$PKG/sacmi/libsacmi_$name.so"
