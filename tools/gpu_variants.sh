#!/bin/bash
# Timeline of the config-2 update for each tuning / timing-experiment build
# (sacmi/libsacmi_<name>.so from tools/build_variant.sh; "main" = the library build).
# usage: VARIANTS="main nomfma" tools/gpu_variants.sh   Every GPU step is time-limited;
# the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-var}
mkdir -p $O
for v in ${VARIANTS:-main}; do
  if [ "$v" = main ]; then L=""; else L="$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi/libsacmi_$v.so"; fi
  SACMI_LIB_PATH=$L timeout -k 10 200 python3 tools/timeline_dump.py --config ${CONFIG:-2} > $O/tl_$v.txt 2>&1 || { tail $O/tl_$v.txt; exit 1; }
  echo "== $v"; tail -1 $O/tl_$v.txt
done
