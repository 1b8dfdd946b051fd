#!/bin/bash
# Per-phase breakdown (tools/phase_dump.py) of several diagnostic builds
# (sacmi/libsacmi_<name>.so, each from tools/build_variant.sh with -DSACMI_DIAG_PHASES).
#   VARIANTS="phases noload" CONFIG=2 bash tools/gpu_phase_variants.sh
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-phv}
mkdir -p $O
C=${CONFIG:-2}
for v in ${VARIANTS:-phases}; do
  SACMI_DIAG_DUMP=$O/dump_$v.bin SACMI_LIB_PATH=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi/libsacmi_$v.so \
    timeout -k 10 200 python3 tools/timeline_dump.py --config $C --n 4 > $O/tl_${v}_c$C.txt 2>&1 || { tail $O/tl_${v}_c$C.txt; exit 1; }
  python3 tools/phase_dump.py $O/dump_$v.bin ${SLOW:-0} > $O/phases_${v}_c$C.txt || exit 1
  rm -f $O/dump_$v.bin
  echo "== $v"; cat $O/phases_${v}_c$C.txt; tail -1 $O/tl_${v}_c$C.txt
done
