#!/bin/bash
# Per-phase breakdown of the GEMM levels in the real update chain (diagnostic build
# sacmi/libsacmi_phases.so from `tools/build_variant.sh phases -DSACMI_DIAG_PHASES`; LIB=<name>
# selects another diagnostic build, libsacmi_<name>.so).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-phases}
mkdir -p $O
SACMI_DIAG_DUMP=$O/dump_c${CONFIG:-2}.bin SACMI_LIB_PATH=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi/libsacmi_${LIB:-phases}.so \
  timeout -k 10 200 python3 tools/timeline_dump.py --config ${CONFIG:-2} --n 4 > $O/tl_c${CONFIG:-2}.txt 2>&1 || { tail $O/tl_c${CONFIG:-2}.txt; exit 1; }
python3 tools/phase_dump.py $O/dump_c${CONFIG:-2}.bin ${SLOW:-0} > $O/phases_c${CONFIG:-2}.txt && cat $O/phases_c${CONFIG:-2}.txt
rm -f $O/dump_c${CONFIG:-2}.bin
