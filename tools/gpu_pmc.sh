#!/bin/bash
# PMC passes over one bench command (MI355X_MICROARCH.md "rocprofv3 PMC": one counter
# group per run, --kernel-trace only, the program itself right after --):
#   FETCH_SIZE | WRITE_SIZE | MFMA busy + MFMA ops + GUI active
# then tools/pmc_summary.py -> $OUT/pmc_<tag>.json.  usage: tools/gpu_pmc.sh <tag> [bench args]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-c2}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
ARGS=${*:---steps 20 --warmup 5 --profile-only}
mkdir -p $OUT
cd /tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf $OUT/p$i
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc pass $i ($C) rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/p$i.log; exit $rc; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.json "$ARGS"
