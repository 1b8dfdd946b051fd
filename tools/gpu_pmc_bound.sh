#!/bin/bash
# What bounds a kernel: five PMC passes over one bench command (MI355X_MICROARCH.md
# "rocprofv3 PMC": one counter group per run, --kernel-trace only, the program itself right
# after --; at most 8 SQ / 4 TCC / 4 TCP counters a pass):
#   p1  wave-time split   SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
#                         SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE
#   p2  instruction mix   SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
#                         SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA
#   p3  LDS / VMEM time   SQ_LEVEL_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR
#                         + TCP_TCR_TCP_STALL_CYCLES TCP_WRITE_TAGCONFLICT_STALL_CYCLES
#                           TCP_PENDING_STALL_CYCLES TCP_TCC_WRITE_REQ_LATENCY (TCP sums)
#   p4  fabric requests   TCC_EA0_RDREQ TCC_EA0_RDREQ_LEVEL TCC_EA0_WRREQ TCC_EA0_WRREQ_LEVEL
#                         + TCP_TCC_WRITE_REQ TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY (sums)
#   p5  memory side       TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM TCC_EA0_WRREQ_STALL TCC_TAG_STALL (sums)
# then tools/pmc_bound_summary.py -> gpurun_out/pmc_bound_<tag>.json.
# usage: tools/gpu_pmc_bound.sh <tag> [bench args]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-c5}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcb_$TAG
ARGS=${*:---config 5 --steps 20 --warmup 5 --profile-only}
mkdir -p $OUT
cd /tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_LEVEL_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR TCP_TCR_TCP_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_LATENCY_sum" \
         "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
         "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum"; do
  i=$((i+1))
  rm -rf $OUT/p$i
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc bound pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/p$i.log; exit $rc; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_bound_summary.py $OUT $GRAFT_REPO_ROOT/gpurun_out/pmc_bound_$TAG.json "$ARGS" \
  > $GRAFT_REPO_ROOT/gpurun_out/pmc_bound_$TAG.txt
rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/pmc_bound_$TAG.txt; rm -rf $OUT; exit $rc
