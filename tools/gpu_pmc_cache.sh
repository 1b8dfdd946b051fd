#!/bin/bash
# Cache-level PMC passes over one bench command (MI355X_MICROARCH.md "rocprofv3 PMC": one
# counter group per run, --kernel-trace only, the program itself right after --):
#   p1  L2:  TCC_HIT / TCC_MISS / TCC_REQ / TCC_EA0_RDREQ (4 TCC slots)
#   p2  L1:  TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES / TCP_TCC_READ_REQ_LATENCY /
#            TCP_PENDING_STALL_CYCLES (4 TCP slots)
# then tools/pmc_cache_summary.py -> gpurun_out/pmc_cache_<tag>.json.
# usage: tools/gpu_pmc_cache.sh <tag> [bench args]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-c2}; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcc_$TAG
ARGS=${*:---steps 20 --warmup 5 --profile-only}
mkdir -p $OUT
cd /tmp
i=0
for C in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum" \
         "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  rm -rf $OUT/p$i
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc cache pass $i ($C) rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/p$i.log; exit $rc; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_cache_summary.py $OUT $GRAFT_REPO_ROOT/gpurun_out/pmc_cache_$TAG.json "$ARGS" \
  > $GRAFT_REPO_ROOT/gpurun_out/pmc_cache_$TAG.txt
rc=$?; cat $GRAFT_REPO_ROOT/gpurun_out/pmc_cache_$TAG.txt; rm -rf $OUT; exit $rc
