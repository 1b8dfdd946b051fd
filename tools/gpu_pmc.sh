#!/bin/bash
# HBM traffic counters for the bench command: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (each with --kernel-trace only, MI355X_MICROARCH.md "rocprofv3 PMC").
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
ARGS=${PMC_ARGS:---steps 100 --warmup 20 --fill 200000 --no-cpu-baseline --no-roofline --no-trainer-loop}
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf $OUT/pmc_$C
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$C -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/pmc_$C.log; exit $rc; }
done
find $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE -name "*.csv" | head
