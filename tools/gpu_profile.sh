#!/bin/bash
# Profile pass of one round: the three PMC counter passes (tools/gpu_pmc.sh) for configs
# 2, 3 and 5, then a rocprofv3 --kernel-trace --stats run of the driver's bench command
# (its JSON line and the per-level summary agree on the GEMM-level mean).  Every GPU step
# has its own time limit (inside gpu_pmc.sh too); the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-prof}
mkdir -p $O
for c in ${CONFIGS:-2 3 5}; do
  bash tools/gpu_pmc.sh c$c --config $c --steps 20 --warmup 5 --profile-only || exit 1
  cp gpurun_out/pmc_c$c.json $O/ || exit 1
  rm -rf gpurun_out/pmc_c$c                       # raw counter CSVs (tens of MB)
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-trainer-loop \
  > $O/trace_bench.json 2> $O/trace_bench.err || { tail -20 $O/trace_bench.err; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/rocprof_kgemm.py $(ls $O/trace/*kernel_stats.csv | head -1) > $O/rocprof_summary_config2.txt
cp $(ls $O/trace/*kernel_stats.csv | head -1) $O/kernel_stats_config2.csv
rm -rf $O/trace                                   # the per-dispatch trace (tens of MB)
tail -2 $O/rocprof_summary_config2.txt
