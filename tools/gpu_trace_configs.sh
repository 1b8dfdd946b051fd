#!/bin/bash
# rocprofv3 --kernel-trace --stats of the config-3 and config-5 bench commands (per-kernel
# means + the GEMM-level mean, tools/rocprof_kgemm.py), beside the line each run printed.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-trace_cfg}
mkdir -p $O
cd /tmp
for c in ${CONFIGS:-3 5}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --no-trainer-loop \
    > $O/bench_config$c.json 2> $O/bench_config$c.err || { tail -20 $O/bench_config$c.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/tools/rocprof_kgemm.py $(ls $O/t$c/*kernel_stats.csv | head -1) > $O/rocprof_summary_config$c.txt
  rm -rf $O/t$c
  tail -1 $O/rocprof_summary_config$c.txt
done
