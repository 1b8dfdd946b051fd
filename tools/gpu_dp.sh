#!/bin/bash
# Data-parallel bench lines at world 1 (the forced DP path: RCCL all-reduces + captured
# phase graphs), config 2 (uniform shard), config 3 (prioritized shard, BASELINE configs[3]
# per GPU) and config 5 (BASELINE configs[4] per GPU, bf16).  Each GPU step has its own time limit; the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-dp}
mkdir -p $O
timeout -k 10 400 python3 bench.py --force-dp --steps 20 --warmup 5 > $O/dp_c2.json 2> $O/dp_c2.err || { tail -20 $O/dp_c2.err; exit 1; }
cut -c1-400 $O/dp_c2.json
timeout -k 10 400 python3 bench.py --force-dp --config 3 --steps 20 --warmup 5 > $O/dp_c3.json 2> $O/dp_c3.err || { tail -20 $O/dp_c3.err; exit 1; }
cut -c1-400 $O/dp_c3.json
timeout -k 10 400 python3 bench.py --force-dp --config 5 --steps 20 --warmup 5 > $O/dp_c5.json 2> $O/dp_c5.err || { tail -20 $O/dp_c5.err; exit 1; }
cut -c1-400 $O/dp_c5.json
