#!/bin/bash
# Bench lines (config CONFIG, default 2) of several library builds on one box, alternating:
# LIBS="fp32 main x6e1" (sacmi/libsacmi_<name>.so from tools/build_variant.sh; main = the
# library build), REPS rounds.  usage: LIBS="fp32 main" TAG=r6b bash tools/gpu_libs_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-libs}
mkdir -p $O
for r in $(seq 1 ${REPS:-1}); do
  for v in ${LIBS:-main}; do
    if [ "$v" = main ]; then L=""; else L="$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi/libsacmi_$v.so"; fi
    SACMI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline --config ${CONFIG:-2} \
      ${BENCH_ARGS:-} > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail $O/${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${v}_$r.json')); r=d.get('roofline') or {}
print('$v', d['value'], d['ms_per_step'], r.get('frac'), {k: v for k, v in (r.get('sites_us') or {}).items()})"
  done
done
