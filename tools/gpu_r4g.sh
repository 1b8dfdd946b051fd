#!/bin/bash
# staged core x L2 residency of the activations (plain stores + row-affine XCD grid)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4g}
mkdir -p $O
L=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi
B="timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline"
run() { name=$1; shift; env "$@" $B > $O/b_$name.json 2> $O/b_$name.err || { tail $O/b_$name.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/b_$name.json')); r=d.get('roofline') or {}; print('$name', d['value'], d['ms_per_step'], r.get('frac'), r.get('sites_us'))"; }
run stg SACMI_STAGED=1
run stg_wt0_gr8 SACMI_STAGED=1 SACMI_LIB_PATH=$L/libsacmi_wt0.so SACMI_XCD_GR=8
run stg_wt0 SACMI_STAGED=1 SACMI_LIB_PATH=$L/libsacmi_wt0.so
run stg_gr1 SACMI_STAGED=1 SACMI_XCD_GR=1
for st in 0 1; do
  SACMI_STAGED=$st SACMI_EXP_DUP_LEVELS=1 timeout -k 10 200 python3 tools/timeline_dump.py --config 2 --n 4 > $O/tl_dup_stg$st.txt 2>&1 || { tail $O/tl_dup_stg$st.txt; exit 1; }
  echo "== dup staged=$st"; cat $O/tl_dup_stg$st.txt
done
