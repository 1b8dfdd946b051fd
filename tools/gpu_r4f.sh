#!/bin/bash
# config-2 A/B of L2-residency knobs: XCD grid (SACMI_XCD_GR), nt A-operand loads (nta build),
# plain epilogue stores (wt0 build)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4f}
mkdir -p $O
L=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi
B="timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline"
run() { name=$1; shift; env "$@" $B > $O/b_$name.json 2> $O/b_$name.err || { tail $O/b_$name.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/b_$name.json')); r=d.get('roofline') or {}; print('$name', d['value'], d['ms_per_step'], r.get('frac'))"; }
run base X=1
run gr1 SACMI_XCD_GR=1
run gr8 SACMI_XCD_GR=8
run nta SACMI_LIB_PATH=$L/libsacmi_nta.so
run nta_gr1 SACMI_LIB_PATH=$L/libsacmi_nta.so SACMI_XCD_GR=1
run wt0_gr1 SACMI_LIB_PATH=$L/libsacmi_wt0.so SACMI_XCD_GR=1
run wt0_gr8 SACMI_LIB_PATH=$L/libsacmi_wt0.so SACMI_XCD_GR=8
run wt0 SACMI_LIB_PATH=$L/libsacmi_wt0.so
run base2 X=1
