#!/bin/bash
# dedicated scalar-Adam workgroup: GPU tests, config-2 A/B, phase stamps
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
B="timeout -k 10 200 python3 bench.py --no-trainer-loop --no-cpu-baseline"
run() { name=$1; shift; env "$@" $B > $O/b_$name.json 2> $O/b_$name.err || { tail $O/b_$name.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/b_$name.json')); r=d.get('roofline') or {}; print('$name', d['value'], d['ms_per_step'], r.get('frac'))"; }
run awg X=1
run noawg SACMI_NO_ADAM_WG=1
run awg2 X=1
run noawg2 SACMI_NO_ADAM_WG=1
SACMI_DIAG_DUMP=$O/dump.bin SACMI_LIB_PATH=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi/libsacmi_phases.so \
  timeout -k 10 200 python3 tools/timeline_dump.py --config 2 --n 4 > $O/tl.txt 2>&1 || { tail $O/tl.txt; exit 1; }
python3 tools/phase_dump.py $O/dump.bin 2 > $O/phases.txt; rm -f $O/dump.bin; grep -v "^  slow" $O/phases.txt; tail -1 $O/tl.txt
bash tools/gpu_r4g.sh
