#!/bin/bash
# phase stamps of the config-2 chain: staged core vs register-direct core (same diag build)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4e}
mkdir -p $O
for st in 1 0; do
  SACMI_STAGED=$st SACMI_DIAG_DUMP=$O/dump_$st.bin SACMI_LIB_PATH=$GRAFT_REPO_ROOT/humanoid-walking-with-sac_amd/sacmi/libsacmi_phases.so \
    timeout -k 10 200 python3 tools/timeline_dump.py --config 2 --n 4 > $O/tl_stg$st.txt 2>&1 || { tail $O/tl_stg$st.txt; exit 1; }
  python3 tools/phase_dump.py $O/dump_$st.bin 3 > $O/phases_stg$st.txt || exit 1
  rm -f $O/dump_$st.bin
  echo "== staged=$st"; grep -v "^  slow" $O/phases_stg$st.txt; tail -1 $O/tl_stg$st.txt
done
