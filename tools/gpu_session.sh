#!/bin/bash
# One parameterised GPU session (replaces round 4's one-off gpu_r4*.sh scripts).  Steps, in
# order, each with its own time limit; the first failure ends the session:
#   tests    pytest -m gpu (PYTEST_ARGS, PYTEST_K = a -k expression; SACMI_GRAD_TABLE -> $O/grad_table.jsonl)
#   smoke    __graft_entry__.smoke()
#   ab       alternating bench lines without / with AB_ENV (BENCH_ARGS), AB_REPS pairs
#   configs  bench lines of CONFIGS (default "2 3 5"), BENCH_ARGS appended
#   dp8      the data-parallel sequence at a simulated world of 8, both optimizer forms
#   dpab     the data-parallel bench at one rank over real RCCL with the phase sequence forced
#            (SACMI_DP_PHASES_AT_WORLD1): the line's form and the other one (dp_form_ab);
#            dpabr the same with the sharded form as the line's
#   driver   `python3 bench.py` with no arguments (the driver's round-end line)
#   pmcb     the bound-analysis PMC passes (tools/gpu_pmc_bound.sh) of CONFIGS_PMCB ("5 3")
#   prof     the round's profile set (tools/gpu_profile.sh: PMC passes of CONFIGS, the
#            rocprofv3 kernel-trace summary of the driver's config-2 command)
# usage: STEPS="tests ab" AB_ENV="SACMI_NO_GRAPH=1" TAG=r6b bash tools/gpu_session.sh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-session}
mkdir -p $O
B="python3 bench.py --no-trainer-loop --no-cpu-baseline"
line() { python3 -c "
import json; d=json.load(open('$1')); r=d.get('roofline') or {}
print('$1', d['value'], d['ms_per_step'], r.get('frac'), {k: v for k, v in (r.get('sites_us') or {}).items() if 'L' in k or 'chain' in k})"; }
for step in ${STEPS:-tests smoke configs}; do
  case $step in
    tests)
      SACMI_GRAD_TABLE=$PWD/$O/grad_table.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 \
        --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
      rc=$?; tail -3 $O/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; } ;;
    ab)
      for r in $(seq 1 ${AB_REPS:-2}); do
        timeout -k 10 300 $B ${BENCH_ARGS:-} > $O/a$r.json 2> $O/a$r.err || { tail $O/a$r.err; exit 1; }
        timeout -k 10 300 env ${AB_ENV} $B ${BENCH_ARGS:-} > $O/b$r.json 2> $O/b$r.err || { tail $O/b$r.err; exit 1; }
      done
      for f in $O/a*.json $O/b*.json; do line $f; done ;;
    configs)
      for c in ${CONFIGS:-2 3 5}; do
        timeout -k 10 400 $B --config $c ${BENCH_ARGS:-} > $O/c$c.json 2> $O/c$c.err || { tail $O/c$c.err; exit 1; }
        line $O/c$c.json
      done ;;
    dp8)
      SACMI_DP_SHARD=1 SACMI_DP_LOOPBACK_ONE_RANK=1 timeout -k 10 300 $B --force-dp --dp-sim-world 8 --steps 20 \
        > $O/dp8_shard.json 2> $O/dp8_shard.err || { tail $O/dp8_shard.err; exit 1; }
      SACMI_DP_SHARD=0 SACMI_DP_LOOPBACK_ONE_RANK=1 timeout -k 10 300 $B --force-dp --dp-sim-world 8 --steps 20 > $O/dp8_ar.json 2> $O/dp8_ar.err || { tail $O/dp8_ar.err; exit 1; }
      line $O/dp8_shard.json; line $O/dp8_ar.json
      python3 -c "import json; [print(f, json.load(open(f))['dp_form_ab']) for f in ('$O/dp8_shard.json', '$O/dp8_ar.json')]" ;;
    dpab|dpabr)
      # dpabr: the same with the sharded form as the line's (the all-reduce form the other leg)
      f=dp1_ab; e=""; if [ $step = dpabr ]; then f=dp1_abr; e="SACMI_DP_SHARD=1"; fi
      env $e SACMI_DP_PHASES_AT_WORLD1=1 timeout -k 10 300 $B --force-dp --steps 20 > $O/$f.json 2> $O/$f.err \
        || { tail $O/$f.err; exit 1; }
      line $O/$f.json
      python3 -c "import json; d=json.load(open('$O/$f.json')); print(d['dp_optimizer_step'], d['replicas_bitwise_equal'], d['dp_form_ab'])" ;;
    driver)   # the driver's own round-end command (defaults: trainer loop and cpu_baseline included)
      timeout -k 10 600 python3 bench.py > $O/driver_bench.json 2> $O/driver_bench.err || { tail $O/driver_bench.err; exit 1; }
      line $O/driver_bench.json ;;
    pmcb)
      for c in ${CONFIGS_PMCB:-5 3}; do
        bash tools/gpu_pmc_bound.sh c$c --config $c --steps 20 --warmup 5 --profile-only || exit 1
        cp gpurun_out/pmc_bound_c$c.json gpurun_out/pmc_bound_c$c.txt $O/ || exit 1
      done ;;
    prof)
      TAG=${TAG:-session} bash tools/gpu_profile.sh || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
