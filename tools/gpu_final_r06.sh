#!/bin/bash
# Round-6 evidence (two GPU calls: PART=bench, PART=prof) (each step time-limited; a failure ends the script):
# tests + smoke, the bench lines of every config, rocprofv3 kernel-trace summaries and PMC passes of
# the headline (PGS), its Newton twin and the DBKN MPC, and the phase profile of the contact substep.
#   usage: tools/gpu_final_r06.sh [tag] [--no-tests]; PART=bench (tests, smoke, bench lines) or
#   PART=prof (the rocprofv3 passes) runs one half (two GPU calls within the call limit)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 $lim "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PART=${PART:-all}
if [ "$PART" != "prof" ]; then
if [ "$2" != "--no-tests" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -2 $O/pytest_gpu.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
step bench_contact 600 python bench.py > $O/bench_contact.json 2> $O/bench_contact.err
step bench_driver 300 python bench.py --steps 20 --warmup 5 > $O/bench_contact_steps20_warmup5.json 2> $O/bench_contact_drv.err
step bench_contact_native 600 python bench.py --ccd native --no-cpu-baseline > $O/bench_contact_native.json 2> $O/bench_contact_native.err
step bench_contact_newton 600 python bench.py --solver newton --no-cpu-baseline > $O/bench_contact_newton.json 2> $O/bench_contact_newton.err
step bench_nocontact 300 python bench.py --config nocontact --steps 200 --warmup 20 --cpu-seconds 8 > $O/bench_nocontact.json 2> $O/bench_nocontact.err
step bench_dr 600 python bench.py --config dr --steps 50 --warmup 5 --cpu-seconds 8 > $O/bench_dr.json 2> $O/bench_dr.err
step bench_rollout 600 python bench.py --config rollout --steps 100 --warmup 5 --cpu-seconds 8 > $O/bench_rollout.json 2> $O/bench_rollout.err
step bench_mpc 600 python bench.py --config mpc --cpu-seconds 8 > $O/bench_mpc.json 2> $O/bench_mpc.err
step bench_mpc_dbkn 600 python bench.py --config mpc_dbkn --steps 30 --warmup 5 --cpu-seconds 8 > $O/bench_mpc_dbkn.json 2> $O/bench_mpc_dbkn.err
step bench_plumbing 300 python bench.py --config plumbing > $O/bench_plumbing.json 2> $O/bench_plumbing.err
step bench_rollout_nccl 600 python bench.py --config rollout --steps 100 --warmup 5 --dist-backend nccl --no-cpu-baseline > $O/bench_rollout_nccl.json 2> $O/bench_rollout_nccl.err
step bench_contact_nccl 600 python bench.py --dist-backend nccl --no-cpu-baseline --no-other-solver > $O/bench_contact_nccl.json 2> $O/bench_contact_nccl.err
step bench_gloo2 300 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline --no-steady --no-other-solver > $O/bench_gloo2.json 2> $O/bench_gloo2.err
# (the phase profile needs the diagnostic build in tools/_prof, which .gpurunignore keeps off the
#  box by default: SKIP_PHASE=1 when it is not there)
if [ -n "$WITH_PHASE" ]; then
  step phase_pgs 300 env EVERY=20 PROF_LIB=tools/_rsprof/libsoarm_sim_prof.so python tools/phase_prof.py 120 > $O/phase_pgs.log 2>&1
fi
fi
if [ "$PART" = "bench" ]; then echo final-ok; exit 0; fi
KRE="k_substep|k_collide|k_step|k_geom|k_mpc_step|k_bias|k_bilinear"
cd /tmp
for SPEC in contact:contact: contact_native:contact:--ccd_native contact_newton:contact:--solver_newton mpc_dbkn:mpc_dbkn:; do
  IFS=: read TAGC C EXTRA <<< "$SPEC"
  EXTRA=${EXTRA//_/ }
  P=$O/prof_${TAG}_$TAGC
  step trace_$TAGC 600 rocprofv3 --kernel-trace --stats -f csv -d $P -o trace -- python3 $R/bench.py --config $C $EXTRA --no-cpu-baseline > $O/bench_${TAGC}_traced.json
  NP="--steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-steady --no-other-solver"
  step pmc_fetch_$TAGC 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $P -o pmc_fetch -- python3 $R/bench.py --config $C $EXTRA $NP
  step pmc_write_$TAGC 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $P -o pmc_write -- python3 $R/bench.py --config $C $EXTRA $NP
  step pmc_sq_$TAGC 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$KRE" -f csv -d $P -o pmc_sq -- python3 $R/bench.py --config $C $EXTRA $NP
done
echo final-ok
