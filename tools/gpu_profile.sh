#!/bin/bash
# One GPU session for the round's evidence: gpu tests, smoke, bench lines
# (contact with CPU baseline, nocontact, dr), the rocprofv3 kernel-trace
# summary of the bench command, and separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ instruction/wait counters) on the hot kernels.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 $lim "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then exit $rc; fi
}
timeout -k 10 900 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step bench_contact 600 python bench.py > $O/bench_contact.json 2> $O/bench_contact.err
cat $O/bench_contact.json
step bench_nocontact 300 python bench.py --config nocontact --steps 200 --warmup 20 --cpu-seconds 8 > $O/bench_nocontact.json 2> $O/bench_nocontact.err
step bench_dr 600 python bench.py --config dr --steps 50 --warmup 5 --cpu-seconds 8 > $O/bench_dr.json 2> $O/bench_dr.err
step bench_rollout 600 python bench.py --config rollout --steps 100 --warmup 5 --cpu-seconds 8 > $O/bench_rollout.json 2> $O/bench_rollout.err
cd /tmp
step kernel_trace 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$TAG -o trace -- python3 $R/bench.py --no-cpu-baseline > $O/bench_contact_traced.json
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_substep|k_collide|k_step|k_geom" -f csv -d $O/prof_$TAG -o pmc_fetch -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_substep|k_collide|k_step|k_geom" -f csv -d $O/prof_$TAG -o pmc_write -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile
step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_substep|k_collide|k_step|k_geom" -f csv -d $O/prof_$TAG -o pmc_sq -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile
ls -R $O/prof_$TAG | head -40
