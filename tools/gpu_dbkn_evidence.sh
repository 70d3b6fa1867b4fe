#!/bin/bash
# mpc_dbkn evidence: bench line with the CPU baseline, rocprofv3 kernel trace and PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config mpc_dbkn --steps 30 --warmup 5 --cpu-seconds 8 > $O/bench_mpc_dbkn.json 2> $O/bench_mpc_dbkn.err || exit $?
cd /tmp
P=$O/prof_r04_mpc_dbkn
KRE="k_substep|k_collide|k_step|k_geom|k_mpc_step|k_bias|k_bilinear"
NP="--steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-steady --no-other-solver"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $P -o trace -- python3 $R/bench.py --config mpc_dbkn --no-cpu-baseline > $O/bench_mpc_dbkn_traced.json || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $P -o pmc_fetch -- python3 $R/bench.py --config mpc_dbkn $NP || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $P -o pmc_write -- python3 $R/bench.py --config mpc_dbkn $NP || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$KRE" -f csv -d $P -o pmc_sq -- python3 $R/bench.py --config mpc_dbkn $NP || exit $?
echo evidence-ok
