#!/bin/bash
# Round 6 diagnostic (timings only): which of the first k_collide rows makes the launch long
# (SOARM_DIAG_ROWS: first k rows of the dispatch order; SOARM_DIAG_SKIP: pairs that return at once)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
NP="--no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5"
run() {  # tag rows skip
  SOARM_SIM_LIB=$R/tools/_abr6/lib_diag.so SOARM_DIAG_ROWS=$2 SOARM_DIAG_SKIP=$3 timeout -k 10 300 python bench.py $NP > $O/r06j_$1.json 2>> $O/r06j.err || exit $?
  python -c "
import json; d=json.loads(open('$O/r06j_$1.json').read().strip().splitlines()[-1])
print('$1 rows $2 skip [$3]', 'collide us/launch', round(d['roofline']['kernel_ms_per_step']['collide'] * 100, 2))"
}
run r1 1 ""
run r2 2 ""
run r13 13 ""
run r14 14 ""
run r14no27 14 "27"
run r86no27 86 "27"
run only27 86 "~27"
