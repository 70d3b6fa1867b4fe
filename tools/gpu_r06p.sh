#!/bin/bash
# Round 6 diagnostic (timings only): where the table-cube lane's time goes -- only pair 27 runs
# (SOARM_DIAG_SKIP="~27"), stopped after the midphase (stage 1), after the narrowphase and its
# contact stores (stage 2: no mask atomics), or complete; and the empty grid
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
NP="--no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5"
run() {  # tag skip stage
  SOARM_SIM_LIB=$R/tools/_mbr6/lib_diag.so SOARM_DIAG_SKIP=$2 SOARM_DIAG_STAGE=$3 timeout -k 10 300 python bench.py $NP > $O/r06p_$1.json 2>> $O/r06p.err || exit $?
  python -c "
import json; d=json.loads(open('$O/r06p_$1.json').read().strip().splitlines()[-1])
print('$1 skip [$2] stage $3', 'collide us/launch', round(d['roofline']['kernel_ms_per_step']['collide'] * 100, 2))"
}
run empty "~" 0
run s1 "~27" 1
run s2 "~27" 2
run s3 "~27" 0
run all1 "" 1
run all2 "" 2
run all3 "" 0
