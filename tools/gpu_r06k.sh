#!/bin/bash
# Round 6: k_collide dispatch order A/B -- box-box pairs (the table under the cube) first
# (tools/_abr6/lib_bbfirst.so) against the current order; driver and steady windows, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
NP="--no-cpu-baseline --no-other-solver"
for i in 1 2; do
  for v in cur bb; do
    L=$R/lerobot-mujoco-sim2real_amd/csrc/libsoarm_sim.so
    [ $v = bb ] && L=$R/tools/_abr6/lib_bbfirst.so
    SOARM_SIM_LIB=$L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06k_drv_$v$i.json 2>> $O/r06k.err || exit $?
    SOARM_SIM_LIB=$L timeout -k 10 300 python bench.py $NP > $O/r06k_st_$v$i.json 2>> $O/r06k.err || exit $?
    python -c "
import json
for w in ('drv','st'):
    d=json.loads(open('$O/r06k_'+w+'_$v$i.json').read().strip().splitlines()[-1])
    print('$v$i', w, round(d['value']), {k: round(x, 4) for k, x in d['roofline']['kernel_ms_per_step'].items()})"
  done
done
