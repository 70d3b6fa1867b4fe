#!/bin/bash
# Round 6: EPA LDS slots per workgroup (native collide): 4 / 8 (default) / 16, steady window
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
NP="--no-cpu-baseline --no-other-solver --ccd native"
for v in 8 4 16 8; do
  L=$R/lerobot-mujoco-sim2real_amd/csrc/libsoarm_sim.so
  [ $v != 8 ] && L=$R/tools/_abr6/lib_slots$v.so
  SOARM_SIM_LIB=$L timeout -k 10 300 python bench.py $NP > $O/r06i_slots$v.json 2>> $O/r06i.err || exit $?
  python -c "
import json; d=json.loads(open('$O/r06i_slots$v.json').read().strip().splitlines()[-1])
print('slots $v', round(d['value']), {k: round(x, 4) for k, x in d['roofline']['kernel_ms_per_step'].items()})"
done
