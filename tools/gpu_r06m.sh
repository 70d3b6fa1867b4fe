#!/bin/bash
# Round 6 experiment: the RS kernel built for two waves per SIMD (spills) at 4096 envs (one wave per
# SIMD: the spills' cost alone) and 8192 (two per SIMD), against the default build
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
NP="--no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5"
run() {
  timeout -k 10 300 "$@" > $O/r06m.json 2>> $O/r06m.err || exit $?
  python -c "
import json; d=json.loads(open('$O/r06m.json').read().strip().splitlines()[-1])
print(round(d['value']), {k: round(x, 4) for k, x in d['roofline']['kernel_ms_per_step'].items()})"
}
echo "rs 4096"; run python bench.py $NP
echo "rs2 4096"; SOARM_SIM_LIB=$R/tools/_mbr6/lib_rs2.so SOARM_RS2=1 run python bench.py $NP
echo "rs2 8192 (dr)"; SOARM_SIM_LIB=$R/tools/_mbr6/lib_rs2.so SOARM_RS2=1 run python bench.py $NP --config dr
echo "quad 8192 (dr)"; run python bench.py $NP --config dr
