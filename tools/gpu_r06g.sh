#!/bin/bash
# Round 6 diagnostic (timings only): k_collide launched with only the first k rows of its dispatch
# order (SOARM_DIAG_ROWS, diagnostic build tools/_abr6/lib_diag.so): how the launch time grows with
# the grid, i.e. how much of it is the grid's own size
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
NP="--no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5"
for k in 1 14 27 50 72 86; do
  SOARM_SIM_LIB=$R/tools/_abr6/lib_diag.so SOARM_DIAG_ROWS=$k timeout -k 10 300 python bench.py $NP > $O/r06g_rows$k.json 2>> $O/r06g.err || exit $?
done
python - <<'PY'
import json
for k in (1, 14, 27, 50, 72, 86):
    d = json.loads(open(f"gpurun_out/r06g_rows{k}.json").read().strip().splitlines()[-1])
    print(k, "collide us/launch", round(d["roofline"]["kernel_ms_per_step"]["collide"] * 100, 2))
PY
