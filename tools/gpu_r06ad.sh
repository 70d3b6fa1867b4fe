#!/bin/bash
# Round 6: the soft-reset fix in a second shape (status bits cleared around check_state, lib_fix2)
# against the build before the fix -- bench A/B pairs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
NP="--no-cpu-baseline --no-other-solver"
for v in pre fix2 pre_b fix2_b; do
  L="SOARM_SIM_LIB=$R/tools/_abr6/lib_${v%_b}.so"
  [ ${v%_b} = pre ] && L="SOARM_SIM_LIB=$R/tools/_abr6/lib_prefix.so"
  env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06ad_drv_$v.json 2>> $O/r06ad_bench.err || exit $?
  env $L timeout -k 10 300 python bench.py $NP > $O/r06ad_st_$v.json 2>> $O/r06ad_bench.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06ad_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items() if v})
PY
