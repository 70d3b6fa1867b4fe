#!/bin/bash
# Round 6: the soft-reset fix (check_state's return) against the build before it -- bench A/B pairs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
P=$R/tools/_abr6/lib_prefix.so
NP="--no-cpu-baseline --no-other-solver"
for v in fix pre fix2 pre2; do
  if [ ${v%2} = fix ]; then L=""; else L="SOARM_SIM_LIB=$P"; fi
  env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06ac_drv_$v.json 2>> $O/r06ac_bench.err || exit $?
  env $L timeout -k 10 300 python bench.py $NP > $O/r06ac_st_$v.json 2>> $O/r06ac_bench.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06ac_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items() if v})
PY
