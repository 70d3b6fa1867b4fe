#!/bin/bash
# Round 6: hull cube-map resolution HULL_LUT_K 96 (default) / 48 / 64 with the one-trip climbing records -- bit identity and bench A/B (MPR)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
NP="--no-cpu-baseline --no-other-solver"
for v in k96 k48 k64; do
  if [ $v = k96 ]; then L=""; else L="SOARM_SIM_LIB=$R/tools/_abr6/lib_$v.so"; fi
  env $L timeout -k 10 300 python tools/ab_state.py $v 60 > $O/r06x_ab_$v.log 2>&1 || exit $?
  env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06x_drv_$v.json 2>> $O/r06x_bench.err || exit $?
  env $L timeout -k 10 300 python bench.py $NP > $O/r06x_st_$v.json 2>> $O/r06x_bench.err || exit $?
done
python - <<'PY'
import json, glob
import numpy as np
a = np.load('gpurun_out/abstate_k96.npz')
for v in ('k48', 'k64'):
    b = np.load(f'gpurun_out/abstate_{v}.npz')
    print(v, 'bit-identical to k96:', all(np.array_equal(a[k], b[k]) for k in ('obs', 'qpos', 'qvel')))
for f in sorted(glob.glob("gpurun_out/r06x_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
