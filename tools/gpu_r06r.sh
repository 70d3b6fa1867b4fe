#!/bin/bash
# Round 6: native k_collide with 8 / 16 / 24 EPA polytope slots in LDS per workgroup (bench A/B, bit identity)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
NP="--no-cpu-baseline --no-other-solver --ccd native"
for v in base s16 s24; do
  if [ $v = base ]; then L=""; else L="SOARM_SIM_LIB=$R/tools/_abr6/lib_$v.so"; fi
  env $L CCD=native timeout -k 10 300 python tools/ab_state.py n$v 60 > $O/r06r_ab_$v.log 2>&1 || exit $?
  env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06r_drv_$v.json 2>> $O/r06r_bench.err || exit $?
  env $L timeout -k 10 300 python bench.py $NP > $O/r06r_st_$v.json 2>> $O/r06r_bench.err || exit $?
done
python - <<'PY'
import json, glob
import numpy as np
a = np.load('gpurun_out/abstate_nbase.npz')
for v in ('s16', 's24'):
    b = np.load(f'gpurun_out/abstate_n{v}.npz')
    print(v, 'bit-identical to base:', all(np.array_equal(a[k], b[k]) for k in ('obs', 'qpos', 'qvel')))
for f in sorted(glob.glob("gpurun_out/r06r_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
