#!/bin/bash
# Round 6: k_collide workgroup size 128 / 256 (default) / 512 envs -- bit identity and bench A/B (MPR)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
NP="--no-cpu-baseline --no-other-solver"
for v in b256 b512 b128; do
  if [ $v = b256 ]; then L=""; else L="SOARM_SIM_LIB=$R/tools/_abr6/lib_$v.so"; fi
  env $L timeout -k 10 300 python tools/ab_state.py $v 60 > $O/r06w_ab_$v.log 2>&1 || exit $?
  env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06w_drv_$v.json 2>> $O/r06w_bench.err || exit $?
  env $L timeout -k 10 300 python bench.py $NP > $O/r06w_st_$v.json 2>> $O/r06w_bench.err || exit $?
done
python - <<'PY'
import json, glob
import numpy as np
a = np.load('gpurun_out/abstate_b256.npz')
for v in ('b512', 'b128'):
    b = np.load(f'gpurun_out/abstate_{v}.npz')
    print(v, 'bit-identical to b256:', all(np.array_equal(a[k], b[k]) for k in ('obs', 'qpos', 'qvel')))
for f in sorted(glob.glob("gpurun_out/r06w_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
