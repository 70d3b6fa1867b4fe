#!/bin/bash
# Round 6: per-lane LDS copy of the last cube-map cell record (k_collide, -DSOARM_SUPCACHE, EPA slots 4)
# against the default -- bit identity and bench A/B, both narrowphases
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
P=$R/tools/_abr6/lib_sc.so
for c in mpr native; do
  CCD=$c timeout -k 10 300 python tools/ab_state.py ${c}base 60 > $O/r06ab_ab.log 2>&1 || exit $?
  CCD=$c SOARM_SIM_LIB=$P timeout -k 10 300 python tools/ab_state.py ${c}sc 60 >> $O/r06ab_ab.log 2>&1 || exit $?
  python -c "
import numpy as np
a=np.load('gpurun_out/abstate_${c}base.npz'); b=np.load('gpurun_out/abstate_${c}sc.npz')
print('$c sc vs base bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
  NP="--no-cpu-baseline --no-other-solver --ccd $c"
  for v in base sc base2 sc2; do
    if [ ${v%2} = base ]; then L=""; else L="SOARM_SIM_LIB=$P"; fi
    env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06ab_${c}_drv_$v.json 2>> $O/r06ab_bench.err || exit $?
    env $L timeout -k 10 300 python bench.py $NP > $O/r06ab_${c}_st_$v.json 2>> $O/r06ab_bench.err || exit $?
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06ab_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items() if k == "collide"})
PY
