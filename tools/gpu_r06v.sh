#!/bin/bash
# Round 6: k_collide at two waves per SIMD (256 VGPRs, no spills) against three (168 VGPRs, 88 B of
# scratch per lane for MPR) -- bit identity and bench A/B, both narrowphases
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
P=$R/tools/_abr6/lib_w2.so
for c in mpr native; do
  CCD=$c timeout -k 10 300 python tools/ab_state.py ${c}w3 60 > $O/r06v_ab.log 2>&1 || exit $?
  CCD=$c SOARM_SIM_LIB=$P timeout -k 10 300 python tools/ab_state.py ${c}w2 60 >> $O/r06v_ab.log 2>&1 || exit $?
  python -c "
import numpy as np
a=np.load('gpurun_out/abstate_${c}w3.npz'); b=np.load('gpurun_out/abstate_${c}w2.npz')
print('$c w2 vs w3 bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
  NP="--no-cpu-baseline --no-other-solver --ccd $c"
  for v in w3 w2; do
    if [ $v = w3 ]; then L=""; else L="SOARM_SIM_LIB=$P"; fi
    env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06v_${c}_drv_$v.json 2>> $O/r06v_bench.err || exit $?
    env $L timeout -k 10 300 python bench.py $NP > $O/r06v_${c}_st_$v.json 2>> $O/r06v_bench.err || exit $?
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06v_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
