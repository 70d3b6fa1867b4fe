#!/bin/bash
# Round 6: a substep's start reuses the kinematics the previous substep's end (or k_geom) wrote with
# the body frames (soarm_collide.h fk_extra) -- the GPU suite, bit identity against the previous
# build (tools/_abr6/lib_prev.so) for PGS (RS), Newton and the 8192-env quad kernel (dr), bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
P=$R/tools/_abr6/lib_prev.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06y_pytest.log 2>&1 || { tail -30 $O/r06y_pytest.log; exit 1; }
tail -1 $O/r06y_pytest.log
for spec in pgs:4096:PGS newton:4096:newton quad:8192:PGS; do
  IFS=: read T NE SOLV <<< "$spec"
  N=$NE timeout -k 10 300 python tools/ab_state.py ${T}new 60 $SOLV > $O/r06y_ab.log 2>&1 || exit $?
  N=$NE SOARM_SIM_LIB=$P timeout -k 10 300 python tools/ab_state.py ${T}prev 60 $SOLV >> $O/r06y_ab.log 2>&1 || exit $?
  python -c "
import numpy as np
a=np.load('gpurun_out/abstate_${T}new.npz'); b=np.load('gpurun_out/abstate_${T}prev.npz')
print('$T new vs prev bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
done
for cfg in "contact:" "contact:--solver newton" "dr:--steps 50 --warmup 5"; do
  C=${cfg%%:*}; X=${cfg#*:}
  T=$C$(echo "$X" | tr -d ' -' | cut -c1-10)
  for v in new prev; do
    if [ $v = new ]; then L=""; else L="SOARM_SIM_LIB=$P"; fi
    env $L timeout -k 10 300 python bench.py --config $C $X --no-cpu-baseline --no-other-solver > $O/r06y_${T}_$v.json 2>> $O/r06y_bench.err || exit $?
  done
done
env timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5 > $O/r06y_drv_new.json 2>> $O/r06y_bench.err || exit $?
env SOARM_SIM_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5 > $O/r06y_drv_prev.json 2>> $O/r06y_bench.err || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06y_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
