#!/bin/bash
# Round 6: box-box on 4-lane quads in k_collide (slices) -- parity tests, bit identity against the
# previous build (tools/_abr6/lib_prev.so), and the contact bench A/B (driver window and steady)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 $lim "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  return $rc
}
step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -k "full_size or contacts_match or separating or shard or soft_reset or cube_rests or one_substep_with_contacts" > $O/r06e_pytest.log 2>&1
rc=$?
grep -E "env-step vs oracle|contacts:|PASS|FAIL|Error" $O/r06e_pytest.log | tail -24
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step ab_new 300 python tools/ab_state.py new 60 || exit $?
SOARM_SIM_LIB=$R/tools/_abr6/lib_prev.so step ab_prev 300 python tools/ab_state.py prev 60 || exit $?
python -c "
import numpy as np
a=np.load('gpurun_out/abstate_new.npz'); b=np.load('gpurun_out/abstate_prev.npz')
d=np.abs(a['obs']-b['obs']).max(axis=(1,2))
print('new vs prev bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')), 'first differing env-step', int(np.argmax(d>0)) if (d>0).any() else -1, 'max obs diff', float(d.max()))"
NP="--no-cpu-baseline --no-other-solver"
for i in 1 2; do
  step drv_new$i 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06e_drv_new$i.json 2>> $O/r06e_bench.err || exit $?
  SOARM_SIM_LIB=$R/tools/_abr6/lib_prev.so step drv_prev$i 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06e_drv_prev$i.json 2>> $O/r06e_bench.err || exit $?
done
step st_new 300 python bench.py $NP > $O/r06e_st_new.json 2>> $O/r06e_bench.err || exit $?
SOARM_SIM_LIB=$R/tools/_abr6/lib_prev.so step st_prev 300 python bench.py $NP > $O/r06e_st_prev.json 2>> $O/r06e_bench.err || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06e_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
exit $rc
