#!/bin/bash
# Round 6: native GJK/EPA with the EPA polytopes in LDS slots (k_collide<native>) -- native contact
# tests, bit identity against the previous build (tools/_abr6/lib_prev.so) and the native bench A/B
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
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -k "native or contacts_match" > $O/r06h_pytest.log 2>&1
rc=$?
grep -E "contacts:|PASS|FAIL|Error" $O/r06h_pytest.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
CCD=native step ab_new 300 python tools/ab_state.py nnew 60 || exit $?
CCD=native SOARM_SIM_LIB=$R/tools/_abr6/lib_prev.so step ab_prev 300 python tools/ab_state.py nprev 60 || exit $?
python -c "
import numpy as np
a=np.load('gpurun_out/abstate_nnew.npz'); b=np.load('gpurun_out/abstate_nprev.npz')
print('native new vs prev bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
NP="--no-cpu-baseline --no-other-solver --ccd native"
step drv_new 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06h_drv_new.json 2>> $O/r06h_bench.err || exit $?
SOARM_SIM_LIB=$R/tools/_abr6/lib_prev.so step drv_prev 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06h_drv_prev.json 2>> $O/r06h_bench.err || exit $?
step st_new 300 python bench.py $NP > $O/r06h_st_new.json 2>> $O/r06h_bench.err || exit $?
SOARM_SIM_LIB=$R/tools/_abr6/lib_prev.so step st_prev 300 python bench.py $NP > $O/r06h_st_prev.json 2>> $O/r06h_bench.err || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06h_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
exit $rc
