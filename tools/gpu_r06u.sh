#!/bin/bash
# Round 6: climbing records that carry their neighbours' coordinates (one round trip per climbing
# step) -- contact tests, bit identity against the previous build (tools/_abr6/lib_prev.so) for
# both narrowphases, bench A/B (MPR headline and native), driver window and steady
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
P=$R/tools/_abr6/lib_prev.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -k "native or contacts_match or separating or full_size" > $O/r06u_pytest.log 2>&1
rc=$?
grep -E "contacts:|PASS|FAIL|Error" $O/r06u_pytest.log | tail -14
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in mpr native; do
  CCD=$c timeout -k 10 300 python tools/ab_state.py ${c}new 60 > $O/r06u_ab.log 2>&1 || exit $?
  CCD=$c SOARM_SIM_LIB=$P timeout -k 10 300 python tools/ab_state.py ${c}prev 60 >> $O/r06u_ab.log 2>&1 || exit $?
  python -c "
import numpy as np
a=np.load('gpurun_out/abstate_${c}new.npz'); b=np.load('gpurun_out/abstate_${c}prev.npz')
print('$c new vs prev bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
done
for c in mpr native; do
  NP="--no-cpu-baseline --no-other-solver --ccd $c"
  for v in new prev; do
    if [ $v = new ]; then L=""; else L="SOARM_SIM_LIB=$P"; fi
    env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06u_${c}_drv_$v.json 2>> $O/r06u_bench.err || exit $?
    env $L timeout -k 10 300 python bench.py $NP > $O/r06u_${c}_st_$v.json 2>> $O/r06u_bench.err || exit $?
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06u_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
exit $rc
