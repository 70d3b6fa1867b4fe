#!/bin/bash
# Round 6: EPA visibility as a mask from unrolled independent loads + running-minimum compaction
# (k_collide<native>) -- native contact tests, bit identity against the previous build
# (tools/_abr6/lib_prev.so), native bench A/B and the per-pair collide profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
P=$R/tools/_abr6/lib_prev.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -k "native or contacts_match" > $O/r06s_pytest.log 2>&1
rc=$?
grep -E "contacts:|PASS|FAIL|Error" $O/r06s_pytest.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
CCD=native timeout -k 10 300 python tools/ab_state.py nnew 60 > $O/r06s_ab.log 2>&1 || exit $?
CCD=native SOARM_SIM_LIB=$P timeout -k 10 300 python tools/ab_state.py nprev 60 >> $O/r06s_ab.log 2>&1 || exit $?
python -c "
import numpy as np
a=np.load('gpurun_out/abstate_nnew.npz'); b=np.load('gpurun_out/abstate_nprev.npz')
print('native new vs prev bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
NP="--no-cpu-baseline --no-other-solver --ccd native"
for v in new prev; do
  if [ $v = new ]; then L=""; else L="SOARM_SIM_LIB=$P"; fi
  env $L timeout -k 10 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06s_drv_$v.json 2>> $O/r06s_bench.err || exit $?
  env $L timeout -k 10 300 python bench.py $NP > $O/r06s_st_$v.json 2>> $O/r06s_bench.err || exit $?
done
CCD=native timeout -k 10 200 python tools/collide_prof.py 120 > $O/r06s_cprof.log 2>&1 || exit $?
grep max-wave $O/r06s_cprof.log | cut -c1-200
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"),
          {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
exit $rc
