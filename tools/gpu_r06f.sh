#!/bin/bash
# Round 6: the RS kernel compiled for 2 waves per SIMD (SOARM_RS2=1) at config 4's 8192 envs per GPU
# against the quad kernel (default above rs_cap): time and the full-size DR parity test
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
NP="--no-cpu-baseline --no-other-solver --no-steady --config dr --steps 20 --warmup 5"
step dr_quad 300 python bench.py $NP > $O/r06f_dr_quad.json 2> $O/r06f.err || exit $?
SOARM_RS2=1 step dr_rs2 300 python bench.py $NP > $O/r06f_dr_rs2.json 2>> $O/r06f.err || exit $?
SOARM_RS2=1 step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -k "dr_env_step_full_size" > $O/r06f_pytest.log 2>&1
grep -E "env-step vs oracle|PASS|FAIL" $O/r06f_pytest.log | tail -4
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06f_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
PY
