#!/bin/bash
# Round 6: contact/full-size parity (measured values printed), the paired RS sweep A/B (bit identity
# + time) against the sequential build (tools/_abr6/lib_seq.so, -DSOARM_RS_SEQ=1), and where the
# nccl rollout's per-step cost comes from (rccl_cost --pg-first; hip API stats of both bench runs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 $lim "$@"
  local rc=$?
  echo "== $name rc=$rc" >&2
  return $rc
}
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 300 --timeout-method thread -k "full_size or contacts_match" > $O/r06c_pytest.log 2>&1
rc=$?
grep -E "env-step vs oracle|contacts:|PASS|FAIL" $O/r06c_pytest.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step ab_paired 300 python tools/ab_state.py paired 60 || exit $?
SOARM_SIM_LIB=$R/tools/_abr6/lib_seq.so step ab_seq 300 python tools/ab_state.py seq 60 || exit $?
python -c "
import numpy as np
a=np.load('gpurun_out/abstate_paired.npz'); b=np.load('gpurun_out/abstate_seq.npz')
print('paired vs seq bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
NP="--no-cpu-baseline --no-other-solver"
for i in 1 2; do
  step b_paired$i 300 python bench.py $NP > $O/r06c_paired$i.json 2>> $O/r06c_bench.err || exit $?
  SOARM_SIM_LIB=$R/tools/_abr6/lib_seq.so step b_seq$i 300 python bench.py $NP > $O/r06c_seq$i.json 2>> $O/r06c_bench.err || exit $?
done
step rccl_pgfirst 300 python tools/rccl_cost.py --config rollout --pg-first --phases none,nccl_used > $O/r06c_rccl_pgfirst.json 2> $O/r06c_rccl_pgfirst.err || exit $?
grep -v Warn $O/r06c_rccl_pgfirst.err | tail -3
cd /tmp
B="--config rollout --steps 50 --warmup 5 --no-cpu-baseline --no-profile --no-steady --no-other-solver"
step hip_none 300 rocprofv3 --hip-trace --stats -f csv -d $O/r06c_hip_none -o t -- python3 $R/bench.py $B > $O/r06c_hip_none.json || exit $?
step hip_nccl 300 rocprofv3 --hip-trace --stats -f csv -d $O/r06c_hip_nccl -o t -- python3 $R/bench.py $B --dist-backend nccl > $O/r06c_hip_nccl.json || exit $?
cd $R
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06c_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, round(d.get("value", 0)), round(d.get("ms_per_step", 0), 4), (d.get("steady_state") or {}).get("value"),
              {k: round(v, 4) for k, v in ((d.get("roofline") or {}).get("kernel_ms_per_step") or {}).items()})
    except Exception as e:
        print(f, "unreadable", e)
PY
exit $rc
