#!/bin/bash
# Round 6: the parity tests touched by the MPR-normal fix / soft-reset contacts / oracle-only envelope,
# the contact bench on this build, and bench.py's rollout with and without a one-rank nccl group (x2).
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
K=${K:-"full_size or soft_reset or pgs_vs_reference or mixed_contacts or extra_contact or contacts_match or separating or shadowing"}
step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $O/r06b_pytest.log 2>&1
rc=$?
tail -4 $O/r06b_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NP="--no-cpu-baseline --no-other-solver"
step bench_contact 300 python bench.py $NP > $O/r06b_contact.json 2> $O/r06b_contact.err || exit $?
step bench_contact_drv 300 python bench.py $NP --no-steady --steps 20 --warmup 5 > $O/r06b_contact_drv.json 2>> $O/r06b_contact.err || exit $?
for i in 1 2; do
  step rollout_none$i 300 python bench.py --config rollout --steps 100 --warmup 5 $NP --no-profile --no-steady > $O/r06b_rollout_none$i.json 2> $O/r06b_rollout.err || exit $?
  step rollout_nccl$i 300 python bench.py --config rollout --steps 100 --warmup 5 $NP --no-profile --no-steady --dist-backend nccl > $O/r06b_rollout_nccl$i.json 2>> $O/r06b_rollout.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06b_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e); continue
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("steady_state") or {}).get("value"), (d.get("dist") or {}).get("rollout_gather_s"))
PY
exit $rc
