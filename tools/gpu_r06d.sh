#!/bin/bash
# Round 6: paired vs sequential RS sweep (same build path) bit identity, substep anatomy of the first
# difference, and the rollout bench with / without a one-rank nccl group after the timing fix
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
step ab_paired 300 python tools/ab_state.py paired 60 || exit $?
SOARM_SIM_LIB=$R/tools/_abr6/lib_seq.so step ab_seq 300 python tools/ab_state.py seq 60 || exit $?
python -c "
import numpy as np
a=np.load('gpurun_out/abstate_paired.npz'); b=np.load('gpurun_out/abstate_seq.npz')
d=np.abs(a['obs']-b['obs']).max(axis=(1,2)); t=int(np.argmax(d>0)) if (d>0).any() else -1
print('paired vs seq bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')), 'first differing env-step', t)
open('gpurun_out/ab_first.txt','w').write(str(t))"
T=$(cat $O/ab_first.txt)
if [ "$T" != "-1" ]; then
  step sub_paired 300 python tools/ab_substeps.py paired $T || exit $?
  SOARM_SIM_LIB=$R/tools/_abr6/lib_seq.so step sub_seq 300 python tools/ab_substeps.py seq $T || exit $?
  python tools/ab_substeps.py --compare paired seq
fi
NP="--no-cpu-baseline --no-other-solver --no-profile --no-steady"
for i in 1 2; do
  step rollout_none$i 300 python bench.py --config rollout --steps 100 --warmup 5 $NP > $O/r06d_rollout_none$i.json 2> $O/r06d_rollout.err || exit $?
  step rollout_nccl$i 300 python bench.py --config rollout --steps 100 --warmup 5 $NP --dist-backend nccl > $O/r06d_rollout_nccl$i.json 2>> $O/r06d_rollout.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06d_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 4), (d.get("dist") or {}).get("rollout_gather_s"), (d.get("dist") or {}).get("rollout_gather_exact"))
PY
