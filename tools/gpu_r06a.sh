#!/bin/bash
# Round 6, first call: the GPU suite on a fresh box, then what a live process group costs the step
# loop (tools/rccl_cost.py: no PG / gloo / nccl eager / nccl after use / destroyed, rollout and contact).
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
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -z "$NO_TESTS" ]; then
  step pytest 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/r06a_pytest.log 2>&1
  tail -2 $O/r06a_pytest.log
fi
step rccl_rollout 300 python tools/rccl_cost.py --config rollout > $O/r06a_rccl_rollout.json 2> $O/r06a_rccl_rollout.err
step rccl_rollout_lazy 300 python tools/rccl_cost.py --config rollout --lazy --phases none,nccl,nccl_used > $O/r06a_rccl_rollout_lazy.json 2> $O/r06a_rccl_rollout_lazy.err
step rccl_rollout_pin 300 python tools/rccl_cost.py --config rollout --pin --phases none,nccl,nccl_used > $O/r06a_rccl_rollout_pin.json 2> $O/r06a_rccl_rollout_pin.err
step rccl_contact 300 python tools/rccl_cost.py --config contact --steps 30 > $O/r06a_rccl_contact.json 2> $O/r06a_rccl_contact.err
cat $O/r06a_rccl_*.err | grep -v Warning
echo r06a-ok
