#!/bin/bash
# Round 6: soft resets decided by check_state's return (status bits are sticky: a second reset for
# the same cause had kept the discarded state's contacts) -- the GPU suite, the repeated-reset test
# on the previous build (expected to fail there), bit identity against it on the bench workload
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
P=$R/tools/_abr6/lib_prev.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r06aa_pytest.log 2>&1 || { tail -30 $O/r06aa_pytest.log; exit 1; }
tail -1 $O/r06aa_pytest.log
SOARM_SIM_LIB=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "soft_reset_contact_scene" > $O/r06aa_prev_reset.log 2>&1
echo "previous build, repeated-reset test rc=$? (1 = failed as expected)"
grep -E "passed|failed" $O/r06aa_prev_reset.log | tail -1
for spec in pgs:4096:PGS newton:4096:newton quad:8192:PGS; do
  IFS=: read T NE SOLV <<< "$spec"
  N=$NE timeout -k 10 300 python tools/ab_state.py ${T}new 60 $SOLV > $O/r06aa_ab.log 2>&1 || exit $?
  N=$NE SOARM_SIM_LIB=$P timeout -k 10 300 python tools/ab_state.py ${T}prev 60 $SOLV >> $O/r06aa_ab.log 2>&1 || exit $?
  python -c "
import numpy as np
a=np.load('gpurun_out/abstate_${T}new.npz'); b=np.load('gpurun_out/abstate_${T}prev.npz')
print('$T new vs prev bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
done
