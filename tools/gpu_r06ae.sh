#!/bin/bash
# Round 6: bit identity of the final soft-reset shape against the build before the fix (bench workload:
# RS PGS, Newton, the 8192-env quad kernel)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
P=$R/tools/_abr6/lib_prefix.so
for spec in pgs:4096:PGS newton:4096:newton quad:8192:PGS; do
  IFS=: read T NE SOLV <<< "$spec"
  N=$NE timeout -k 10 300 python tools/ab_state.py ${T}new 60 $SOLV > $O/r06ae_ab.log 2>&1 || exit $?
  N=$NE SOARM_SIM_LIB=$P timeout -k 10 300 python tools/ab_state.py ${T}prev 60 $SOLV >> $O/r06ae_ab.log 2>&1 || exit $?
  python -c "
import numpy as np
a=np.load('gpurun_out/abstate_${T}new.npz'); b=np.load('gpurun_out/abstate_${T}prev.npz')
print('$T final vs pre-fix bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
done
