#!/bin/bash
# Round 6: EPA closest-face scan with the running minimum in a register -- native contact tests,
# bit identity against the previous build (tools/_mbr6/lib_prev.so), native bench A/B (steady)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "native" > $O/r06o_pytest.log 2>&1
tail -1 $O/r06o_pytest.log
CCD=native timeout -k 10 300 python tools/ab_state.py onew 60 || exit $?
CCD=native SOARM_SIM_LIB=$R/tools/_mbr6/lib_prev.so timeout -k 10 300 python tools/ab_state.py oprev 60 || exit $?
python -c "
import numpy as np
a=np.load('gpurun_out/abstate_onew.npz'); b=np.load('gpurun_out/abstate_oprev.npz')
print('native new vs prev bit-identical:', all(np.array_equal(a[k], b[k]) for k in ('obs','qpos','qvel')))"
NP="--no-cpu-baseline --no-other-solver --ccd native"
for i in 1 2; do
  for v in new prev; do
    L=$R/lerobot-mujoco-sim2real_amd/csrc/libsoarm_sim.so
    [ $v = prev ] && L=$R/tools/_mbr6/lib_prev.so
    SOARM_SIM_LIB=$L timeout -k 10 300 python bench.py $NP > $O/r06o_$v$i.json 2>> $O/r06o.err || exit $?
    python -c "
import json; d=json.loads(open('$O/r06o_$v$i.json').read().strip().splitlines()[-1])
print('$v$i', round(d['value']), {k: round(x, 4) for k, x in d['roofline']['kernel_ms_per_step'].items()})"
  done
done
