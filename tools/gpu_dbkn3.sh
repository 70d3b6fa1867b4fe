#!/bin/bash
# DBKN: GPU tests, the phase profile (diagnostic library) and the mpc_dbkn bench line
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_koopman_mpc.py tests/test_gpu_parity.py::test_pgs_vs_reference_newton -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/dbkn_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/dbkn_pytest.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SOARM_SIM_LIB=$PWD/tools/_prof/libsoarm_bl.so timeout -k 10 200 python tools/bl_prof.py > gpurun_out/bl_prof.json 2>&1 || exit $?
cat gpurun_out/bl_prof.json
timeout -k 10 300 python bench.py --no-cpu-baseline --config mpc_dbkn > gpurun_out/bench_mpc_dbkn.json 2> gpurun_out/bench_mpc_dbkn.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_mpc_dbkn.json').read().strip().split(chr(10))[-1]); print('mpc_dbkn', round(d['value']), d['ms_per_step'])"
