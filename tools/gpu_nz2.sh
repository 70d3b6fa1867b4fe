#!/bin/bash
# zone-prediction test + DBKN tests + DBKN bench (XCD-chunked k_bilinear)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py::test_newton_zone_prediction_same_optimum tests/test_gpu_parity.py::test_newton_solver_matches_oracle tests/test_koopman_mpc.py -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/nz2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/nz2_pytest.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --config mpc_dbkn > gpurun_out/bench_mpc_dbkn_x.json 2> gpurun_out/bench_mpc_dbkn_x.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_mpc_dbkn_x.json').read().strip().split(chr(10))[-1]); print('mpc_dbkn', round(d['value']), d['ms_per_step'])"
