#!/bin/bash
# DBKN GPU tests and the mpc_dbkn bench line (no diagnostic build)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_koopman_mpc.py -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/dbkn_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/dbkn_pytest.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --config mpc_dbkn > gpurun_out/bench_mpc_dbkn_s.json 2> gpurun_out/bench_mpc_dbkn_s.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_mpc_dbkn_s.json').read().strip().split(chr(10))[-1]); print('mpc_dbkn', round(d['value']), d['ms_per_step'])"
