#!/bin/bash
# r04: all GPU tests, the contact bench, the DBKN phase profile and the DBKN MPC bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/bench_contact.json 2> gpurun_out/bench_contact.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_contact.json').read().strip().split(chr(10))[-1]); print('contact value', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()})"
SOARM_SIM_LIB=$PWD/tools/_prof/libsoarm_bl.so timeout -k 10 200 python tools/bl_prof.py > gpurun_out/bl_prof.json 2>&1 || exit $?
cat gpurun_out/bl_prof.json
timeout -k 10 300 python bench.py --no-cpu-baseline --config mpc_dbkn > gpurun_out/bench_mpc_dbkn.json 2> gpurun_out/bench_mpc_dbkn.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_mpc_dbkn.json').read().strip().split(chr(10))[-1]); print('mpc_dbkn', round(d['value']), d['ms_per_step'])"
