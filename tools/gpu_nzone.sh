#!/bin/bash
# Newton zone prediction: all GPU tests, the Newton bench line and the Newton phase profile
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --solver newton --no-cpu-baseline > gpurun_out/bench_contact_newton.json 2> gpurun_out/bench_contact_newton.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_contact_newton.json').read().strip().split(chr(10))[-1]); print('newton value', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, d.get('other_solver'))"
timeout -k 10 300 env SOLVER=NEWTON EVERY=20 python tools/phase_prof.py 120 > gpurun_out/phase_newton.log 2>&1 || exit $?
tail -4 gpurun_out/phase_newton.log | cut -c1-600
