#!/bin/bash
# full GPU test suite, then the contact bench (RS kernel) in the steady and driver windows
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -n 6 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/bench_rs1.json 2> gpurun_out/bench_rs1.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5 > gpurun_out/benchd_rs1.json 2>> gpurun_out/bench_rs1.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_rs1.json').read().strip().split(chr(10))[-1]); e=json.loads(open('gpurun_out/benchd_rs1.json').read().strip().split(chr(10))[-1]); print('steady', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, 'driver', round(e['value']), {k: round(x,4) for k,x in e['roofline']['kernel_ms_per_step'].items()})"
exit $rc
