#!/bin/bash
# contact-path GPU tests, the contact bench (steady + driver windows) and the steady-window phase profile
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "contact or substep or cube or separating or odd or full_size" > gpurun_out/pytest_iter.log 2>&1
rc=$?
tail -n 4 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/bench_rs1.json 2> gpurun_out/bench_rs1.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5 > gpurun_out/benchd_rs1.json 2>> gpurun_out/bench_rs1.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_rs1.json').read().strip().split(chr(10))[-1]); e=json.loads(open('gpurun_out/benchd_rs1.json').read().strip().split(chr(10))[-1]); print('steady', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, 'driver', round(e['value']), {k: round(x,4) for k,x in e['roofline']['kernel_ms_per_step'].items()})"
bash tools/gpu_phase_late.sh
exit $rc
