#!/bin/bash
# XCD-aware block numbering: all GPU tests, contact (PGS) and Newton bench lines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_contact_x.json 2> gpurun_out/bench_contact_x.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_contact_x.json').read().strip().split(chr(10))[-1]); print('contact', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, d.get('other_solver'))"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-solver > gpurun_out/bench_drv_x.json 2> gpurun_out/bench_drv_x.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_drv_x.json').read().strip().split(chr(10))[-1]); print('driver window', round(d['value']), d['ms_per_step'])"
timeout -k 10 600 python bench.py --ccd native --no-cpu-baseline --no-other-solver > gpurun_out/bench_native_x.json 2> gpurun_out/bench_native_x.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_native_x.json').read().strip().split(chr(10))[-1]); print('native', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()})"
