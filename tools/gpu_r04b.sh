#!/bin/bash
# r04: all GPU tests, then the contact bench with the wide kernel (default) and the quad kernel
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in 1 0; do
  SOARM_WIDE=$w timeout -k 10 600 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/bench_w$w.json 2> gpurun_out/bench_w$w.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_w$w.json').read().strip().split(chr(10))[-1]); print('wide $w value', round(d['value']), 'steady', round(d['steady_state']['value']) if d['steady_state'] else None, {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()})"
done
