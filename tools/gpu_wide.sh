#!/bin/bash
# wide-PGS iteration: gpu tests, then the contact bench with the wide kernel and without (A/B)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in 1 0; do
  SOARM_WIDE=$w timeout -k 10 600 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/bench_w$w.json 2> gpurun_out/bench_w$w.err || exit $?
  SOARM_WIDE=$w timeout -k 10 600 python bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5 > gpurun_out/benchd_w$w.json 2>> gpurun_out/bench_w$w.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_w$w.json').read().strip().split(chr(10))[-1]); e=json.loads(open('gpurun_out/benchd_w$w.json').read().strip().split(chr(10))[-1]); print('wide=$w', 'steady', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, 'driver', round(e['value']), {k: round(x,4) for k,x in e['roofline']['kernel_ms_per_step'].items()})"
done
