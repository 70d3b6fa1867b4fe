#!/bin/bash
# quick GPU iteration: gpu tests, contact bench, phase profile (one line per window)
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_contact.json 2> gpurun_out/bench_contact.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/bench_contact.json')); print('BENCH', round(d['value']), d['roofline']['kernel_ms_per_step'])"
timeout -k 10 300 python tools/phase_prof.py 120 > gpurun_out/phase.log 2>&1 || exit $?
tail -3 gpurun_out/phase.log | python -c "
import sys,json
for l in sys.stdin:
    t,j=l.split(' ',1); d=json.loads(j); print(t, round(d['cycles_per_wave']), d['variant_max_cycles'], d['stamps_per_wave'])"
