#!/bin/bash
# quick GPU iteration: gpu tests + contact bench.  Test failures (rc 1) still
# run the bench; a crash / abort / timeout ends the script there.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_contact.json 2> gpurun_out/bench_contact.err && cat gpurun_out/bench_contact.json
