#!/bin/bash
# quick GPU iteration: gpu tests + contact bench
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -25
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_contact.json 2> gpurun_out/bench_contact.err && cat gpurun_out/bench_contact.json
