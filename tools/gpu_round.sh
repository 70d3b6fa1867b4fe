#!/bin/bash
# one GPU session: tests, smoke, bench (each step time-limited, chained)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -25 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -3 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py --config nocontact --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/bench_nocontact.json 2> gpurun_out/bench_nocontact.err && cat gpurun_out/bench_nocontact.json &&
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --cpu-seconds 8 > gpurun_out/bench_contact.json 2> gpurun_out/bench_contact.err && cat gpurun_out/bench_contact.json
