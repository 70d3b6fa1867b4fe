#!/bin/bash
# the round-end GPU tiers on the final build: all -m gpu tests and smoke()
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -3 gpurun_out/smoke.log
