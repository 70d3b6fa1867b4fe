#!/bin/bash
# r04: wide-step microbenchmark, GPU tests (incl. native CCD contacts), contact bench MPR vs native
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o gpurun_out/mb_wide tools/mb_wide.hip 2>/dev/null && timeout -k 5 60 gpurun_out/mb_wide > gpurun_out/mb_wide.log 2>&1; rm -f gpurun_out/mb_wide; cat gpurun_out/mb_wide.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in mpr native; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --no-other-solver --ccd $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_$c.json').read().strip().split(chr(10))[-1]); print('$c', 'value', round(d['value']), 'steady', round(d['steady_state']['value']) if d['steady_state'] else None, {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()})"
done
timeout -k 10 600 python bench.py --no-cpu-baseline --config mpc_dbkn > gpurun_out/bench_mpc_dbkn.json 2> gpurun_out/bench_mpc_dbkn.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_mpc_dbkn.json').read().strip().split(chr(10))[-1]); print('mpc_dbkn', round(d['value']), d['ms_per_step'])"
timeout -k 10 180 python tools/collide_prof.py 120 > gpurun_out/collide_prof.log 2>&1 || exit $?
tail -2 gpurun_out/collide_prof.log
