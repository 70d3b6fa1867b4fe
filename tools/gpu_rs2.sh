#!/bin/bash
# RS iteration: benches (RS kernel and quad kernel), then the parity-bar measurements of the RS kernel
mkdir -p gpurun_out
for w in 1 0; do
  SOARM_RS=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/bench_rs$w.json 2> gpurun_out/bench_rs$w.err || exit $?
  SOARM_RS=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5 > gpurun_out/benchd_rs$w.json 2>> gpurun_out/bench_rs$w.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_rs$w.json').read().strip().split(chr(10))[-1]); e=json.loads(open('gpurun_out/benchd_rs$w.json').read().strip().split(chr(10))[-1]); print('rs=$w', 'steady', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, 'driver', round(e['value']), {k: round(x,4) for k,x in e['roofline']['kernel_ms_per_step'].items()})"
done
SOARM_RS=1 timeout -k 10 400 python tools/rs_bars.py > gpurun_out/rs_bars.log 2>&1; rc=$?
cat gpurun_out/rs_bars.log | grep -v amdgpu.ids
exit $rc
