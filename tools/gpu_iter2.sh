#!/bin/bash
# iteration: contact-path GPU tests (RS default), then the contact bench (steady + driver window)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "contact or substep or cube or shard or separating or odd or config1" > gpurun_out/pytest_iter.log 2>&1
rc=$?
tail -n 15 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in 1 0; do
  SOARM_RS=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/bench_rs$w.json 2> gpurun_out/bench_rs$w.err || exit $?
  SOARM_RS=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 20 --warmup 5 > gpurun_out/benchd_rs$w.json 2>> gpurun_out/bench_rs$w.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_rs$w.json').read().strip().split(chr(10))[-1]); e=json.loads(open('gpurun_out/benchd_rs$w.json').read().strip().split(chr(10))[-1]); print('rs=$w', 'steady', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, 'driver', round(e['value']), {k: round(x,4) for k,x in e['roofline']['kernel_ms_per_step'].items()})"
done
