#!/bin/bash
# Round-3 GPU call: gpu tests (all, failures listed), then bench lines: contact (PGS, headline),
# contact with the Newton solver, the driver's window.  Every GPU step has its own limit; a
# crash / abort / timeout ends the script (test failures, rc 1, do not).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for args in "--cpu-seconds 4" "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"; do
  tag=$(echo $args | tr -d ' -' | cut -c1-40)
  timeout -k 10 400 python bench.py $args > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); r=d['roofline'] or {}; s=d.get('steady_state') or {}; print('$args |', round(d['value']), 'env-steps/s', round(d['ms_per_step'],4), 'ms/step; steady', s.get('value') and round(s['value']), '; kernel', r.get('kernel'), r.get('avg_launch_ms'), r.get('kernel_ms_per_step'), '; other', d.get('other_solver'))"
done
exit $rc
