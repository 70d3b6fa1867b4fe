#!/bin/bash
# Round-3 GPU call: gpu tests (all, failures listed), the PGS-vs-Newton gap measurement on the
# device, and the headline bench (default window and the driver's window).  Every GPU step has
# its own limit; a crash / abort / timeout ends the script (test failures, rc 1, do not).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
grep -E "FAILED|Error" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/newton_gap.py --out $O/r03_newton_gap.json > $O/newton_gap.log 2>&1 || { tail -20 $O/newton_gap.log; exit 1; }
timeout -k 10 400 python bench.py --cpu-seconds 4 > $O/bench_contact.json 2> $O/bench_contact.err || { tail -20 $O/bench_contact.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
for f in bench_contact bench_driver; do
  python -c "import json; d=json.load(open('$O/$f.json')); r=d['roofline'] or {}; print('$f', round(d['value']), 'env-steps/s', round(d['ms_per_step'],4), 'ms/step', r.get('avg_launch_ms'), r.get('kernel_ms_per_step'))"
done
exit $rc
