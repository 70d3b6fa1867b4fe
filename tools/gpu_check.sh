#!/bin/bash
# One GPU call: the gpu test suite (or a -k selection), smoke, and bench lines for the
# configs given (default: contact).  Every GPU step has its own limit; the script stops at
# the first failure.   usage: tools/gpu_check.sh "<pytest -k expr or empty>" cfg...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
K=$1; shift
CFGS=${@:-contact}
if [ -n "$K" ]; then KK=(-k "$K"); else KK=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${KK[@]}" > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log | tail -20; exit 1; }
tail -4 $O/smoke.log
for c in $CFGS; do
  timeout -k 10 400 python bench.py --config $c --cpu-seconds 4 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$c.json')); r=d['roofline'] or {}; print('$c', round(d['value']), 'env-steps/s', round(d['ms_per_step'],4), 'ms/step', r.get('kernel_ms_per_step'), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']))"
done
