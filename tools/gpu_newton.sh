#!/bin/bash
# Newton-solver iteration: its GPU tests, then its bench line (and PGS's for reference).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "newton or late_states or extra_contact" > $O/pytest_newton.log 2>&1
rc=$?
tail -3 $O/pytest_newton.log
grep -E "^E .*Assert" $O/pytest_newton.log | head -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for args in "--solver newton --no-cpu-baseline" "--no-cpu-baseline"; do
  tag=$(echo $args | tr -d ' -' | cut -c1-40)
  timeout -k 10 400 python bench.py $args > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$tag.json')); r=d['roofline'] or {}; print('$args |', round(d['value']), 'env-steps/s', round(d['ms_per_step'],4), 'ms/step; kernel', r.get('kernel'), r.get('avg_launch_ms'), r.get('kernel_ms_per_step'))"
done
exit $rc
