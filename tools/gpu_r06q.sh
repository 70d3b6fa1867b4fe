#!/bin/bash
# Round 6, last build: the whole GPU suite, smoke, and the default bench line (driver window)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/r06q_pytest.log 2>&1 || { tail -30 $O/r06q_pytest.log; exit 1; }
tail -1 $O/r06q_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r06q_smoke.log 2>&1 || exit $?
tail -1 $O/r06q_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r06q_bench.json 2> $O/r06q_bench.err || exit $?
python -c "
import json; d=json.loads(open('$O/r06q_bench.json').read().strip().splitlines()[-1])
print(round(d['value']), round(d['ms_per_step'], 4), (d.get('steady_state') or {}).get('value'), d['roofline']['frac'], d['cpu_baseline']['value'])"
