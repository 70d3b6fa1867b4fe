#!/bin/bash
# kernel trace of the DBKN MPC bench (which kernels take the 1 ms per frame)
mkdir -p gpurun_out/prof_dbkn
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dbkn -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config mpc_dbkn --no-cpu-baseline --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_dbkn/bench.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/prof_dbkn -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:12]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms total', r['Percentage'])
"
