#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u tools/newton_dbg.py 120 > $R/gpurun_out/newton_dbg.log 2>&1; rc=$?
cat $R/gpurun_out/newton_dbg.log | tail -20
timeout -k 10 300 python -u tools/newton_dbg.py 20 >> $R/gpurun_out/newton_dbg.log 2>&1 || exit 1
tail -14 $R/gpurun_out/newton_dbg.log
exit $rc
