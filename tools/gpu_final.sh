#!/bin/bash
# Round-end evidence in one GPU call: gpu tests, smoke and every bench line (tools/gpu_profile.sh
# bench half), the phase profiles of the contact substep (PGS and Newton), and the PGS-vs-Newton
# gap measurement.  Each step time-limited; a failure ends the script.
#   usage: tools/gpu_final.sh tag
set -o pipefail
TAG=${1:-r03}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $O
PART=bench bash tools/gpu_profile.sh $TAG || exit $?
timeout -k 10 300 python tools/phase_prof.py 120 > $O/phase_pgs.log 2>&1 || exit $?
SOLVER=NEWTON timeout -k 10 300 python tools/phase_prof.py 120 > $O/phase_newton.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/newton_gap.py --out $O/${TAG}_newton_gap.json > $O/newton_gap.log 2>&1 || { tail -5 $O/newton_gap.log; exit 1; }
echo final-ok
