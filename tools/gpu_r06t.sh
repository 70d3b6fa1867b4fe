#!/bin/bash
# Round 6: where native k_collide's longest waves go -- GJK alone (SOARM_DIAG_STAGE=3, the
# diagnostic build) against GJK + EPA and against MPR, per pair, on the same t = 60 / 120 states
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
D=$R/tools/_abr6/lib_diag.so
for T in 60 120; do
  CCD=native timeout -k 10 200 python tools/collide_prof_state.py save $T > /dev/null || exit $?
  CCD=native SOARM_SIM_LIB=$D timeout -k 10 200 python tools/collide_prof_state.py load native_t$T || exit $?
  CCD=native SOARM_SIM_LIB=$D SOARM_DIAG_STAGE=3 timeout -k 10 200 python tools/collide_prof_state.py load gjk_t$T || exit $?
  CCD=mpr SOARM_SIM_LIB=$D timeout -k 10 200 python tools/collide_prof_state.py load mpr_t$T || exit $?
done
