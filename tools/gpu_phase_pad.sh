#!/bin/bash
# phase profile of the RS substep (per-wave profile rows) and of the quad kernel
mkdir -p gpurun_out
for w in 1 0; do
  SOARM_RS=$w PROF_LIB=tools/_rsprof/libsoarm_sim_prof.so EVERY=20 timeout -k 10 300 python tools/phase_prof.py 30 > gpurun_out/phase_rs$w.log 2>&1 || exit $?
done
python tools/phase_summary.py 1 0 | grep -v "^29\|^ *{" | head -12; python tools/phase_summary.py 1 0 | grep "^ *{" | head -4
