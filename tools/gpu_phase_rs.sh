#!/bin/bash
# phase profile of the contact substep: RS kernel (and, with BOTH=1, the quad kernel)
mkdir -p gpurun_out
for w in 1 ${BOTH:+0}; do
  SOARM_RS=$w PROF_LIB=tools/_rsprof/libsoarm_sim_prof.so EVERY=${EVERY:-20} timeout -k 10 300 python tools/phase_prof.py ${T:-120} > gpurun_out/phase_rs$w.log 2>&1 || exit $?
done
