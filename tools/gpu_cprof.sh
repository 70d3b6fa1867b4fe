#!/bin/bash
# per-pair collide cost with MPR and with native GJK/EPA
mkdir -p gpurun_out
timeout -k 10 300 env CCD=mpr python tools/collide_prof.py 120 > gpurun_out/cprof_mpr.log 2>&1 || exit $?
cp gpurun_out/collide_prof.json gpurun_out/collide_prof_mpr.json
timeout -k 10 300 env CCD=native python tools/collide_prof.py 120 > gpurun_out/cprof_native.log 2>&1 || exit $?
cp gpurun_out/collide_prof.json gpurun_out/collide_prof_native.json
grep -E "total|max-wave" gpurun_out/cprof_mpr.log gpurun_out/cprof_native.log | cut -c1-400
