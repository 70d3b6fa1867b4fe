#!/bin/bash
# collide cost by pair subset (diagnostic build with -DSOARM_DIAG_SKIPP; timings only, wrong contacts)
set -o pipefail
L=tools/_rsprof/lib_skipp.so
i=0
for sk in "" "~" "~27" "~26,27,84,85,23,24,25" "84,85,23,24,25,26,27"; do
  i=$((i+1))
  echo "== [$sk] $(date +%T)"
  SOARM_DIAG_SKIP="$sk" SOARM_SIM_LIB=$L timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-solver --no-steady > gpurun_out/skip_$i.json 2> gpurun_out/skip_$i.err || exit 1
done
echo skip-ok
