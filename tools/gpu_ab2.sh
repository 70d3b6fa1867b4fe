#!/bin/bash
# A/B of two library builds on the headline bench (steady window), alternating: A B A B
# usage: A=path B=path bash tools/gpu_ab2.sh tag
set -o pipefail
t=$1
for i in 1 2 3; do
  for v in A B; do
    lib=${!v}
    echo "== $v $lib $(date +%T)"
    SOARM_SIM_LIB=$lib timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-solver > gpurun_out/ab_${t}_${v}$i.json 2> gpurun_out/ab_${t}_${v}$i.err || exit 1
  done
done
echo ab-ok
