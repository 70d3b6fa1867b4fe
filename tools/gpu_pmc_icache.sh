#!/bin/bash
# PMC passes on k_substep: instruction-cache behaviour and issue/wait split
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_ic
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-include-regex "k_substep" -f csv -d $O -o ic -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/b1.json && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_LDS --kernel-include-regex "k_substep" -f csv -d $O -o sq -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/b2.json
rc=$?
find $O -name "*.csv" | head
exit $rc
