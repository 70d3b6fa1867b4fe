#!/bin/bash
# PMC passes on k_substep: scalar-cache behaviour and memory-instruction mix
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_mem
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE --kernel-include-regex "k_substep" -f csv -d $O -o dc -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/b1.json && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS --kernel-include-regex "k_substep" -f csv -d $O -o mi -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/b2.json
