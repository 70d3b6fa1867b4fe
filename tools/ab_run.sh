#!/bin/bash
# run the contact bench once per tools/_ab/lib_*.so (pass names as arguments)
mkdir -p gpurun_out
for v in "$@"; do
  SOARM_SIM_LIB=tools/_ab/lib_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().split(chr(10))[-1]); print('$v', round(d['value']), d['roofline']['kernel_ms_per_step'])"
done
