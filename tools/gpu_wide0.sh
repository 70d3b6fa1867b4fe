#!/bin/bash
# the quad kernel alone (SOARM_WIDE=0): the extra-slot test and the contact bench
mkdir -p gpurun_out
SOARM_WIDE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "extra_contact_sweeps or mixed_contacts" --timeout 150 --timeout-method thread > gpurun_out/w0_pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/w0_pytest.log
SOARM_WIDE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver > gpurun_out/w0_bench.json 2> gpurun_out/w0_bench.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/w0_bench.json').read().strip().split(chr(10))[-1]); print('wide0 value', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()})"
