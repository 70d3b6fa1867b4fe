#!/bin/bash
# A/B of tools/_ab/lib_<name>.so builds on the GPU: bit-identity of a 120-step contact
# trajectory against the first name, then the contact bench per build.
#   usage: tools/gpu_ab.sh base variant [variant...]   (SOLVER=newton for the Newton kernel)
mkdir -p gpurun_out
S=${SOLVER:-PGS}
for v in "$@"; do
  SOARM_SIM_LIB=tools/_ab/lib_$v.so timeout -k 10 300 python tools/ab_state.py $v 120 $S > gpurun_out/abstate_$v.log 2>&1 || exit $?
done
python - "$@" <<'PY'
import sys, numpy as np
names = sys.argv[1:]
a = np.load(f"gpurun_out/abstate_{names[0]}.npz")
for v in names[1:]:
    b = np.load(f"gpurun_out/abstate_{v}.npz")
    same = all(np.array_equal(a[k], b[k]) for k in ("obs", "qpos", "qvel"))
    first = next((t for t in range(a["obs"].shape[0]) if not np.array_equal(a["obs"][t], b["obs"][t])), None)
    print(v, "bit-identical" if same else f"DIFFERS (first obs step {first}, max |dqvel| {np.abs(a['qvel']-b['qvel']).max():.3e})")
PY
SOL=""
[ "$S" != "PGS" ] && SOL="--solver newton"
for v in "$@"; do
  SOARM_SIM_LIB=tools/_ab/lib_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver $SOL > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  SOARM_SIM_LIB=tools/_ab/lib_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-other-solver --no-steady $SOL --steps 20 --warmup 5 > gpurun_out/abd_$v.json 2>> gpurun_out/ab_$v.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().split(chr(10))[-1]); e=json.loads(open('gpurun_out/abd_$v.json').read().strip().split(chr(10))[-1]); print('$v', 'steady', round(d['value']), {k: round(x,4) for k,x in d['roofline']['kernel_ms_per_step'].items()}, 'driver', round(e['value']), {k: round(x,4) for k,x in e['roofline']['kernel_ms_per_step'].items()})"
done
