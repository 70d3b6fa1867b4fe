mkdir -p gpurun_out/ab
for s in 20 100; do
  w=5; [ $s = 100 ] && w=20
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps $s --warmup $w > gpurun_out/ab/main.$s.json 2>gpurun_out/ab/main.$s.err || exit 1
done
timeout -k 10 150 python bench.py --no-cpu-baseline --config dr --steps 50 --warmup 5 > gpurun_out/ab/dr.json 2>gpurun_out/ab/dr.err || exit 1
CONFIG=contact timeout -k 10 150 python tools/phase_prof.py 100 > gpurun_out/pp_contact.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
