#!/bin/bash
# 2-rank gloo rehearsals of the multi-process bench path on one GPU (contact, rollout, mpc configs);
# the 8-GPU RCCL runs are the driver's.  Every step has its own limit; the first failure ends it.
mkdir -p gpurun_out
port=29511
for c in contact rollout mpc; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --dist-backend gloo --config $c --steps 20 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bench_w2_$c.json 2> gpurun_out/bench_w2_$c.err || { tail -20 gpurun_out/bench_w2_$c.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_w2_$c.json').read().strip().split(chr(10))[-1]); print('$c', d['n_gpus'], round(d['value']), d['config']['global_envs'], d['validity']['state_finite'])"
  port=$((port + 1))
done
