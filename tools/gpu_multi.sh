#!/bin/bash
# rollout bench (config 5) + a 2-rank gloo rehearsal of the multi-process bench path on one GPU
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --config rollout --steps 100 --warmup 5 --cpu-seconds 8 > gpurun_out/bench_rollout.json 2> gpurun_out/bench_rollout.err && cat gpurun_out/bench_rollout.json &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_w2.json 2> gpurun_out/bench_w2.err && cat gpurun_out/bench_w2.json &&
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --dist-backend gloo --config rollout --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_w2_rollout.json 2> gpurun_out/bench_w2_rollout.err && cat gpurun_out/bench_w2_rollout.json
