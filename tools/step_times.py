#!/usr/bin/env python3
"""Diagnostic: GPU time of every env-step of the contact bench workload (HIP events),
to see how the step time evolves as the chirp drives the arm onto the table.
    python tools/step_times.py [T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 120
n = 4096
cm = W.model("contact")
ids = np.arange(n)
sim = BatchSim(cm, n, 0)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
       for k, v in W.chirp_tables(ids, 0).items()}
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(T)]
for t in range(T):
    a = W.chirp_action(tab, float(t), lib=torch)
    ev[t][0].record()
    sim.step(a)
    ev[t][1].record()
torch.cuda.synchronize()
ms = np.array([a.elapsed_time(b) for a, b in ev])
for t0 in range(0, T, 10):
    print(f"steps {t0:3d}-{t0 + 9:3d}: mean {ms[t0:t0 + 10].mean():.3f} ms  min {ms[t0:t0 + 10].min():.3f}  max {ms[t0:t0 + 10].max():.3f}")
print(f"bench window (20..{T - 1}): mean {ms[20:].mean():.3f} ms/step; first 20: {ms[:20].mean():.3f}")
