#!/usr/bin/env python3
"""Diagnostic: run the bench's contact workload for T env-steps with the library named by
SOARM_SIM_LIB and save the per-step obs checksums and the final state, so two builds can be
compared bit for bit (an exact change -- e.g. a cheaper separation proof -- must leave them
identical).  usage: ab_state.py TAG [T] [solver]; N=envs (default 4096: 8192 runs the quad PGS kernel)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

tag = sys.argv[1]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 120
solver = sys.argv[3] if len(sys.argv) > 3 else "PGS"
n = int(os.environ.get("N", "4096"))
cm = W.model("contact", solver=solver, ccd=os.environ.get("CCD", W.BENCH_CCD))
ids = np.arange(n)
sim = BatchSim(cm, n, 0)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
       for k, v in W.chirp_tables(ids, 0).items()}
obs_hist = []
for t in range(T):
    obs = sim.step(W.chirp_action(tab, float(t), lib=torch))
    obs_hist.append(obs.detach().cpu().numpy().copy())
torch.cuda.synchronize()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"abstate_{tag}.npz"), obs=np.stack(obs_hist),
                    qpos=sim.qpos.cpu().numpy(), qvel=sim.qvel.cpu().numpy())
print(tag, "done", flush=True)
