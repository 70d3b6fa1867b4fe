#!/usr/bin/env python3
"""Diagnostic (the -DSOARM_DIAG_SUPPORT build via SOARM_SIM_LIB): run the contact workload for T
env-steps and print, per mesh geom, how many support queries repeated the lane's previous query's
cube-map cell or answer vertex on that geom (the batch prints its counters when freed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

n, T = 4096, int(sys.argv[1])
cm = W.model("contact", ccd=os.environ.get("CCD", W.BENCH_CCD))
print({g: name for g, name in enumerate(cm.geom_names)}, flush=True)
ids = np.arange(n)
sim = BatchSim(cm, n, 0)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
       for k, v in W.chirp_tables(ids, 0).items()}
for t in range(T):
    sim.step(W.chirp_action(tab, float(t), lib=torch))
torch.cuda.synchronize()
sim.close()
