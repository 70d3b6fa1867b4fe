#!/usr/bin/env python3
"""Per-pair cost of the collide kernel on the bench workload (diagnostic).

Runs the `contact` workload for T env-steps, then one profiled collide pass
(sim_collide_profile) and prints each candidate pair's summed wave cycles."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

n = 4096
cm = W.model(os.environ.get("CONFIG", "contact"), ccd=os.environ.get("CCD", W.BENCH_CCD))
ids = np.arange(n)
sim = BatchSim(cm, n, 0)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
       for k, v in W.chirp_tables(ids, 0).items()}
res = {}
T = int(sys.argv[1]) if len(sys.argv) > 1 else 120
for t in range(T + 1):
    if t in (5, T // 2, T):
        cyc, mx = sim.collide_profile(with_max=True)
        tot = cyc.sum()
        top = np.argsort(-cyc)[:12]
        d = cm.desc
        rows = [(int(p), cm.geom_names[d.pair_geom1[p]], cm.geom_names[d.pair_geom2[p]], round(cyc[p] / tot, 4))
                for p in top]
        topm = np.argsort(-mx)[:12]
        rows_max = [(int(p), cm.geom_names[d.pair_geom1[p]], cm.geom_names[d.pair_geom2[p]], int(mx[p])) for p in topm]
        res[t] = {"total_wave_cycles": tot, "top": rows, "top_max_wave": rows_max}
        print(t, "max-wave", rows_max, flush=True)
        print(t, f"total {tot:.3e}", rows, flush=True)
    sim.step(W.chirp_action(tab, float(t), lib=torch))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "collide_prof.json"), "w"), indent=1)
