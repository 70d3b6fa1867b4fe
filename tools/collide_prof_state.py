#!/usr/bin/env python3
"""Per-pair collide cost on a saved bench state (diagnostic): `save T` runs the contact workload
for T env-steps with the library SOARM_SIM_LIB names (default: the product build) and saves qpos;
`load TAG` loads it into a fresh batch (e.g. the -DSOARM_DIAG_SKIPP build under SOARM_DIAG_STAGE)
and prints, per pair, the longest wave's cycles of a profiled collide pass (the second of two, so
the separating-axis cache is warm), so builds that change the dynamics compare on one state."""
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
cm = W.model("contact", ccd=os.environ.get("CCD", W.BENCH_CCD))
path = os.path.join(ROOT, "gpurun_out", "cprof_state.npy")
sim = BatchSim(cm, n, 0)
ids = np.arange(n)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
if sys.argv[1] == "save":
    tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
           for k, v in W.chirp_tables(ids, 0).items()}
    for t in range(int(sys.argv[2])):
        sim.step(W.chirp_action(tab, float(t), lib=torch))
    np.save(path, sim.qpos.cpu().numpy())
    print("saved", path)
    sys.exit(0)
sim.qpos.copy_(torch.as_tensor(np.load(path), device=sim.device))
sim.collide_profile(with_max=True)
cyc, mx = sim.collide_profile(with_max=True)
d = cm.desc
top = np.argsort(-mx)[:8]
rows = [(int(p), cm.geom_names[d.pair_geom1[p]], cm.geom_names[d.pair_geom2[p]], int(mx[p]), int(cyc[p])) for p in top]
print(sys.argv[2], "max-wave (pair, g1, g2, max, sum):", rows, flush=True)
json.dump({"max": mx.tolist(), "sum": cyc.tolist()},
          open(os.path.join(ROOT, "gpurun_out", f"cprof_state_{sys.argv[2]}.json"), "w"))
