#!/usr/bin/env python3
"""Diagnostic: which test decides each candidate pair (midphase / support bound / cached axis /
MPR), per pair, on the bench's contact workload.  Needs a build with -DSOARM_COLLIDE_STATS
(tools/ab_build.sh cstats -DSOARM_COLLIDE_STATS; run with SOARM_SIM_LIB=tools/_ab/lib_cstats.so)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

CODES = ["midphase", "bound", "cached", "mpr_sep_axis", "mpr_no_axis", "mpr_contact", "other_narrow", "-"]
n = 4096
cm = W.model("contact")
ids = np.arange(n)
sim = BatchSim(cm, n, 0)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
       for k, v in W.chirp_tables(ids, 0).items()}
T = int(sys.argv[1]) if len(sys.argv) > 1 else 120
d = cm.desc
for t in range(T + 1):
    if t in (5, T // 2, T):
        w0, w1 = sim.collide_profile(with_max=True)
        for p in range(d.npair):
            cnt = {}
            for c in range(8):
                w = int(w0[p] if c < 4 else w1[p])
                k = (w >> (13 * (c & 3))) & 8191
                if k:
                    cnt[CODES[c]] = k
            if set(cnt) - {"midphase"}:
                print(t, p, cm.geom_names[d.pair_geom1[p]], cm.geom_names[d.pair_geom2[p]], cnt, flush=True)
    sim.step(W.chirp_action(tab, float(t), lib=torch))
