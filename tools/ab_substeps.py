#!/usr/bin/env python3
"""Diagnostic: the headline workload for T env-steps with the library SOARM_SIM_LIB names, then
env-step T substep by substep (ctrl = that step's action, as sim_step stages it), saving the state
after every substep and the contact list at every substep's start for the envs ENVS (default: all).
Two builds that must agree bit for bit (tools/ab_state.py found the first differing env-step) are
compared substep by substep with --compare.

    python tools/ab_substeps.py TAG T [first_env n_envs]
    python tools/ab_substeps.py --compare TAG_A TAG_B
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

if sys.argv[1] == "--compare":
    a = np.load(os.path.join(ROOT, "gpurun_out", f"absub_{sys.argv[2]}.npz"))
    b = np.load(os.path.join(ROOT, "gpurun_out", f"absub_{sys.argv[3]}.npz"))
    for s in range(a["qvel"].shape[0]):
        dq = np.abs(a["qvel"][s] - b["qvel"][s]).max(1)
        bad = np.flatnonzero(dq > 0)
        nc_a, nc_b = a["ncon"][s], b["ncon"][s]
        print(f"substep {s}: envs differing {bad[:8].tolist()} ({len(bad)}), max {dq.max():.3g}; "
              f"contact counts differ in {int((nc_a != nc_b).sum())} envs")
        if len(bad):
            e = bad[0]
            pid = lambda x, k, m: x["con"][s][k][:m, 7].astype(np.float32).view(np.int32).tolist()
            print("   env", int(a["ids"][e]), "pairs A", pid(a, e, nc_a[e]), "B", pid(b, e, nc_b[e]))
            w0 = e - e % 4
            print("   its wave's pair lists:", [pid(a, k, nc_a[k]) for k in range(w0, w0 + 4)])
            break
    sys.exit(0)

import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

tag, T = sys.argv[1], int(sys.argv[2])
e0 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
ne = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
n = 4096
cm = W.model("contact")
ids = np.arange(n)
sim = BatchSim(cm, n, 0)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
       for k, v in W.chirp_tables(ids, 0).items()}
for t in range(T):
    sim.step(W.chirp_action(tab, float(t), lib=torch))
a = W.chirp_action(tab, float(T), lib=torch)
sim.ctrl[:5].copy_(a.T)
qv, con, ncon = [], [], []
for s in range(10):
    out, nc = sim.contacts()
    con.append(out.cpu().numpy()[e0:e0 + ne])
    ncon.append(nc.cpu().numpy()[e0:e0 + ne])
    sim.substeps(1)
    qv.append(sim.qvel.cpu().numpy().T[e0:e0 + ne].copy())
torch.cuda.synchronize()
np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"absub_{tag}.npz"), qvel=np.stack(qv), con=np.stack(con),
                    ncon=np.stack(ncon), ids=np.arange(e0, e0 + ne))
print(tag, "done", flush=True)
