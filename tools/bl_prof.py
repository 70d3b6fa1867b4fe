#!/usr/bin/env python3
"""Phase cycles of the DBKN first-move kernel k_bilinear (diagnostic; needs the library built
with -DSOARM_BL_PROF, passed as SOARM_SIM_LIB): 4096 envs, a few control steps."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import abi  # noqa: E402
from lerobot_mujoco_sim2real_amd.control.koopman import KoopmanBlinear  # noqa: E402
from lerobot_mujoco_sim2real_amd.control.MPC_Controler import MPCController  # noqa: E402


class Args:
    x_dim, u_dim, model, layers, MPC_type = 8, 5, "DBKN", [8, 64, 64, 64, 64, 24], "delta_mpc"


torch.manual_seed(0)
net = KoopmanBlinear(8, 5, Args.layers, False).double()
with torch.no_grad():
    net.H.weight.normal_(0.0, 0.02)
ctl = MPCController(net, Args())
lib = abi.load_lib()
prof = lib.sim_koopman_bl_profile
prof.argtypes = [C.c_void_p]
n, H = 4096, 10
rng = np.random.default_rng(0)
x = torch.as_tensor(np.concatenate([rng.uniform([0.1, -0.2, 0.0], [0.45, 0.2, 0.35], (n, 3)),
                                    rng.uniform(-1, 1, (n, 5))], 1).astype(np.float32), device=ctl.device)
win = torch.as_tensor(rng.normal(0, 0.3, (H, 32, n)), device=ctl.device)
up = torch.zeros((5, n), dtype=torch.float64, device=ctl.device)
out = np.zeros(9)
for it in range(4):
    ctl.step_bilinear(x, win, up)
    torch.cuda.synchronize()
    prof(out.ctypes.data)
names = ["z0 + B_total", "M_k / X_k", "rhs", "Gram (MFMA)", "Hessian", "Cholesky", "solves", "store"]
w = out[8]
res = {nm: out[k] / w for k, nm in enumerate(names)}
res["waves"] = w
res["total_cycles_per_wave"] = sum(out[:8]) / w
print(json.dumps(res, indent=1))
