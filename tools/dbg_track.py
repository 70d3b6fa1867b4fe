"""Debug: GPU env-step vs oracle from a reset state, with/without qfrc_applied, and the
tracking loop's first frame."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import soarm_pkg  # noqa
import torch
from oracle import Oracle
from lerobot_mujoco_sim2real_amd import mjcf
from lerobot_mujoco_sim2real_amd.sim import BatchSim

cm = mjcf.compile_mjcf(mjcf.SCENE_XML)
orc = Oracle(cm)
n = 64
rng = np.random.default_rng(0)
q0 = rng.uniform(-0.3, 0.3, (n, 5)).astype(np.float32)
a = rng.uniform(-0.5, 0.5, (n, 5)).astype(np.float32)
for mode in ("none", "zero", "bias"):
    S = BatchSim(cm, n)
    if mode != "none":
        S.enable_qfrc_applied()
    S.reset(init_qpos=q0, init_qvel=np.zeros_like(q0))
    st = orc.new_state(n)
    orc.reset(st, init_qpos=q0.astype(np.float64))
    ap = None
    if mode == "bias":
        S.bias(out=S.qfrc_applied)
        ap = orc.bias(st)
        print("bias gpu", S.qfrc_applied[:, 0].cpu().numpy(), "orc", ap[0])
    elif mode == "zero":
        ap = np.zeros((n, cm.nv))
    og = S.step(a).cpu().numpy()
    oc = orc.step(st, a.astype(np.float64), applied=ap)
    e = np.abs(og - oc)
    print(mode, "median", np.median(e), "max", e.max())
    print("  gpu", og[0], "\n  orc", oc[0])
