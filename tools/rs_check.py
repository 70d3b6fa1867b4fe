#!/usr/bin/env python3
"""Diagnostic: one substep and one 10-substep env-step from oracle bench states (contact workload,
PGS) on the GPU with the row-space kernel (SOARM_RS=1) and the quad kernel (SOARM_RS=0), against the
fp64 oracle's mj_solPGS restatement; qvel error percentiles over block-only envs (the cube's resting
contacts only) and arm-contact envs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from test_gpu_parity import _bench_states, make_sim, load_state, to_np  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096


def pct(e):
    return f"p50 {np.median(e):.2e} p99 {np.percentile(e, 99):.2e} max {e.max():.2e}"


for t in (20, 120):
    cm, orc, st0, _ = _bench_states("contact", N, t, nthreads=16)
    st = {k: v.copy() for k, v in st0.items()}
    st["ncon"][:] = 0
    orc.step(st, None, nsub=1)
    arm = st["ncon"] > 4
    for rs in ("1", "0"):
        os.environ["SOARM_RS"] = rs
        S = make_sim(cm, N)
        s = {k: v.copy() for k, v in st0.items()}
        load_state(S, s)
        S.substeps(1)
        dv = np.abs(to_np(S.qvel).T - st["qvel"])
        dq = np.abs(to_np(S.qpos).T - st["qpos"]).max()
        print(f"t={t} rs={rs} n_arm={int(arm.sum())} qpos max {dq:.2e}", flush=True)
        for nm, msk in (("block", ~arm), ("arm-contact", arm)):
            if msk.any():
                print(f"   {nm:12s} cube qvel {pct(dv[msk, 6:].max(1))} | arm qvel {pct(dv[msk, :6].max(1))}", flush=True)
