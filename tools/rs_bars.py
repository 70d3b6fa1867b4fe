#!/usr/bin/env python3
"""Diagnostic: the measurements behind the contact parity bars of tests/test_gpu_parity.py, on the
kernel the library runs (SOARM_RS selects row-space / quad).  Prints JSON:
  * pgs_vs_oracle_pgs: device PGS vs the fp64 oracle's mj_solPGS, one substep from bench states
    (t = 20, 120; 4096 envs), qvel error percentiles over block-only and arm-contact envs;
  * pgs_vs_exact_newton: the same device substep against the exact optimum (oracle Newton, tol 0);
  * env_step: one graph-captured 10-substep env-step from t = 100 states against the oracle, with
    the fp32 re-rounding envelope (oracle 10 x (1 substep + state rounded to fp32)) per env."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from oracle import Oracle  # noqa: E402
from test_gpu_parity import _bench_states, make_sim, load_state, to_np  # noqa: E402

N = int(os.environ.get("ENVS", 4096))


def pct(e):
    e = np.asarray(e)
    if e.size == 0:
        return None
    return {"n": int(e.size), "p50": float(np.median(e)), "p99": float(np.percentile(e, 99)), "max": float(e.max())}


def arm_mask(cm, orc, st, n):
    names = cm.geom_names
    table, cube = names.index("table"), names.index("cube")
    return np.array([any({int(c[7]), int(c[8])} != {table, cube} for c in
                         orc.forward(st["qpos"][i], st["qvel"][i], st["ctrl"][i], st["warm"][i])["contacts"])
                     for i in range(n)])


out = {}
for t0 in (20, 120):
    cm, orc, st, _ = _bench_states("contact", N, t0, nthreads=16)
    S = make_sim(cm, N)
    load_state(S, st)
    S.substeps(1)
    gq = to_np(S.qvel).T
    arm = arm_mask(cm, orc, st, N)
    pg = {k: v.copy() for k, v in st.items()}
    orc.step(pg, None, nsub=1, nthreads=16)
    ex = {k: v.copy() for k, v in st.items()}
    Oracle(cm, solver="newton", tolerance=0.0).step(ex, None, nsub=1, nthreads=16)
    r = {"n_arm_envs": int(arm.sum())}
    for nm, ref in (("pgs_vs_oracle_pgs", pg), ("pgs_vs_exact_newton", ex), ("oracle_pgs_vs_exact_newton", None)):
        dv = np.abs((gq if ref is not None else pg["qvel"]) - (ref["qvel"] if ref is not None else ex["qvel"]))
        r[nm] = {"block_cube": pct(dv[~arm, 6:].max(1)), "block_arm": pct(dv[~arm, :6].max(1)),
                 "arm_cube": pct(dv[arm, 6:].max(1)), "arm_arm": pct(dv[arm, :6].max(1)), "all": pct(dv.max(1))}
    out[f"substep_t{t0}"] = r
    print(t0, json.dumps(r), flush=True)

from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
cm, orc, st, _ = _bench_states("contact", N, 100, nthreads=16)
a = W.chirp_action(W.chirp_tables(np.arange(N)), 100).astype(np.float32)
S = make_sim(cm, N)
st["ncon"][:] = 0
load_state(S, st)
og = to_np(S.step(a))
b = {k: v.copy() for k, v in st.items()}
oc = orc.step(st, a.astype(np.float64), nthreads=16)
ob = orc.step(b, a.astype(np.float64), nsub=1, nthreads=16)
for _ in range(9):
    for k in ("qpos", "qvel", "warm"):
        b[k][:] = b[k].astype(np.float32)
    ob = orc.step(b, None, nsub=1, nthreads=16)
dv = np.abs(to_np(S.qvel).T - st["qvel"])
env = np.abs(b["qvel"] - st["qvel"])
ratio = dv.max(1) / (env.max(1) + 1e-12)
out["env_step_t100"] = {"obs": pct(np.abs(og - oc).max(1)), "cube_qvel": pct(dv[:, 6:].max(1)),
                        "arm_qvel": pct(dv[:, :6].max(1)), "envelope_arm": pct(env[:, :6].max(1)),
                        "envelope_cube": pct(env[:, 6:].max(1)), "err_over_envelope": pct(ratio),
                        "worst_excess_arm": float((dv[:, :6].max(1) - 10 * env[:, :6].max(1)).max()),
                        "worst_excess_cube": float((dv[:, 6:].max(1) - 10 * env[:, 6:].max(1)).max())}
print("env_step", json.dumps(out["env_step_t100"]), flush=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"rs_bars_rs{os.environ.get('SOARM_RS', '1')}.json"), "w"), indent=1)
