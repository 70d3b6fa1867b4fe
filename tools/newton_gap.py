#!/usr/bin/env python3
"""How far the PGS solve (the kernels', and the oracle's restatement of mj_solPGS) lands from
the solution the reference computes: MuJoCo's default primal Newton solver (the reference scene
has no <option>, SOARM101/SO101/scene_with_table_v.xml:1-32, so SOARM101_Env.py:131-132 runs
Newton with tolerance 1e-8).

States: the headline bench workload (pick scene, chirp inputs, 4096 envs) after t = 20 and
t = 120 env-steps of the fp64 oracle, rounded to fp32.  From every state:
  * one substep: exact Newton optimum (oracle, tolerance 0) = the reference point; MuJoCo's
    Newton at tolerance 1e-8; the oracle's PGS (fp64); the device's PGS (fp32, if a GPU is
    present) -> qvel after the substep and qacc (= qacc_warmstart after it);
  * one env-step (10 substeps, graph-captured sim_step on the device): obs, qvel;
  * per-contact normal forces (sum of the 4 pyramid edges), PGS vs Newton (oracle).
Envs are split into "block" (only the cube's table contacts) and "arm" (any contact touching
an arm link).  Writes a JSON summary (default profiles/r03_newton_gap.json).

    python tools/newton_gap.py [--n 4096] [--out profiles/r03_newton_gap.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import soarm_pkg  # noqa: E402,F401
from oracle import Oracle  # noqa: E402
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402


def f32(st):
    return {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}


def bench_states(cm, n, steps, seed=0, nthreads=16):
    orc = Oracle(cm)
    ids = np.arange(n)
    st = orc.new_state(n)
    q = W.initial_qpos(cm, ids, seed)
    orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
    tab = W.chirp_tables(ids, seed)
    for t in range(steps):
        orc.step(st, W.chirp_action(tab, t), nthreads=nthreads)
    return f32(st), W.chirp_action(tab, steps)


def categories(cm, orc, st):
    names = cm.geom_names
    table, cube = names.index("table"), names.index("cube")
    arm = np.zeros(len(st["qpos"]), bool)
    for i in range(len(arm)):
        fw = orc.forward(st["qpos"][i], st["qvel"][i], st["ctrl"][i], st["warm"][i])
        arm[i] = any({int(c[7]), int(c[8])} != {table, cube} for c in fw["contacts"])
    return arm


def pct(x):
    x = np.asarray(x, np.float64).ravel()
    if x.size == 0:
        return None
    return {"p50": float(np.median(x)), "p99": float(np.percentile(x, 99)), "max": float(x.max()), "n": int(x.size)}


def one(orc, st, action=None, nsub=1, nthreads=16):
    s = {k: v.copy() for k, v in st.items()}
    obs = orc.step(s, action, nsub=nsub, nthreads=nthreads)
    return s, obs


def contact_forces(orc_a, orc_b, st, idx):
    """per-contact normal force (sum of the contact's 4 pyramid edges) under both solvers"""
    ea, rel = [], []
    for i in idx:
        fa = orc_a.forward(st["qpos"][i], st["qvel"][i], st["ctrl"][i], st["warm"][i])
        fb = orc_b.forward(st["qpos"][i], st["qvel"][i], st["ctrl"][i], st["warm"][i])
        nc = fa["ncon"]
        if nc == 0 or fb["ncon"] != nc:
            continue
        off = len(fa["efc_force"]) - 4 * nc
        na = fa["efc_force"][off:].reshape(nc, 4).sum(1)
        nb = fb["efc_force"][off:].reshape(nc, 4).sum(1)
        ea.append(np.abs(na - nb))
        rel.append(np.abs(na - nb) / np.maximum(np.abs(nb), 1e-3))
    return (np.concatenate(ea) if ea else np.zeros(0)), (np.concatenate(rel) if rel else np.zeros(0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--times", default="20,120")
    ap.add_argument("--nforce", type=int, default=512, help="envs whose contact forces are compared")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_newton_gap.json"))
    a = ap.parse_args()
    cm = W.model("contact")
    exact = Oracle(cm, solver="newton", tolerance=0.0)
    mjn = Oracle(cm, solver="newton")
    pgs = Oracle(cm)
    gpu = None
    try:
        import torch
        if torch.cuda.is_available():
            from lerobot_mujoco_sim2real_amd.sim import BatchSim
            gpu = BatchSim(cm, a.n)
    except Exception as e:  # noqa: BLE001
        print("no device leg:", e, file=sys.stderr)
    out = {"n": a.n, "workload": "contact (pick scene, chirp)", "model": {"meaninertia": cm.desc.meaninertia,
           "tolerance": cm.desc.tolerance, "iterations": cm.desc.iterations}, "times": {}}
    for T in [int(x) for x in a.times.split(",")]:
        t0 = time.time()
        st, act = bench_states(cm, a.n, T)
        arm = categories(cm, pgs, st)
        rec = {"arm_contact_envs": int(arm.sum()), "block_envs": int((~arm).sum())}
        ref, _ = one(exact, st)
        legs = {"newton_tol1e-8": one(mjn, st)[0], "pgs_fp64": one(pgs, st)[0]}
        refstep, refobs = one(exact, st, act, nsub=10)
        pstep, pobs = one(pgs, st, act, nsub=10)
        if gpu is not None:
            import torch
            dev = gpu.device
            def load(s):
                gpu.qpos.copy_(torch.as_tensor(s["qpos"].T, dtype=torch.float32, device=dev))
                gpu.qvel.copy_(torch.as_tensor(s["qvel"].T, dtype=torch.float32, device=dev))
                gpu.qacc_warmstart.copy_(torch.as_tensor(s["warm"].T, dtype=torch.float32, device=dev))
                gpu.ctrl.copy_(torch.as_tensor(s["ctrl"].T, dtype=torch.float32, device=dev))
                gpu.status.zero_()
            load(st)
            gpu.substeps(1)
            legs["pgs_device_fp32"] = {"qvel": gpu.qvel.double().cpu().numpy().T,
                                       "warm": gpu.qacc_warmstart.double().cpu().numpy().T}
            load(st)
            gobs = gpu.step(act.astype(np.float32)).double().cpu().numpy()
            gq = gpu.qvel.double().cpu().numpy().T
        for name, s in legs.items():
            r = {}
            for cat, m in (("block", ~arm), ("arm", arm)):
                dv = np.abs(s["qvel"] - ref["qvel"])[m]
                dq = np.abs(s["warm"] - ref["warm"])[m]
                r[cat] = {"qvel_cube": pct(dv[:, 6:].max(1)), "qvel_arm": pct(dv[:, :6].max(1)),
                          "qacc_cube": pct(dq[:, 6:].max(1)), "qacc_arm": pct(dq[:, :6].max(1))}
            rec[f"substep_{name}_vs_exact_newton"] = r
        # the device against its own restatement (fp32 vs fp64 spread of the same solver)
        if gpu is not None:
            dv = np.abs(legs["pgs_device_fp32"]["qvel"] - legs["pgs_fp64"]["qvel"])
            rec["substep_pgs_device_vs_pgs_fp64"] = {"qvel_cube": pct(dv[:, 6:].max(1)),
                                                    "qvel_arm": pct(dv[:, :6].max(1))}
        stepr = {"pgs_fp64": {"obs": pct(np.abs(pobs - refobs).max(1)),
                              "qvel_cube": pct(np.abs(pstep["qvel"] - refstep["qvel"])[:, 6:].max(1))}}
        if gpu is not None:
            stepr["pgs_device_fp32"] = {"obs": pct(np.abs(gobs - refobs).max(1)),
                                        "qvel_cube": pct(np.abs(gq - refstep["qvel"])[:, 6:].max(1))}
            stepr["pgs_device_vs_pgs_fp64"] = {"obs": pct(np.abs(gobs - pobs).max(1)),
                                               "qvel_cube": pct(np.abs(gq - pstep["qvel"])[:, 6:].max(1))}
        rec["env_step_vs_exact_newton"] = stepr
        idx = list(np.nonzero(arm)[0][: a.nforce // 2]) + list(np.nonzero(~arm)[0][: a.nforce // 2])
        ea, rel = contact_forces(pgs, exact, st, idx)
        rec["contact_normal_force_pgs_vs_newton"] = {"abs_N": pct(ea), "rel": pct(rel)}
        rec["seconds"] = time.time() - t0
        out["times"][str(T)] = rec
        print(json.dumps({T: rec}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
