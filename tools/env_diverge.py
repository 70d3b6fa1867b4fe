#!/usr/bin/env python3
"""Substep-by-substep anatomy of an env whose fp32 env-step leaves the fp64 oracle by more than
state rounding explains (env 2624 of the headline's t = 100 bench states).

For the given envs of a bench workload, from the oracle's fp32-rounded state at env-step t0, it
runs the 10 substeps of one env-step three ways -- the fp64 oracle, the fp64 oracle re-rounded to
fp32 after every substep, and the library (the CPU backend, device = -1, by default; --gpu for the
device) one substep at a time from the SAME start -- and prints per substep: contacts (pair ids) on
each side, the actuator force / clamp state of every arm joint, qacc, qvel, and the library's gap.
It also re-runs the oracle from the library's own state before each substep (one-substep gap with a
common start), which separates "this substep's arithmetic" from "inherited from earlier substeps".

    python tools/env_diverge.py [--config contact] [--t0 100] [--envs 2624,415] [--gpu] [--json out]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="contact")
    p.add_argument("--t0", type=int, default=100)
    p.add_argument("--envs", default="2624")
    p.add_argument("--gpu", action="store_true")
    p.add_argument("--json", default=None)
    p.add_argument("--quiet", action="store_true")
    a = p.parse_args()
    import torch
    import soarm_pkg  # noqa: F401
    from oracle import Oracle
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim

    ids = np.array([int(x) for x in a.envs.split(",")])
    n = len(ids)
    cm = W.model(a.config)
    orc = Oracle(cm)
    st = orc.new_state(n)
    q = W.initial_qpos(cm, ids)
    orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
    tab = W.chirp_tables(ids)
    prm = None
    if W.CONFIGS[a.config]["dr"]:
        pp = W.dr_params(ids)
        prm = np.stack([pp["mass_scale"], pp["friction"], pp["damping_scale"]], 1).astype(np.float32).astype(np.float64)
    for t in range(a.t0):
        orc.step(st, W.chirp_action(tab, t), params=prm)
    st = {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}
    act = W.chirp_action(tab, a.t0).astype(np.float32).astype(np.float64)
    d = cm.desc
    names = cm.geom_names

    S = BatchSim(cm, n, 0 if a.gpu else -1)
    if prm is not None:
        S.set_params(mass_scale=prm[:, 0], friction=prm[:, 1], damping_scale=prm[:, 2])
    dev = S.qpos.device

    def load(sim, s):
        sim.qpos.copy_(torch.as_tensor(s["qpos"].T, dtype=torch.float32, device=dev))
        sim.qvel.copy_(torch.as_tensor(s["qvel"].T, dtype=torch.float32, device=dev))
        sim.qacc_warmstart.copy_(torch.as_tensor(s["warm"].T, dtype=torch.float32, device=dev))
        sim.ctrl.copy_(torch.as_tensor(s["ctrl"].T, dtype=torch.float32, device=dev))
        sim.status.zero_()

    def lib_state(sim):
        g = lambda t: t.detach().cpu().numpy().astype(np.float64).T.copy()
        return dict(qpos=g(sim.qpos), qvel=g(sim.qvel), warm=g(sim.qacc_warmstart), ctrl=g(sim.ctrl),
                    status=np.zeros(n, np.int32), ncon=np.zeros(n))

    # the action enters ctrl before substep 0 (sim_step copies it in), so set ctrl directly
    o64 = {k: v.copy() for k, v in st.items()}
    orr = {k: v.copy() for k, v in st.items()}
    load(S, st)
    na = act.shape[1]
    S.ctrl[:na].copy_(torch.as_tensor(act.T, dtype=torch.float32, device=dev))
    o64["ctrl"][:, :na] = act
    orr["ctrl"][:, :na] = act
    rows = []
    for sub in range(10):
        before = lib_state(S)
        fw_lib = [orc.forward(before["qpos"][i], before["qvel"][i], before["ctrl"][i], before["warm"][i]) for i in range(n)]
        fw_o = [orc.forward(o64["qpos"][i], o64["qvel"][i], o64["ctrl"][i], o64["warm"][i]) for i in range(n)]
        S.substeps(1)
        if a.gpu:
            torch.cuda.synchronize()
        after = lib_state(S)
        # the oracle's own substep from the library's start state (a common start)
        common = {k: v.copy() for k, v in before.items()}
        orc.step(common, None, nsub=1, params=prm)
        orc.step(o64, None, nsub=1, params=prm)
        orc.step(orr, None, nsub=1, params=prm)
        for k in ("qpos", "qvel", "warm"):
            orr[k][:] = orr[k].astype(np.float32)
        for i in range(n):
            cl = [(int(c[7]), int(c[8])) for c in fw_lib[i]["contacts"]]
            co = [(int(c[7]), int(c[8])) for c in fw_o[i]["contacts"]]
            # velocity servo: force = gain * ctrl - kv * qvel, clamped to forcerange (soarm_step.h)
            gain = np.array([d.actuator_gainprm[k] for k in range(d.nu)])
            kv = np.array([d.actuator_biasprm[k][2] for k in range(d.nu)])
            fr = np.array([[d.actuator_forcerange[k][0], d.actuator_forcerange[k][1]] for k in range(d.nu)])
            def act_force(s):
                f = gain * np.clip(s["ctrl"][i], -2, 2) + kv * s["qvel"][i][: d.nu]
                return f, (f <= fr[:, 0]) | (f >= fr[:, 1])
            fl, cl_lib = act_force(before)
            row = dict(
                env=int(ids[i]), sub=sub,
                contacts_lib=[(names[x], names[y]) for x, y in cl], contacts_o64_same=cl == co,
                act_force_lib=fl.round(4).tolist(), act_clamped_lib=cl_lib.astype(int).tolist(),
                qacc_lib=after["warm"][i].tolist(), qacc_common=common["warm"][i].tolist(),
                qvel_gap_vs_o64=float(np.abs(after["qvel"][i] - o64["qvel"][i])[:6].max()),
                qvel_gap_rounded_vs_o64=float(np.abs(orr["qvel"][i] - o64["qvel"][i])[:6].max()),
                qvel_gap_common=float(np.abs(after["qvel"][i] - common["qvel"][i])[:6].max()),
                qacc_gap_common=float(np.abs(after["warm"][i] - common["warm"][i])[:6].max()),
                cube_qvel_gap_common=float(np.abs(after["qvel"][i] - common["qvel"][i])[6:].max()) if d.nv > 6 else 0.0,
                ncon_lib=len(cl), ncon_o64=len(co))
            rows.append(row)
            if not a.quiet:
                print(f"env {row['env']} sub {sub}: ncon lib {len(cl)} o64 {len(co)} same-set {cl == co} | "
                      f"arm qvel gap vs o64 {row['qvel_gap_vs_o64']:.2e} (rounded-oracle {row['qvel_gap_rounded_vs_o64']:.2e}) "
                      f"| one-substep gap, common start: qvel {row['qvel_gap_common']:.2e} qacc {row['qacc_gap_common']:.2e} "
                      f"cube {row['cube_qvel_gap_common']:.2e} | clamp {row['act_clamped_lib']} | {row['contacts_lib']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
