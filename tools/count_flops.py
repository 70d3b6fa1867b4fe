"""Freeze the algorithmic cost per env-step (SURVEY.md §8d binding procedure).

Runs the instrumented float64 oracle on a sample of each bench workload and
writes profiles/algorithmic_cost.json: flops per env-step (total, collision
share, dynamics share) and the algorithmic HBM bytes per env-step.  bench.py
computes every roofline fraction from this frozen file.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from oracle import Oracle  # noqa: E402

N, T = 256, 60  # envs x env-steps sampled per workload


def state_bytes(cm, dr):
    # read qpos, qvel, warmstart, ctrl(nu) + action(5); write qpos, qvel, warmstart, ctrl, obs(8); fp32
    b = 4 * (2 * cm.nq + 4 * cm.nv + 2 * cm.nu + 5 + 8 + 1)
    return b + (4 * 3 if dr else 0)


def mpc_net(seed=0):
    """The bench's random-init DKUC model (bench.py: torch.manual_seed(seed))."""
    import torch
    from lerobot_mujoco_sim2real_amd.control.koopman import Koopmanlinear
    from lerobot_mujoco_sim2real_amd.args import Args
    torch.manual_seed(seed)
    a = Args()
    return Koopmanlinear(a.x_dim, a.u_dim, a.layers).double()


def main():
    args = sys.argv[1:]
    solver = "pgs"
    if "--solver" in args:
        i = args.index("--solver")
        solver = args[i + 1]
        del args[i:i + 2]
    only = args
    path = os.path.join(ROOT, "profiles", "algorithmic_cost.json")
    out = json.load(open(path)) if only else {}
    for name, c in W.CONFIGS.items():
        if only and name not in only:
            continue
        cm = W.model(name, solver=solver)
        orc = Oracle(cm)
        ids = np.arange(N)
        st = orc.new_state(N)
        q = W.initial_qpos(cm, ids)
        orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
        tab = W.chirp_tables(ids)
        prm = None
        if c["dr"]:
            p = W.dr_params(ids)
            prm = np.stack([p["mass_scale"], p["friction"], p["damping_scale"]], 1).astype(np.float64)
        rng = np.random.default_rng(0)
        tot = col = 0.0
        phase, qstar = W.ik_phase(ids), q.astype(np.float64)
        if c["action"] == "koopman_mpc":  # the tracking loop: physics with qfrc_applied = qfrc_bias
            import koopman_mpc as KO
            net = mpc_net()
            A, B = net.lA.weight.detach().numpy(), net.lB.weight.detach().numpy()
            layers = net.encoder_layers()
            cart = np.stack([W.fig8_targets(t - 1.0, phase) for t in range(T)])
            sref = np.concatenate([cart, np.repeat(q[None, :, :5], T, 0)], -1)  # joint refs: start pose
            zref = KO.encode(layers, sref.reshape(T * N, 8)).reshape(T, N, -1)
            x, up = sref[0], np.zeros((N, 5))
        for t in range(T):
            if c["action"] == "koopman_mpc":
                u0, a = KO.get_control(A, B, KO.encode(layers, x), KO.lifted_window(zref, t, 10), up)
                up = u0
                obs = orc.step(st, a, nthreads=8, applied=orc.bias(st))
                x = obs.astype(np.float32).astype(np.float64)
                tot += orc.last_flops
                col += orc.last_collision_flops
                continue
            if c["action"] == "chirp":
                a = W.chirp_action(tab, t)
            elif c["action"] == "ik_fig8":  # IK flops are not counted: physics only
                qstar, _, _ = orc.ik(W.fig8_targets(t, phase), qstar)
                a = W.ik_action(qstar[:, :5], st["qpos"][:, :5])
            elif c["action"] == "zero":
                a = np.zeros((N, 5))
            else:
                a = rng.uniform(-0.5, 0.5, (N, 5))
            orc.step(st, a, params=prm, nthreads=8)
            tot += orc.last_flops
            col += orc.last_collision_flops
        fs = 10
        key = name if solver == "pgs" else f"{name}_{solver}"
        out[key] = dict(
            flops_per_env_step=tot / (N * T),
            collision_flops_per_env_step=col / (N * T),
            dynamics_flops_per_env_step=(tot - col) / (N * T),
            flops_per_env_substep_collision=col / (N * T * fs),
            flops_per_env_substep_dynamics=(tot - col) / (N * T * fs),
            contacts_per_env_substep=float(st["ncon"].sum() / (N * T * fs)),
            hbm_bytes_per_env_step=state_bytes(cm, c["dr"]),
            sample=f"{N} envs x {T} env-steps, oracle float64, seed 0",
        )
        out[key]["solver"] = solver
        if c["action"] == "koopman_mpc":
            # per env and frame: encoder 2 sum(in*out) + control 2 u (nz + u), counted from the widths
            ws = [l[0].shape for l in layers]
            enc = 2.0 * sum(o * i for o, i in ws)
            out[key]["mpc_flops_per_env_step"] = enc + 2.0 * 5 * (32 + 5)
            out[key]["mpc_note"] = ("encoder + [Gz|Gu] per env-step (f64 MFMA, k_mpc_step); the physics "
                                     "share above is the arm scene with gravity compensation")
        print(key, json.dumps(out[key]))
    json.dump(out, open(path, "w"), indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
