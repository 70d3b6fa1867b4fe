"""Synthetic workloads of BASELINE.json ``configs``.

Every random draw is Philox4x32-10 keyed by (seed, global env id), so the
same env gets the same initial state, inputs and DR parameters whether the
batch runs on 1 or 8 GPUs.

* ``plumbing`` (config 1): one env of the reference scene, zero action, qpos ~ U(-0.3, 0.3)^5
  (``SOARM101_Env.py:77-142`` driven by hand); its CPU leg is the oracle on one core.
* ``nocontact`` (config 2): arm on the table, collision disabled (frictionloss
  and joint limits on), qpos ~ U(-0.3, 0.3)^5, random actions U[-0.5, 0.5)^5
  every env-step (``SOARM101_DataCollection.py:132``).
* ``contact`` (config 3, the headline): build-defined pick scene — the cube
  (half-size 0.015 m, 0.03 kg) rests on the table at (0.25 +- 0.05, +-0.05);
  arm starts U(-0.3, 0.3)^5; chirp actions (``SineInputGenerator`` mode
  "chirp", tables drawn per env, ``:31-74``); contacts via PGS.
* ``dr`` (config 4): ``contact`` + per-env domain randomisation: body mass
  x U(0.8, 1.2) (inertia scaled alike), sliding friction U(0.5, 1.5), dof
  damping x U(0.8, 1.2).
* ``rollout`` (config 5, build-defined extension ii of SURVEY.md §8a): the
  reference scene (arm + table, contacts on); each env follows a Fig8 path
  (``control/TrajectoryGenerator.py:138-152``) with a per-env phase; every
  env-step runs position-only DLS IK (warm-started) and applies
  ``clip((q* - q) / dt, +-max_speed)`` (``SOARM101_Env.py:57``); rows
  ``[u(5) | ee(3) | q(5)]`` as in ``SOARM101_DataCollection.py:106-134``.
* ``mpc``: the reference's Koopman-MPC tracking loop
  (``Koopman_MPC.py:110-136,197-222``) for every env: a Fig8 reference per env (per-env phase)
  with joint angles from warm-started DLS IK (``control/TrajectoryGenerator.py:180-205``), a
  random-init DKUC Koopman model (``models/KoopmanBase.py``), delta-MPC with H = 10, gravity
  compensation ``qfrc_applied = qfrc_bias``.
"""
import numpy as np

from .mjcf import CUBE_SCENE_XML, SCENE_XML, compile_mjcf
from .sim import philox4x32

CONFIGS = {
    "plumbing": dict(xml=SCENE_XML, disable_contact=False, action="zero", dr=False, envs=1,
                     desc="1 SO-ARM101 env, reference scene (arm + table, contacts on), zero action "
                          "(config 1: SOARM101_Env plumbing)"),
    "nocontact": dict(xml=SCENE_XML, disable_contact=True, action="random", dr=False,
                      desc="4096 SO-ARM101 envs, contact-free arm dynamics (config 2)"),
    "contact": dict(xml=CUBE_SCENE_XML, disable_contact=False, action="chirp", dr=False,
                    desc="4096 SO-ARM101 envs, tabletop+cube contacts, PGS (config 3, pick scene)"),
    "dr": dict(xml=CUBE_SCENE_XML, disable_contact=False, action="chirp", dr=True, envs=8192,
               desc="SO-ARM101 pick scene with per-env mass/friction/damping DR (config 4)"),
    "rollout": dict(xml=SCENE_XML, disable_contact=False, action="ik_fig8", dr=False,
                    desc="SOARM101_DataCollection rollout: batched DLS-IK actions toward Fig8 targets, "
                         "rows [T+1, N, 13] on device, gathered to rank 0 (config 5)"),
    "mpc": dict(xml=SCENE_XML, disable_contact=False, action="koopman_mpc", dr=False,
                desc="Koopman-MPC Fig8 tracking (Koopman_MPC.py loop, SURVEY 8f rank 2): per env and frame "
                     "gravity compensation + f64 MFMA encoder/MPC + env step, 4096 envs"),
    "mpc_dbkn": dict(xml=SCENE_XML, disable_contact=False, action="koopman_mpc", dr=False, koopman="DBKN",
                     desc="Koopman-MPC Fig8 tracking with the bilinear DBKN model: per env and frame its QP "
                          "linearised at the lifted state and solved in f64 on the device, 4096 envs"),
}


def philox_uniform(seed, ids, k):
    """[n, k] float32 uniforms in [0, 1) keyed by (seed, env id)."""
    ids = np.asarray(ids, dtype=np.uint64)
    key = (int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF)
    blocks = []
    for b in range((k + 3) // 4):
        ctr = np.stack([ids & 0xFFFFFFFF, ids >> np.uint64(32), np.full_like(ids, b), np.zeros_like(ids)], 1)
        blocks.append(philox4x32(ctr, key))
    r = np.concatenate(blocks, 1)[:, :k]
    return (r >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)


def keyed_uniform(seed, ids, counter, k, lo, hi):
    """Host mirror of ``sim_rand_uniform`` (bit-exact): [n, k] float32 lo + (hi - lo) u, u from
    Philox4x32-10 keyed by `seed`, counter (id, id >> 32, counter, 1 + j // 4)."""
    ids = np.asarray(ids, dtype=np.uint64)
    key = (int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF)
    blocks = []
    for b in range((k + 3) // 4):
        ctr = np.stack([ids & 0xFFFFFFFF, ids >> np.uint64(32), np.full_like(ids, int(counter) & 0xFFFFFFFF),
                        np.full_like(ids, 1 + b)], 1)
        blocks.append(philox4x32(ctr, key))
    r = np.concatenate(blocks, 1)[:, :k]
    u = (r >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)
    lo32 = np.float32(lo)
    return lo32 + (np.float32(hi) - lo32) * u


# the bench workloads' narrowphase: libccd MPR, labelled in every bench line (`bench.py --ccd`);
# the library's own default is native GJK/EPA (mjcf.compile_mjcf), what current MuJoCo runs
BENCH_CCD = "mpr"


def model(name, **kw):
    c = CONFIGS[name]
    kw.setdefault("ccd", BENCH_CCD)
    return compile_mjcf(c["xml"], disable_contact=c["disable_contact"], **kw)


def initial_qpos(cm, ids, seed=0):
    """Full qpos [n, nq] float32: arm U(-0.3, 0.3)^5 (gripper 0), cube resting on the table."""
    n = len(ids)
    q = np.tile(cm.qpos0().astype(np.float32), (n, 1))
    q[:, :5] = -0.3 + 0.6 * philox_uniform(seed, ids, 5)
    if cm.nq > 6:
        u = philox_uniform(seed + 1, ids, 2)
        q[:, 6] = 0.25 + 0.1 * (u[:, 0] - 0.5)
        q[:, 7] = 0.1 * (u[:, 1] - 0.5)
        q[:, 8] = -0.0009 + 0.015
    return q


def chirp_tables(ids, seed=0, udim=5, freq_range=(0.0025, 0.05), amp_range=(-0.5, 0.5)):
    u = philox_uniform(seed + 2, ids, 3 * udim).astype(np.float64)
    f = freq_range[0] + (freq_range[1] - freq_range[0]) * u[:, :udim]
    a = amp_range[0] + (amp_range[1] - amp_range[0]) * u[:, udim:2 * udim]
    p = 2 * np.pi * u[:, 2 * udim:]
    return dict(freq=f, amp=a, phase=p, freq_start=freq_range[0], freq_end=freq_range[1])


def chirp_action(tab, t, lib=np, T_total=200):
    """u = amp sin(2 pi (f + (f_end - f_start) t / T) t + phase)  (SineInputGenerator 'chirp')."""
    f = tab["freq"] + (tab["freq_end"] - tab["freq_start"]) * (t / T_total)
    return tab["amp"] * lib.sin(2 * np.pi * f * t + tab["phase"])


def dr_params(ids, seed=0):
    u = philox_uniform(seed + 3, ids, 3)
    return dict(mass_scale=0.8 + 0.4 * u[:, 0], friction=0.5 + 1.0 * u[:, 1], damping_scale=0.8 + 0.4 * u[:, 2])


def ik_phase(ids, seed=0):
    """Per-env phase of the Fig8 target stream (config 5)."""
    return 2 * np.pi * philox_uniform(seed + 4, ids, 1)[:, 0].astype(np.float64)


def fig8_targets(t, phase, lib=np):
    """Fig8 target of env-step t (``TrajectoryGenerator.py:138-152``, idx 1, scale 0.5):
    parameter 1.6 + 0.02 (t + 1) + phase."""
    tp = 1.6 + 0.02 * (t + 1) + phase
    one = lib.ones_like(tp)
    s, c = lib.sin(tp), lib.cos(tp)
    a = b = 0.2 * 0.5
    return lib.stack([0.4 * one, b * c / (1 + s ** 2), 0.2 + 2 * a * s * c / (1 + s ** 2)], -1)


def ik_action(qstar, q, dt=0.02, max_speed=0.5, lib=np):
    """action = clip((q* - q) / dt, +-max_speed) over the 5 arm joints."""
    return lib.clip((qstar - q) / dt, -max_speed, max_speed)


def reference_trajectory(sim, phase, T, lib=None):
    """Per-env Fig8 reference [T, n, 3] and its joint angles [T, n, 5] by warm-started DLS IK,
    repeating the previous solution where a point fails (control/TrajectoryGenerator.py:180-205).
    phase: [n] device tensor; runs on sim's device."""
    import torch
    q = sim.qpos.clone()
    cart, joints = [], []
    prev = q[:5].clone()
    for t in range(T):
        tgt = fig8_targets(float(t) - 1.0, phase, lib=torch)  # parameter 1.6 + 0.02 t + phase
        last = q.clone()
        qn, ok, _ = sim.ik(tgt, q=q)  # warm start, updated in place
        good = ok.bool()
        q = torch.where(good[None], qn, last)
        prev = torch.where(good[None], q[:5], prev)
        cart.append(tgt.float())
        joints.append(prev.T.clone())
    return torch.stack(cart), torch.stack(joints)
