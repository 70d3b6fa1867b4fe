import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import soarm_pkg  # noqa: E402,F401  (registers lerobot_mujoco_sim2real_amd)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


@pytest.fixture(scope="session")
def arm_model():
    from lerobot_mujoco_sim2real_amd import mjcf
    return mjcf.compile_mjcf(mjcf.SCENE_XML)


@pytest.fixture(scope="session")
def arm_model_nocontact():
    from lerobot_mujoco_sim2real_amd import mjcf
    return mjcf.compile_mjcf(mjcf.SCENE_XML, disable_contact=True)


@pytest.fixture(scope="session")
def cube_model():
    from lerobot_mujoco_sim2real_amd import mjcf
    return mjcf.compile_mjcf(mjcf.CUBE_SCENE_XML)


@pytest.fixture(scope="session")
def gpu_lib():
    """Build (if stale) and load the HIP library; only for gpu-marked tests."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lerobot_mujoco_sim2real_amd import abi, build
    build.build()
    return abi.load_lib()


def cube_qpos(cm, n, rng, arm_q=None):
    """Build-defined pick-scene pose: cube on the table near the EE workspace
    at (0.25 +- 0.05, +-0.05, -0.0009 + 0.015)."""
    q = np.tile(cm.qpos0(), (n, 1))
    if arm_q is not None:
        q[:, :arm_q.shape[1]] = arm_q
    q[:, 6] = 0.25 + rng.uniform(-0.05, 0.05, n)
    q[:, 7] = rng.uniform(-0.05, 0.05, n)
    q[:, 8] = -0.0009 + 0.015
    return q


def limit_qpos0_model(margin=0.05, inside=0.02):
    """The pick scene with qpos0 of the shoulder-lift hinge inside its lower limit's margin (qpos0 =
    range[0] + `inside`, jnt_margin = `margin`): a soft reset (mj_checkPos/Vel/Acc -> mj_resetData)
    lands on an active joint-limit row, with the cube's resting contacts on the table."""
    from lerobot_mujoco_sim2real_amd import mjcf
    cm = mjcf.compile_mjcf(mjcf.CUBE_SCENE_XML, ccd="mpr")
    j = 1
    cm.desc.jnt_margin[j] = margin
    cm.desc.qpos0[j] = cm.desc.jnt_range[j][0] + inside
    # the cube's qpos0 rests exactly on the table (distance -2e-18 in fp64, >= 0 in fp32: a grazing
    # tie); 0.1 mm lower it penetrates in both precisions, so the reset pose has 4 contacts
    cm.desc.qpos0[cm.nq - 5] -= 1e-4
    return cm


def soft_reset_states(cm, orc, n, bad, steps=5, seed=0):
    """Oracle states of the pick scene after `steps` chirp env-steps (fp32-rounded), with qvel of the
    envs `bad` set to NaN so the next substep soft-resets them (mj_checkVel)."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    ids = np.arange(n)
    st = orc.new_state(n)
    q = W.initial_qpos(cm, ids, seed)
    orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
    tab = W.chirp_tables(ids, seed)
    for t in range(steps):
        orc.step(st, W.chirp_action(tab, t), nthreads=8)
    st = {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}
    st["qvel"][bad, 2] = np.nan
    return st


def fp32_noise_envelope(orc, st, action, params=None, kulp=8, trials=2, seed=0, nthreads=8):
    """Per-env qvel envelope of one env-step from the state st, from the fp64 oracle alone: the
    oracle stepped substep by substep with its state (qpos, qvel, warm start) rounded to fp32 and
    moved by a random +-kulp fp32 ulps per component after every substep -- fp32-sized arithmetic
    noise injected where the device's own arithmetic injects it -- `trials` times; the largest
    deviation from the unperturbed oracle env-step, per env and dof [n, nv].

    Why ulps and not the state rounding alone: the device's one-substep error from a common start is
    a few fp32 ulps of qvel (tools/env_diverge.py: 3e-8 .. 1.3e-7 on the headline's t = 100 states),
    and the velocity servo (h kv / M ~ 3) amplifies it over the 10 substeps; rounding moves each
    component by at most half an ulp.  (no library code in the reference's envelope.)"""
    rng = np.random.default_rng(seed)
    ref = {k: v.copy() for k, v in st.items()}
    orc.step(ref, action, params=params, nthreads=nthreads)
    out = np.zeros_like(st["qvel"])
    for _ in range(trials):
        c = {k: v.copy() for k, v in st.items()}
        for sub in range(10):
            orc.step(c, action if sub == 0 else None, nsub=1, params=params, nthreads=nthreads)
            for k in ("qpos", "qvel", "warm"):
                x = c[k].astype(np.float32)
                u = np.spacing(np.abs(x)).astype(np.float64)
                c[k][:] = x.astype(np.float64) + rng.integers(-kulp, kulp + 1, x.shape) * u
        out = np.maximum(out, np.abs(c["qvel"] - ref["qvel"]))
    return out
