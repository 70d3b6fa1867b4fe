"""The library's CPU backend (sim_batch_create(..., device = -1, ...)) against
the float64 oracle.  These run without a GPU: the same ABI, host buffers.

The backend runs the kernels' per-env code compiled for the host (soarm_step.h, soarm_collide.h,
soarm_env.h) and solves the constraint rows densely in MuJoCo's row order (soarm_cpu.hip), so
its bars are the device path's (tests/test_gpu_parity.py) at smaller sizes; where its PGS follows
the oracle's sweep order exactly the bars are tighter (stated per test)."""
import os

import numpy as np
import pytest

from conftest import cube_qpos, fp32_noise_envelope
from oracle import Oracle

RNG = np.random.default_rng(17)
QVEL_BARS = (2e-6, 3.5e-4, 2.5e-3)  # = test_gpu_parity.QVEL_BARS


@pytest.fixture(scope="module")
def cpu_lib():
    from lerobot_mujoco_sim2real_amd import abi, build
    build.build()
    return abi.load_lib()


def make_sim(cm, n):
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    return BatchSim(cm, n, -1)


def to_np(t):
    return t.detach().cpu().numpy().astype(np.float64)


def load_state(S, st):
    import torch
    S.qpos.copy_(torch.as_tensor(st["qpos"].T, dtype=torch.float32))
    S.qvel.copy_(torch.as_tensor(st["qvel"].T, dtype=torch.float32))
    S.qacc_warmstart.copy_(torch.as_tensor(st["warm"].T, dtype=torch.float32))
    S.ctrl.copy_(torch.as_tensor(st["ctrl"].T, dtype=torch.float32))
    S.status.zero_()


def f32(st):
    return {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}


def random_states(orc, n, steps=3, lo=-1.0, hi=1.0, rng=None):
    rng = RNG if rng is None else rng
    st = orc.new_state(n)
    orc.reset(st, init_qpos=rng.uniform(lo, hi, (n, 5)))
    for _ in range(steps):
        orc.step(st, rng.uniform(-0.5, 0.5, (n, 5)))
    return f32(st)


def assert_pct(err, p50, p99, mx, what=""):
    e = np.asarray(err, np.float64).ravel()
    got = (float(np.median(e)), float(np.percentile(e, 99)), float(e.max()))
    assert got[0] <= p50 and got[1] <= p99 and got[2] <= mx, (what, "p50/p99/max", got, "bars", (p50, p99, mx))


# envs of the headline workload (seed 0) with arm-table / arm-cube contacts at env-step 100
# (found with the CPU backend over all 4096 envs; 13 of them)
ARM_CONTACT_ENVS_T100 = [415, 562, 1174, 1560, 1812, 2023, 2235, 2589, 2624, 2982, 3205, 3505, 3815]


def bench_states(name, ids, steps, seed=0, solver=None):
    """Oracle states of envs `ids` of a bench workload after `steps` env-steps, fp32-rounded."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    cm = W.model(name) if solver is None else W.model(name, solver=solver)
    orc = Oracle(cm)
    ids = np.asarray(ids)
    n = len(ids)
    st = orc.new_state(n)
    q = W.initial_qpos(cm, ids, seed)
    orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
    tab = W.chirp_tables(ids, seed)
    for t in range(steps):
        orc.step(st, W.chirp_action(tab, t), nthreads=8)
    return cm, orc, f32(st)


def test_cpu_batch_is_explicit(cpu_lib, arm_model):
    """device = -1 only when asked: a GPU ordinal never lands on the host path (it needs a GPU)."""
    import torch
    S = make_sim(arm_model, 4)
    assert S.cpu and S.qpos.device.type == "cpu"
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError):
            from lerobot_mujoco_sim2real_amd.sim import BatchSim
            BatchSim(arm_model, 4, 0)


def test_cpu_reset_matches_oracle(cpu_lib, arm_model, cube_model):
    from lerobot_mujoco_sim2real_amd.sim import reset_qpos_draw
    for cm in (arm_model, cube_model):
        n = 256
        S, orc = make_sim(cm, n), Oracle(cm)
        iq = RNG.uniform(-1.5, 1.5, (n, 5)).astype(np.float32)
        ex = cube_qpos(cm, n, RNG).astype(np.float32) if cm.nq > 6 else None
        og = to_np(S.reset(init_qpos=iq, extra_qpos=ex))
        st = orc.new_state(n)
        oc = orc.reset(st, init_qpos=iq.astype(np.float64), extra_qpos=ex)
        np.testing.assert_allclose(og, oc, atol=2e-6)
        np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=1e-7)
    S = make_sim(arm_model, 300)
    S.reset(seed=123456789, env_offset=5000)
    np.testing.assert_array_equal(S.qpos.numpy()[:5].T, reset_qpos_draw(123456789, np.arange(5000, 5300)))


def test_cpu_rand_uniform_matches_host_mirror(cpu_lib, arm_model):
    from lerobot_mujoco_sim2real_amd import workloads as W
    S = make_sim(arm_model, 200)
    d = S.rand_uniform(2 ** 40 + 3, 123, 9, 0.0, 2 * np.pi, env_offset=5000).numpy()
    np.testing.assert_array_equal(d, W.keyed_uniform(2 ** 40 + 3, np.arange(5000, 5200), 123, 9, 0.0, 2 * np.pi))


def test_cpu_one_substep_no_contact(cpu_lib, arm_model_nocontact):
    cm = arm_model_nocontact
    n = 256
    S, orc = make_sim(cm, n), Oracle(cm)
    st = random_states(orc, n)
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=2e-6)
    np.testing.assert_allclose(to_np(S.qvel).T, st["qvel"], atol=5e-4)
    assert (to_np(S.status) == st["status"]).all()


def test_cpu_bias_matches_oracle(cpu_lib, cube_model):
    cm = cube_model
    n = 128
    S, orc = make_sim(cm, n), Oracle(cm)
    st = orc.new_state(n)
    orc.reset(st, init_qpos=RNG.uniform(-1, 1, (n, 5)), extra_qpos=cube_qpos(cm, n, RNG))
    st["qvel"][:] = RNG.uniform(-1, 1, st["qvel"].shape)
    st = f32(st)
    load_state(S, st)
    np.testing.assert_allclose(to_np(S.bias()).T, orc.bias(st), atol=2e-5)


def _divergence(cm, n, T, rng):
    orc = Oracle(cm)
    iq = rng.uniform(-0.3, 0.3, (n, 5)).astype(np.float32).astype(np.float64)
    acts = rng.uniform(-0.5, 0.5, (T, n, 5)).astype(np.float32).astype(np.float64)
    a, b = orc.new_state(n), orc.new_state(n)
    orc.reset(a, init_qpos=iq)
    orc.reset(b, init_qpos=iq)
    dev = []
    for t in range(T):
        oa, ob = orc.step(a, acts[t]), orc.step(b, acts[t])
        for k in ("qpos", "qvel", "warm"):
            b[k][:] = b[k].astype(np.float32)
        dev.append(np.abs(oa - ob))
    return iq, acts, np.stack(dev)


def test_cpu_trajectory_shadowing(cpu_lib, arm_model_nocontact):
    """fp32 CPU backend vs fp64 oracle over 20 env-steps: within 10x the oracle's fp32 envelope."""
    cm = arm_model_nocontact
    n, T = 128, 20
    iq, acts, envelope = _divergence(cm, n, T, np.random.default_rng(3))
    S, orc = make_sim(cm, n), Oracle(cm)
    st = orc.new_state(n)
    S.reset(init_qpos=iq.astype(np.float32))
    orc.reset(st, init_qpos=iq)
    for t in range(T):
        e = np.abs(to_np(S.step(acts[t].astype(np.float32))) - orc.step(st, acts[t]))
        assert np.median(e) <= 10 * np.median(envelope[t]) + 1e-5, (t, np.median(e))
        assert np.quantile(e, 0.9) <= 10 * np.quantile(envelope[t], 0.9) + 2e-4


def _contact_poses(n, rng):
    q = np.zeros((n, 6))
    q[:, 0] = rng.uniform(-1.0, 1.0, n)
    q[:, 1] = rng.uniform(0.6, 1.6, n)
    q[:, 2] = rng.uniform(-0.5, 1.0, n)
    q[:, 3] = rng.uniform(0.3, 1.6, n)
    q[:, 4] = rng.uniform(-2.0, 2.0, n)
    q[:, 5] = rng.uniform(0.0, 1.5, n)
    half = n // 2
    q[half:, 1] = rng.uniform(-1.7, -1.3, n - half)
    q[half:, 2] = rng.uniform(1.3, 1.69, n - half)
    return q.astype(np.float32).astype(np.float64)


def contact_point_split(dp, normal):
    """Native GJK/EPA's contact point is its witness-point midpoint on the final polytope face;
    for a face-on-face contact (a link lying flat on the table) many nearly coplanar faces tie,
    so fp32 and fp64 can pick witness points centimetres apart WITHIN the contact patch, while
    depth and normal agree to ~1e-8 (measured on these poses: point offset along the normal
    p99 2.5e-7 / max 4.3e-7 m, across it p99 1.3e-2 / max 1.6e-2 m; the fp64 oracle itself jumps
    > 2 mm on 2 of 207 contacts under a 1-ulp fp32 qpos perturbation).  So the point must stay
    on the oracle's contact plane (|n . dp| <= 5e-6 m) and its slide within the plane is only
    counted (<= 15% of contacts beyond 2 mm, all within 3 cm: the patch size)."""
    along = abs(float(dp @ normal))
    tang = float(np.linalg.norm(dp - along * np.sign(dp @ normal) * normal))
    return along <= 5e-6 and tang <= 3e-2, tang


@pytest.mark.parametrize("ccd", ["mpr", "native"])
def test_cpu_contacts_match_oracle(cpu_lib, ccd):
    """sim_contacts on the CPU backend: same pairs in the same order, geometry at the device
    path's bars (test_gpu_parity.test_contacts_match_oracle), both convex narrowphases."""
    import torch
    from lerobot_mujoco_sim2real_amd import mjcf
    rng = np.random.default_rng(5)
    for xml in (mjcf.SCENE_XML, mjcf.CUBE_SCENE_XML):
        cm = mjcf.compile_mjcf(xml, ccd=ccd)
        n = 256
        S, orc = make_sim(cm, n), Oracle(cm)
        q = _contact_poses(n, rng)
        full = (cube_qpos(cm, n, rng, q) if cm.nq > 6 else q).astype(np.float32).astype(np.float64)
        S.qpos.copy_(torch.as_tensor(full.T, dtype=torch.float32))
        out, nc = S.contacts()
        out, nc = to_np(out), to_np(nc).astype(int)
        pid = out.astype(np.float32).view(np.int32)[..., 7]
        d = cm.desc
        checked = total = shallow = geo_bad = nrm_bad = deep = deep_bad = skipped = slide = 0
        for e in range(n):
            rc = orc.forward(full[e])["contacts"]
            if len(rc) and np.min(np.abs(rc[:, 0])) < 2e-5 or nc[e] != len(rc):
                skipped += 1
                continue
            total += len(rc)
            for k in range(nc[e]):
                assert (d.pair_geom1[pid[e, k]], d.pair_geom2[pid[e, k]]) == (int(rc[k, 7]), int(rc[k, 8]))
                assert out[e, k, 0] < 0
                if abs(rc[k, 0]) < 5e-3:
                    shallow += 1
                    ok_d = abs(out[e, k, 0] - rc[k, 0]) <= 5e-5 + 2e-2 * abs(rc[k, 0])
                    dp = out[e, k, 1:4] - rc[k, 1:4]
                    if ccd == "native":
                        ok_p, tang = contact_point_split(dp, rc[k, 4:7])
                        slide += tang > 2e-3
                    else:
                        ok_p = np.abs(dp).max() <= 2e-3
                    geo_bad += not (ok_d and ok_p)
                    nrm_bad += np.abs(out[e, k, 4:7] - rc[k, 4:7]).max() > 2e-2
                else:
                    deep += 1
                    deep_bad += abs(out[e, k, 0] - rc[k, 0]) > 3e-2 * abs(rc[k, 0])
            checked += 1
        assert checked > 0.9 * n and total > n // 4 and skipped <= 0.03 * n, (checked, total, skipped)
        # (as the device test: native GJK/EPA's depth / normal / deep depth must agree -- r05 here:
        # 0 / <= 1 / 0 off; its point may slide within the patch: 7.2% and 5.3% of 207 / 227 here,
        # 2.6% and 4.0% on the device's 512 envs)
        frac = 0.0 if ccd == "native" else 1.0
        assert deep_bad <= max(2, 0.05 * frac * deep) and nrm_bad <= max(2, 0.06 * frac * shallow)
        assert geo_bad <= max(2, 0.06 * frac * shallow), (geo_bad, shallow)
        assert slide <= 0.10 * shallow, (slide, shallow)


def test_cpu_one_substep_with_contacts(cpu_lib, cube_model):
    cm = cube_model
    n = 256
    S, orc = make_sim(cm, n), Oracle(cm)
    st = orc.new_state(n)
    orc.reset(st, init_qpos=RNG.uniform(-0.3, 0.3, (n, 5)), extra_qpos=cube_qpos(cm, n, RNG))
    for _ in range(5):
        orc.step(st, RNG.uniform(-0.5, 0.5, (n, 5)))
    st = f32(st)
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - st["qvel"])
    assert_pct(dv.max(1), *QVEL_BARS, what="qvel")
    assert to_np(S.ncon).sum() == st["ncon"].sum()


@pytest.mark.parametrize("solver", ["PGS", "Newton"])
def test_cpu_env_step_bench_states(cpu_lib, solver):
    """One 10-substep env-step of the headline workload from t = 100 bench states (cube resting;
    13 envs with arm contacts), PGS (north star) and Newton (MuJoCo's default), vs the oracle's
    same solver.  Bars: the device path's full-size env-step bars
    (test_gpu_parity.test_contact_env_step_late_states_full_size)."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    ids = np.r_[ARM_CONTACT_ENVS_T100, np.arange(115)]
    n = len(ids)
    cm, _, st = bench_states("contact", ids, 100, solver=solver)
    orc = Oracle(cm) if solver == "PGS" else Oracle(cm, solver="newton")
    a = W.chirp_action(W.chirp_tables(ids), 100).astype(np.float32)
    S = make_sim(cm, n)
    st["ncon"][:] = 0
    load_state(S, st)
    og = to_np(S.step(a))
    env = fp32_noise_envelope(orc, st, a.astype(np.float64))
    oc = orc.step(st, a.astype(np.float64), nthreads=8)
    arm = st["ncon"] > 40  # more than the cube's 4 resting contacts in some substep
    blk = ~arm
    assert arm.sum() >= 10, "arm contacts in the sample"
    e = np.abs(og - oc).max(1)
    dv = np.abs(to_np(S.qvel).T - st["qvel"])
    # envs with the cube resting on the table only (measured: obs max 1.1e-7; cube qvel p99 4.2e-5
    # PGS / 2.5e-6 Newton; arm qvel max 2.3e-5)
    assert_pct(e[blk], 1e-6, 2e-6, 2e-6, what="block envs obs")
    assert_pct(dv[blk, 6:].max(1), 5e-6, 5e-4, 5e-4, what="block envs cube qvel")
    assert_pct(dv[blk, :6].max(1), 5e-6, 5e-5, 1e-4, what="block envs arm qvel")
    # envs whose arm touches the table or pushes the cube (r06: MPR's normal in fp64, soarm_collide.h
    # mpr; before it, a grazing arm-link contact's fp32 normal tilted up to 5 degrees and the arm qvel
    # max was 9.7e-2; measured now: arm qvel max 5.3e-6, cube 8.2e-5 PGS)
    assert_pct(e[arm], 1e-6, 2e-5, 2e-5, what="arm-contact envs obs")
    # (Newton's path meets a deep jaw-cube contact, env 2023 at substep 5, where MPR's portal -- and
    # with it the normal -- is decided by near-tied support vertices: fp32 (0.452, -0.229, 0.862)
    # against fp64 (0.445, -0.249, 0.860), 5.6e-3 m/s of cube velocity; tools/env_diverge.py)
    assert_pct(dv[arm, 6:].max(1), 5e-5, 1e-3 if solver == "PGS" else 2e-2, 1e-3 if solver == "PGS" else 2e-2,
               what="arm-contact envs cube qvel")
    am = 1e-4 if solver == "PGS" else 2e-3  # (Newton: the same env, arm qvel 1.1e-3)
    assert_pct(dv[arm, :6].max(1), 2e-5, am, am, what="arm-contact envs arm qvel")
    # every env's arm qvel within 10x the oracle's own fp32-noise envelope (conftest.fp32_noise_envelope;
    # PGS -- Newton's path crosses the MPR portal flip above, which no fp32-sized noise reproduces)
    if solver == "PGS":
        ratio = dv[:, :6].max(1) / (10 * env[:, :6].max(1) + 1e-6)
        k = int(ratio.argmax())
        assert ratio.max() <= 1.0, ("arm qvel vs fp32-noise envelope", ratio.max(), int(ids[k]), dv[k, :6].max(),
                                    env[k, :6].max())
    # (a grazing contact, |depth| ~ fp32 resolution, can exist on one side only)
    assert abs(float(to_np(S.ncon).sum()) - float(st["ncon"].sum())) <= max(2.0, 1e-3 * float(st["ncon"].sum()))


def test_cpu_domain_randomised_substep(cpu_lib):
    """DR parameters (sim_batch_set_params: mass scale, friction, damping scale), one substep."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    n = 256
    cm = W.model("dr")
    orc = Oracle(cm)
    ids = np.arange(n)
    p = W.dr_params(ids, 0)
    prm = np.stack([p["mass_scale"], p["friction"], p["damping_scale"]], 1).astype(np.float32).astype(np.float64)
    st = orc.new_state(n)
    q = W.initial_qpos(cm, ids, 0)
    orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
    tab = W.chirp_tables(ids, 0)
    for t in range(10):  # (t0 of test_gpu_parity.test_one_substep_domain_randomised)
        orc.step(st, W.chirp_action(tab, t), params=prm, nthreads=8)
    st = f32(st)
    S = make_sim(cm, n)
    S.set_params(prm[:, 0], prm[:, 1], prm[:, 2])
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1, params=prm)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    assert_pct(np.abs(to_np(S.qvel).T - st["qvel"]).max(1), *QVEL_BARS, what="qvel")


def test_cpu_config1_single_env_zero_action_1000_steps(cpu_lib):
    """BASELINE.json configs[0] on the CPU backend: one SOARM101Env(device=-1), zero action,
    1000 env-steps vs the fp64 oracle, the bars of the device test
    (test_gpu_parity.test_config1_single_env_zero_action_1000_steps)."""
    from lerobot_mujoco_sim2real_amd.SOARM101 import SOARM101Env
    env = SOARM101Env(device=-1)
    T = 1000
    init = np.r_[np.random.default_rng(0).uniform(-0.3, 0.3, 5), np.zeros(5)].astype(np.float32).astype(np.float64)
    og, _ = env.reset(options={"initial_state": init})
    orc = Oracle(env.model)
    a, b = orc.new_state(1), orc.new_state(1)
    oa = orc.reset(a, init_qpos=init[None, :5], init_qvel=init[None, 5:])
    orc.reset(b, init_qpos=init[None, :5], init_qvel=init[None, 5:])
    np.testing.assert_allclose(og, oa[0], atol=2e-6)
    zero = np.zeros(5, np.float32)
    err, envl = np.zeros(T), np.zeros(T)
    for t in range(T):
        og, r, term, trunc, info = env.step(zero)
        oa, ob = orc.step(a, np.zeros((1, 5))), orc.step(b, np.zeros((1, 5)))
        for k in ("qpos", "qvel", "warm"):
            b[k][:] = b[k].astype(np.float32)
        err[t] = np.abs(og - oa[0]).max()
        envl[t] = np.abs(oa[0] - ob[0]).max()
    run = np.maximum.accumulate(envl)
    bad = np.nonzero(err > 10 * run + 2e-4)[0]
    assert bad.size == 0, ("shadowing", bad[:5], err[bad[:5]], run[bad[:5]])
    assert abs(float(og[2]) - float(oa[0, 2])) < 2e-4 and float(og[2]) < 0.02
    assert np.abs(og - oa[0]).max() < 10 * envl[-20:].max() + 1e-3
    assert int(env.sim.status.numpy()[0]) == int(a["status"][0]) == 0


def test_cpu_ik_matches_oracle(cpu_lib, arm_model):
    import torch
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import cartesian_targets
    n = 200
    tgt = cartesian_targets("Fig8", 1.6 + 0.02 * RNG.uniform(0, 300, n)).astype(np.float32)
    q0 = np.zeros((n, 6), np.float32)
    q0[:, :5] = RNG.uniform(-0.3, 0.3, (n, 5))
    S, orc = make_sim(arm_model, n), Oracle(arm_model)
    qg, okg, _ = S.ik(tgt, q=torch.as_tensor(q0.T.copy()))
    qg, okg = to_np(qg).T, to_np(okg).astype(bool)
    qc, okc, _ = orc.ik(tgt.astype(np.float64), q0.astype(np.float64))
    assert okc.mean() > 0.95 and (okg == okc).mean() > 0.98
    np.testing.assert_allclose(qg[okg & okc][:, :5], qc[okg & okc][:, :5], atol=2e-3)


def test_cpu_bad_state_soft_reset(cpu_lib, arm_model_nocontact):
    import torch
    from lerobot_mujoco_sim2real_amd import abi
    S = make_sim(arm_model_nocontact, 16)
    S.reset()
    S.qvel[2, 5] = float("nan")
    S.qpos[1, 7] = 1e12
    S.step(torch.zeros((16, 5)))
    st = to_np(S.status).astype(int)
    assert st[5] & abi.ST_BADQVEL and st[7] & abi.ST_BADQPOS
    assert np.isfinite(to_np(S.qpos)).all() and (st[[0, 1, 2, 3]] == 0).all()


def test_cpu_thread_count_invariance(cpu_lib, cube_model, monkeypatch):
    """Envs are independent: 1 thread and 4 threads give bit-identical trajectories."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    n = 48
    ids = np.arange(n)
    q0 = W.initial_qpos(cube_model, ids, 0)
    tab = W.chirp_tables(ids, 0)
    out = []
    for th in ("1", "4"):
        monkeypatch.setenv("SOARM_CPU_THREADS", th)
        S = make_sim(cube_model, n)
        S.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
        for t in range(5):
            S.step(W.chirp_action(tab, t).astype(np.float32))
        out.append((S.obs.clone(), S.qpos.clone(), S.qvel.clone(), S.ncon.clone()))
    for x, y in zip(*out):
        assert bool((x == y).all())


def test_cpu_native_ccd_centred_symmetric_overlap(cpu_lib, tmp_path):
    """The kernels' GJK completion (soarm_collide.h gjk_complete) on the host: a mesh cube
    centred inside the table box (test_oracle.test_native_ccd_centred_symmetric_overlap) gives
    the oracle's contact.  The two faces normal to the smallest extent tie, so the normal is
    compared up to sign; depth to fp32 rounding of the 0.13 m overlap."""
    from lerobot_mujoco_sim2real_amd import mjcf
    from test_oracle import probe_states, write_probe_scene
    cm = mjcf.compile_mjcf(write_probe_scene(tmp_path))
    qs = probe_states(cm)
    check_probe_contacts(cm, make_sim(cm, len(qs)), qs)


def check_probe_contacts(cm, S, qs):
    import torch
    orc = Oracle(cm)
    gt, gp = cm.geom_names.index("table"), cm.geom_names.index("probe")
    S.qpos.copy_(torch.as_tensor(qs.T, dtype=torch.float32))
    out, nc = S.contacts()
    out, nc = to_np(out), to_np(nc).astype(int)
    pid = out.astype(np.float32).view(np.int32)[..., 7]
    d = cm.desc
    for e, q in enumerate(qs.astype(np.float32).astype(np.float64)):
        rc = [r for r in orc.forward(q)["contacts"] if {int(r[7]), int(r[8])} == {gt, gp}]
        got = [k for k in range(nc[e]) if {d.pair_geom1[pid[e, k]], d.pair_geom2[pid[e, k]]} == {gt, gp}]
        assert len(rc) == 1 and len(got) == 1, (e, rc, got)
        r, k = rc[0], got[0]
        assert abs(out[e, k, 0] - r[0]) <= 2e-6, (e, out[e, k, 0], r[0])
        assert abs(abs(out[e, k, 4:7] @ r[4:7]) - 1) <= 1e-5, (e, out[e, k, 4:7], r[4:7])


def test_cpu_soft_reset_contact_scene_limit_at_qpos0(cpu_lib):
    """mj_checkVel soft reset in the pick scene on a model whose qpos0 sits inside a joint-limit
    margin (conftest.limit_qpos0_model): the reset env's substep runs mj_forward at qpos0 with the
    cube's resting contacts and the active limit row, as the oracle does."""
    from conftest import limit_qpos0_model, soft_reset_states
    from lerobot_mujoco_sim2real_amd import abi
    cm = limit_qpos0_model()
    orc = Oracle(cm)
    n, bad = 64, [1, 6, 17, 30, 63]
    st = soft_reset_states(cm, orc, n, bad)
    S = make_sim(cm, n)
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    stat = to_np(S.status).astype(int)
    assert all(stat[b] & abi.ST_BADQVEL for b in bad) and (stat == st["status"]).all()
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - st["qvel"]).max(1)
    assert_pct(dv, *QVEL_BARS, what="qvel")
    assert dv[bad].max() < 1e-5, dv[bad]
    # the same envs go bad again (status bits already set): reset, qpos0 contacts, as the oracle
    S.qvel[2, bad] = float("nan")
    st["qvel"][bad, 2] = np.nan
    S.substeps(1)
    orc.step(st, None, nsub=1)
    assert (to_np(S.status).astype(int) == st["status"]).all()
    np.testing.assert_allclose(to_np(S.qpos).T[bad], st["qpos"][bad], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - st["qvel"]).max(1)
    assert dv[bad].max() < 1e-5, dv[bad]
