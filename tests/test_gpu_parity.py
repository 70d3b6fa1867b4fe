"""HIP path vs the float64 oracle (tests marked gpu run on the MI355X box).

Tolerances (fp32 kernel vs fp64 oracle):
* reset / kinematics / contacts / one substep: absolute, stated per test;
* whole trajectories: the SO-ARM101 velocity servo (kv = 50, force clamp
  3.5 N m, h kv / M ~ 3) chatters chaotically, so two fp64 runs that start
  1e-7 apart separate just like fp32 vs fp64 does.  Trajectory parity is
  therefore a shadowing bound: the GPU-vs-oracle divergence must stay within
  a small factor of the oracle-vs-perturbed-oracle divergence.
"""
import numpy as np
import pytest

from conftest import cube_qpos, fp32_noise_envelope, limit_qpos0_model, soft_reset_states
from oracle import Oracle
from test_cpu_backend import contact_point_split

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(7)


def make_sim(cm, n):
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    return BatchSim(cm, n)


def to_np(t):
    return t.detach().cpu().numpy().astype(np.float64)


def load_state(S, st):
    import torch
    dev = S.device
    S.qpos.copy_(torch.as_tensor(st["qpos"].T, dtype=torch.float32, device=dev))
    S.qvel.copy_(torch.as_tensor(st["qvel"].T, dtype=torch.float32, device=dev))
    S.qacc_warmstart.copy_(torch.as_tensor(st["warm"].T, dtype=torch.float32, device=dev))
    S.ctrl.copy_(torch.as_tensor(st["ctrl"].T, dtype=torch.float32, device=dev))
    S.status.zero_()


def f32(st):
    """Round an oracle state to float32 so both sides start bit-identical."""
    return {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}


def random_states(cm, orc, n, steps=3, lo=-1.0, hi=1.0, rng=None):
    """Mid-trajectory states (qvel, warm start and ctrl populated) from the oracle."""
    rng = RNG if rng is None else rng
    st = orc.new_state(n)
    orc.reset(st, init_qpos=rng.uniform(lo, hi, (n, 5)))
    for _ in range(steps):
        orc.step(st, rng.uniform(-0.5, 0.5, (n, 5)))
    return f32(st)


def assert_pct(err, p50, p99, mx, what=""):
    """Percentile bars on an error sample (per env: the max over the compared fields)."""
    e = np.asarray(err, np.float64).ravel()
    got = (float(np.median(e)), float(np.percentile(e, 99)), float(e.max()))
    assert got[0] <= p50 and got[1] <= p99 and got[2] <= mx, (what, "p50/p99/max", got, "bars", (p50, p99, mx))


# Contact-path bars (one substep from oracle states, fp32 device PGS vs fp64 oracle PGS), set at
# ~10x the spread measured on 4096 bench states at t = 20 and 120 (profiles/r03_newton_gap.json,
# "substep_pgs_device_vs_pgs_fp64": qvel p50 2e-7, p99 3.3e-5 -- fp32 and fp64 PGS stopping one
# sweep apart --, max 3.3e-5 on the cube, 2.4e-4 on the arm of an arm-contact env)
QVEL_BARS = (2e-6, 3.5e-4, 2.5e-3)


def test_reset_obs(gpu_lib, arm_model, cube_model):
    for cm in (arm_model, cube_model):
        n = 512
        S, orc = make_sim(cm, n), Oracle(cm)
        iq = RNG.uniform(-1.5, 1.5, (n, 5)).astype(np.float32)
        ex = cube_qpos(cm, n, RNG).astype(np.float32) if cm.nq > 6 else None
        og = to_np(S.reset(init_qpos=iq, extra_qpos=ex))
        st = orc.new_state(n)
        oc = orc.reset(st, init_qpos=iq.astype(np.float64), extra_qpos=ex)
        np.testing.assert_allclose(og, oc, atol=2e-6)
        np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=1e-7)


def test_reset_device_rng(gpu_lib, arm_model):
    from lerobot_mujoco_sim2real_amd.sim import reset_qpos_draw
    n = 1000
    S = make_sim(arm_model, n)
    S.reset(seed=123456789, env_offset=5000)
    q = to_np(S.qpos)[:5].T
    np.testing.assert_array_equal(q.astype(np.float32), reset_qpos_draw(123456789, np.arange(5000, 5000 + n)))
    assert q.min() >= -0.3 and q.max() < 0.3


def test_one_substep_no_contact(gpu_lib, arm_model_nocontact):
    cm = arm_model_nocontact
    n = 1024
    S, orc = make_sim(cm, n), Oracle(cm)
    st = random_states(cm, orc, n)
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=2e-6)
    np.testing.assert_allclose(to_np(S.qvel).T, st["qvel"], atol=5e-4)
    assert (to_np(S.status) == st["status"]).all()


def test_one_env_step_obs(gpu_lib, arm_model_nocontact):
    cm = arm_model_nocontact
    n = 1024
    S, orc = make_sim(cm, n), Oracle(cm)
    st = random_states(cm, orc, n)
    load_state(S, st)
    a = RNG.uniform(-0.5, 0.5, (n, 5)).astype(np.float32)
    og = to_np(S.step(a))
    oc = orc.step(st, a.astype(np.float64))
    err = np.abs(og - oc)
    assert np.median(err) < 1e-6 and err.max() < 5e-4


def _divergence(cm, n, T):
    """Envelope: fp64 oracle vs the same oracle whose state is re-rounded to fp32 after every
    env-step (an fp32-sized perturbation injected every step, amplified by the chaos)."""
    orc = Oracle(cm)
    iq = RNG.uniform(-0.3, 0.3, (n, 5)).astype(np.float32).astype(np.float64)
    acts = RNG.uniform(-0.5, 0.5, (T, n, 5)).astype(np.float32).astype(np.float64)
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


def test_trajectory_shadowing(gpu_lib, arm_model_nocontact):
    """GPU fp32 vs oracle fp64 over 20 env-steps stays within 10x the oracle's fp32-rounding envelope."""
    cm = arm_model_nocontact
    n, T = 512, 20
    iq, acts, envelope = _divergence(cm, n, T)
    S, orc = make_sim(cm, n), Oracle(cm)
    st = orc.new_state(n)
    S.reset(init_qpos=iq.astype(np.float32))
    orc.reset(st, init_qpos=iq.astype(np.float32).astype(np.float64))
    for t in range(T):
        e = np.abs(to_np(S.step(acts[t].astype(np.float32))) - orc.step(st, acts[t]))
        env = envelope[t]
        # the GPU also rounds every substep's arithmetic, not only the state: 10x + a small floor
        assert np.median(e) <= 10 * np.median(env) + 1e-5, (t, np.median(e), np.median(env))
        assert np.quantile(e, 0.9) <= 10 * np.quantile(env, 0.9) + 2e-4


def _contact_poses(cm, n, rng=RNG):
    """Poses that drive the gripper into the table / fold the arm (self contacts)."""
    q = np.zeros((n, 6))
    q[:, 0] = rng.uniform(-1.0, 1.0, n)
    q[:, 1] = rng.uniform(0.6, 1.6, n)
    q[:, 2] = rng.uniform(-0.5, 1.0, n)
    q[:, 3] = rng.uniform(0.3, 1.6, n)
    q[:, 4] = rng.uniform(-2.0, 2.0, n)
    q[:, 5] = rng.uniform(0.0, 1.5, n)
    half = n // 2
    q[half:, 1] = rng.uniform(-1.7, -1.3, n - half)    # home-like fold: shoulder servo vs lower arm
    q[half:, 2] = rng.uniform(1.3, 1.69, n - half)
    return q.astype(np.float32).astype(np.float64)


@pytest.mark.parametrize("ccd", ["mpr", "native"])
def test_contacts_match_oracle(gpu_lib, arm_model, cube_model, ccd):
    """Same contact pairs in the same order (bit-exact indexing); geometry within fp32 tolerance.
    Both convex-convex narrowphases: libccd MPR and MuJoCo's native GJK/EPA (kernel vs oracle)."""
    import torch
    from lerobot_mujoco_sim2real_amd import mjcf
    models = (mjcf.compile_mjcf(mjcf.SCENE_XML, ccd=ccd), mjcf.compile_mjcf(mjcf.CUBE_SCENE_XML, ccd=ccd))
    for cm in models:
        assert cm.desc.ccd == (1 if ccd == "native" else 0)
        n = 512
        S, orc = make_sim(cm, n), Oracle(cm)
        rng = np.random.default_rng(31 + cm.nq)  # (the poses do not depend on which tests ran before)
        q = _contact_poses(cm, n, rng)
        full = cube_qpos(cm, n, rng, q) if cm.nq > 6 else q
        full = full.astype(np.float32).astype(np.float64)
        S.qpos.copy_(torch.as_tensor(full.T, dtype=torch.float32, device=S.device))
        out, nc = S.contacts()
        out, nc = to_np(out), to_np(nc).astype(int)
        pair_ids = out.astype(np.float32).view(np.int32)[..., 7]
        d = cm.desc
        checked = total = deep = deep_bad = shallow = nrm_bad = geo_bad = slide = 0
        skipped_grazing = skipped_count = 0
        for e in range(n):
            ref = orc.forward(full[e])
            rc = ref["contacts"]
            if len(rc) and np.min(np.abs(rc[:, 0])) < 2e-5:
                skipped_grazing += 1
                continue  # grazing contact: existence is decided below fp32 resolution
            if nc[e] != len(rc):
                skipped_count += 1
                # only a grazing contact may exist on one side: every contact of the pair
                # multisets' symmetric difference is shallower than 100 um (fp32 GJK can stall a
                # few 1e-5 m from the origin on the table-vs-link Minkowski difference, 1.2 m
                # across: tools/ccd_mismatch.py found one 29 um oracle contact in 2048 poses)
                gp = [(int(d.pair_geom1[x]), int(d.pair_geom2[x]), out[e, k, 0]) for k, x in enumerate(pair_ids[e, :nc[e]])]
                op = [(int(a), int(b), r0) for r0, a, b in zip(rc[:, 0], rc[:, 7], rc[:, 8])]
                extra = []
                for key in {c[:2] for c in gp + op}:
                    a = sorted(abs(c[2]) for c in gp if c[:2] == key)
                    b = sorted(abs(c[2]) for c in op if c[:2] == key)
                    extra += (a if len(a) > len(b) else b)[:abs(len(a) - len(b))]  # the shallowest
                assert extra and max(extra) < 1e-4, (e, gp, op)
                continue
            total += len(rc)
            for k in range(nc[e]):
                p = pair_ids[e, k]
                assert (d.pair_geom1[p], d.pair_geom2[p]) == (int(rc[k, 7]), int(rc[k, 8]))
                # geometry for physically relevant depths (soft contacts settle at ~1 mm); the
                # test poses also drive links decimetres into the table, where MPR's portal (and
                # so its depth estimate) is ill-conditioned in any precision
                if abs(rc[k, 0]) < 5e-3:
                    shallow += 1
                    ok_d = abs(out[e, k, 0] - rc[k, 0]) <= 5e-5 + 2e-2 * abs(rc[k, 0])
                    if ccd == "native":  # EPA's witness point may slide within a face contact's patch
                        ok_p, tang = contact_point_split(out[e, k, 1:4] - rc[k, 1:4], rc[k, 4:7])
                        slide += tang > 2e-3
                    else:
                        ok_p = np.abs(out[e, k, 1:4] - rc[k, 1:4]).max() <= 2e-3
                    geo_bad += not (ok_d and ok_p)
                    assert out[e, k, 0] < 0
                    nrm_bad += np.abs(out[e, k, 4:7] - rc[k, 4:7]).max() > 2e-2
                else:
                    deep += 1
                    assert out[e, k, 0] < 0
                    deep_bad += abs(out[e, k, 0] - rc[k, 0]) > 3e-2 * abs(rc[k, 0])
            checked += 1
        assert checked > 0.9 * n and total > n // 4
        # the envs left out of the pair-by-pair comparison: a grazing contact (|depth| < 20 um) on
        # the oracle side, or a count mismatch whose extra contact is grazing on the GPU side
        assert skipped_grazing + skipped_count <= 0.03 * n, (skipped_grazing, skipped_count)
        # MPR: deep (>5 mm) penetrations' depth depends on the portal path, which flips on near-tied
        # support vertices, and its normals / points come from the final portal face, which fp32 can
        # pick differently from fp64 when two faces nearly tie -- bars for the bulk only.  Native
        # GJK/EPA is a minimum-depth method: depth, normal and deep depth must all agree (r05, 512
        # envs per scene: 0 off in every class), its witness point may slide within a face contact's
        # patch on <= 5% of the shallow contacts (r05: 2.6% and 4.0%; VERDICT r4 asked <= 5%)
        frac = 0.0 if ccd == "native" else 1.0
        assert deep_bad <= max(2, 0.05 * frac * deep), (deep_bad, deep)
        assert nrm_bad <= max(2, 0.06 * frac * shallow), ("normals", nrm_bad, shallow)
        assert geo_bad <= max(2, 0.06 * frac * shallow), ("depth/point", geo_bad, shallow)
        assert slide <= 0.05 * shallow, ("EPA point slides", slide, shallow)
        print(f"contacts: {total} checked, shallow {shallow} (geometry off {geo_bad}, normal off {nrm_bad}), "
              f"deep {deep} (off {deep_bad}); envs skipped: grazing {skipped_grazing}, count {skipped_count}")


def test_one_substep_with_contacts(gpu_lib, cube_model):
    cm = cube_model
    n = 512
    S, orc = make_sim(cm, n), Oracle(cm)
    st = orc.new_state(n)
    ex = cube_qpos(cm, n, RNG)
    orc.reset(st, init_qpos=RNG.uniform(-0.3, 0.3, (n, 5)), extra_qpos=ex)
    for _ in range(5):  # settle the cube onto the table (4 resting contacts each)
        orc.step(st, RNG.uniform(-0.5, 0.5, (n, 5)))
    st = f32(st)
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - st["qvel"])
    assert_pct(dv[:, 6:].max(1), *QVEL_BARS, what="cube qvel")
    assert_pct(dv[:, :6].max(1), *QVEL_BARS, what="arm qvel")
    assert to_np(S.ncon).sum() == st["ncon"].sum()


def _bench_states(name, n, steps, seed=0, nthreads=8):
    """Oracle states of a bench workload after `steps` env-steps (chirp inputs), fp32-rounded."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    cm = W.model(name)
    orc = Oracle(cm)
    ids = np.arange(n)
    st = orc.new_state(n)
    q = W.initial_qpos(cm, ids, seed)
    orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
    tab = W.chirp_tables(ids, seed)
    prm = None
    if W.CONFIGS[name]["dr"]:
        p = W.dr_params(ids, seed)
        prm = np.stack([p["mass_scale"], p["friction"], p["damping_scale"]], 1).astype(np.float32).astype(np.float64)
    for t in range(steps):
        orc.step(st, W.chirp_action(tab, t), params=prm, nthreads=nthreads)
    return cm, orc, f32(st), prm


@pytest.mark.parametrize("rs", ["1", "0"])
def test_one_substep_bench_state_mixed_contacts(gpu_lib, rs, monkeypatch):
    """One substep from late bench states (t = 120 env-steps of the contact workload): the
    cube's 4 resting contacts plus, in some envs, arm-table contacts (the waves that take
    the general contact paths).  rs = "1": the row-space kernel (the default; soarm_pgs.h
    RsLayout), "0": the quad kernel (SOARM_RS=0)."""
    monkeypatch.setenv("SOARM_RS", rs)
    cm, orc, st, _ = _bench_states("contact", 512, 120)
    S = make_sim(cm, 512)
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    assert st["ncon"].sum() > 4 * 512, "no arm contacts in the sample"
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - st["qvel"])
    assert_pct(dv[:, 6:].max(1), *QVEL_BARS, what="cube qvel")
    assert_pct(dv.max(1), *QVEL_BARS, what="qvel")
    assert to_np(S.ncon).sum() == st["ncon"].sum()
    # the arm's velocities: rs = "1" sweeps every row in mj_solPGS order (no retirement); rs = "0"
    # (the quad kernel) retires the arm's rows once a sweep moves them by <= 1e-6 (soarm_pgs.h
    # ysweeps).  Either way the bulk stays at fp32 resolution (quad, measured: p99 8e-8, max 2e-5
    # on 1024 envs, identical to a build without retirement)
    err = np.abs(to_np(S.qvel).T[:, :6] - st["qvel"][:, :6]).max(1)
    assert np.percentile(err, 99) < 1e-6 and err.max() < 2e-4, (np.percentile(err, 99), err.max())


def test_one_substep_extra_contact_sweeps(gpu_lib):
    """The contact-space PGS variants (soarm_pgs.h ysweeps): waves whose lanes carry the
    cube's block plus one arm-only extra contact, one arm-cube extra, or both (the two-slot
    variant), assembled from late bench states (oracle census of each env's contacts) so
    that every variant runs; one substep against the oracle."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    nb = 4096  # arm-cube contacts are rare (~0.5% of envs at t = 100)
    cm, orc, st, _ = _bench_states("contact", nb, 100, nthreads=16)
    names = cm.geom_names
    table, cube = names.index("table"), names.index("cube")
    cats = {k: [] for k in ("block", "arm", "coupled", "both")}
    for i in range(nb):
        fw = orc.forward(st["qpos"][i], st["qvel"][i], st["ctrl"][i], st["warm"][i])
        g = [(int(c[7]), int(c[8])) for c in fw["contacts"]]
        blk = [x for x in g if set(x) == {table, cube}]
        ext = [x for x in g if set(x) != {table, cube}]
        if len(blk) == 0 or len(blk) > 4:
            continue
        onc = [cube in x for x in ext]
        if not ext:
            cats["block"].append(i)
        elif len(ext) == 1:
            cats["coupled" if onc[0] else "arm"].append(i)
        elif len(ext) == 2 and not onc[0]:
            cats["both"].append(i)
    counts = {k: len(v) for k, v in cats.items()}
    assert counts["arm"] > 0 and counts["coupled"] + counts["both"] > 0, counts
    # one wave per category (lanes filled with block-only envs), then a mixed wave
    pick = []
    for k in ("arm", "coupled", "both"):
        ids = (cats[k] * 64)[:64] if cats[k] else []
        pick += ids + cats["block"][: 64 - len(ids)] if ids else []
    pick += (cats["arm"] + cats["coupled"] + cats["both"] + cats["block"]) [:64]
    pick = np.array(pick[: (len(pick) // 64) * 64])
    sub = {k: v[pick].copy() for k, v in st.items()}
    n = len(pick)
    S = make_sim(cm, n)
    sub["ncon"][:] = 0
    load_state(S, sub)
    S.substeps(1)
    orc.step(sub, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, sub["qpos"], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - sub["qvel"]).max(1)
    # every env here carries arm contacts; the RS kernel sweeps all their rows in mj_solPGS order
    # (layouts (1, 0), (0, 1), (1, 1)) with no retirement (r05 tools/rs_cat.py on the 4096 bench
    # states at t = 100: arm-only extra max 1.5e-5, arm-cube 6.6e-6, both 4.6e-6; VERDICT r4's
    # p99 2e-4 / max 5e-4)
    assert_pct(dv, 4e-5, 2e-4, 5e-4, what="qvel")
    assert to_np(S.ncon).sum() == sub["ncon"].sum()


def test_one_substep_domain_randomised(gpu_lib):
    """Config 4 DR (mass, friction, damping per env) through sim_batch_set_params."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    cm, orc, st, prm = _bench_states("dr", 512, 10)
    S = make_sim(cm, 512)
    S.set_params(mass_scale=prm[:, 0], friction=prm[:, 1], damping_scale=prm[:, 2])
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1, params=prm)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    assert_pct(np.abs(to_np(S.qvel).T - st["qvel"]).max(1), *QVEL_BARS, what="qvel")
    assert to_np(S.ncon).sum() == st["ncon"].sum()


# qvel max over one full-size env-step (4096 / 8192 envs) against the fp64 oracle, ~3x the r06
# measurement after the MPR normal fix (arm 6.7e-5 / 3.1e-4, cube 6.8e-5 / 6.1e-4 at t = 100 / DR
# t = 40; r05 bars: arm 5e-2, cube 2e-2)
ARM_QVEL_MAX, CUBE_QVEL_MAX = 1e-3, 2e-3


def _within_noise_envelope(dv, env):
    """Every env's arm qvel within 10x the fp64 oracle's own fp32-noise envelope (conftest.
    fp32_noise_envelope: the oracle with +-8 fp32 ulps of state noise injected after every substep,
    no library code).  1e-6: qvel's fp32 resolution at ~10 rad/s."""
    ratio = dv[:, :6].max(1) / (10 * env[:, :6].max(1) + 1e-6)
    k = int(ratio.argmax())
    a, c = dv[:, :6].max(1), dv[:, 6:].max(1)
    print(f"env-step vs oracle: arm qvel p50 {np.median(a):.3g} p99 {np.percentile(a, 99):.3g} max {a.max():.3g}; "
          f"cube qvel p50 {np.median(c):.3g} p99 {np.percentile(c, 99):.3g} max {c.max():.3g}; "
          f"envelope ratio max {ratio.max():.3g} (env {k})")
    assert ratio.max() <= 1.0, ("arm qvel vs fp32-noise envelope", ratio.max(), k, dv[k, :6].max(), env[k, :6].max(),
                                "envs over 1/10 of it", int((ratio > 0.1).sum()))


def test_dr_env_step_full_size(gpu_lib):
    """BASELINE config 4 at its per-GPU size: 8192 envs (65536 over 8 GPUs) of the pick scene with
    per-env mass / friction / damping DR, one graph-captured 10-substep env-step (the one-wave
    kernel: 8192 envs fill the SIMDs without the wide workgroup) from t = 40 bench states against
    one oracle env-step with the same parameters; the bars of the headline's full-size test."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    n = 8192
    cm, orc, st, prm = _bench_states("dr", n, 40, nthreads=16)
    p = W.dr_params(np.arange(n))
    S = make_sim(cm, n)
    S.set_params(**p)
    a = W.chirp_action(W.chirp_tables(np.arange(n)), 40).astype(np.float32)
    st["ncon"][:] = 0
    load_state(S, st)
    og = to_np(S.step(a))
    env = fp32_noise_envelope(orc, st, a.astype(np.float64), params=prm, nthreads=16)
    oc = orc.step(st, a.astype(np.float64), params=prm, nthreads=16)
    assert_pct(np.abs(og - oc).max(1), 1e-6, 2e-6, 2e-4, what="obs")
    dv = np.abs(to_np(S.qvel).T - st["qvel"])
    assert_pct(dv[:, 6:].max(1), 5e-6, 5e-4, CUBE_QVEL_MAX, what="cube qvel")
    assert_pct(dv[:, :6].max(1), 5e-6, 5e-5, ARM_QVEL_MAX, what="arm qvel")
    _within_noise_envelope(dv, env)
    np.testing.assert_allclose(to_np(S.qpos).T[:, 6:9], st["qpos"][:, 6:9], atol=5e-6)
    assert int((to_np(S.status) != 0).sum()) == int((st["status"] != 0).sum())


@pytest.mark.parametrize("n", [1, 100])
def test_odd_batch_sizes(gpu_lib, cube_model, n):
    """Batches that are not a multiple of the 64-lane wave (tail lanes masked)."""
    cm = cube_model
    S, orc = make_sim(cm, n), Oracle(cm)
    st = orc.new_state(n)
    orc.reset(st, init_qpos=RNG.uniform(-0.3, 0.3, (n, 5)), extra_qpos=cube_qpos(cm, n, RNG))
    for _ in range(3):
        orc.step(st, RNG.uniform(-0.5, 0.5, (n, 5)))
    st = f32(st)
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    np.testing.assert_allclose(to_np(S.qvel).T, st["qvel"], atol=QVEL_BARS[2])


def test_ik_rollout_tracks_fig8(gpu_lib):
    """Config 5 (IK-in-the-loop DataCollection): the end effector follows its Fig8 target."""
    import torch
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    cm = W.model("rollout")
    n, T = 256, 120
    ids = np.arange(n)
    S = BatchSim(cm, n)
    q0 = W.initial_qpos(cm, ids)
    obs = S.reset(init_qpos=q0[:, :5])
    phase = torch.as_tensor(W.ik_phase(ids), dtype=torch.float32, device=S.device)
    qstar = S.qpos.clone()
    err = []
    for t in range(T):
        tgt = W.fig8_targets(float(t), phase, lib=torch)
        qstar, ok, _ = S.ik(tgt, q=qstar)
        a = W.ik_action(qstar[:5].T, obs[:, 3:8], lib=torch)
        obs = S.step(a)
        err.append(torch.linalg.norm(obs[:, :3] - tgt, dim=1).median().item())
    assert err[-1] < 0.02 and err[-1] < 0.5 * err[0], err[::20]


@pytest.mark.parametrize("which", ["new_calib_table", "old_calib"])
def test_position_servo_scene_substep(gpu_lib, which):
    """The position-servo scenes: scene_with_table.xml (kp = 50 with
    dampratio 1, force +-33.5, arm-table contacts on) and the old calibration's arm alone
    (kp = 17.8, force +-3.35, self-collision pairs only)."""
    from lerobot_mujoco_sim2real_amd import mjcf
    if which == "old_calib":
        cm = mjcf.compile_mjcf(mjcf.OLD_CALIB_XML, obs_site="gripper")
    else:
        cm = mjcf.compile_mjcf(mjcf.POSITION_SCENE_XML)
    n = 256
    orc = Oracle(cm)
    st = orc.new_state(n)
    orc.reset(st, init_qpos=RNG.uniform(-0.5, 0.5, (n, 5)))
    for _ in range(3):
        orc.step(st, RNG.uniform(-0.5, 0.5, (n, 5)))
    st = f32(st)
    S = make_sim(cm, n)
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=2e-6)
    np.testing.assert_allclose(to_np(S.qvel).T, st["qvel"], atol=1e-3)


def test_generate_and_save_data_cache(gpu_lib, tmp_path):
    """SOARM101_DataCollection.py:138-181: .npy cache names / shapes / dtype, resume from
    the cache, and the Collater split the Koopman trainer consumes (x = [5:13], u = [0:5])."""
    import os
    from lerobot_mujoco_sim2real_amd.args import Args
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import SOARM101DataGenerator
    a = Args(["--data_root", str(tmp_path), "--train_samples", "96", "--train_steps", "5",
              "--test_samples", "32", "--test_steps", "7", "--batch_size", "16", "--eval_batch_size", "8"])
    g = SOARM101DataGenerator(a)
    g.generate_and_save_data()
    d = os.path.join(str(tmp_path), "SOARM101", "data")
    names = sorted(os.listdir(d))
    assert names == sorted(["train_data_96_5.npy", "val_data_32_7.npy", "test_data_random_32_7.npy",
                            "test_data_sin_32_7.npy", "test_data_chirp_32_7.npy"]), names
    assert g.train_data.shape == (96, 6, 13) and g.train_data.dtype == np.float64
    assert g.val_data.shape == (32, 8, 13)
    for t in ("random", "sin", "chirp"):
        assert g.test_data_dict[t].shape == (32, 8, 13)
    assert np.abs(g.train_data[:, :, :5]).max() <= 0.5 + 1e-6
    # splits are independent draws (one advancing stream in the reference, :97-132):
    # no val trajectory starts where a train one does, val and test_random inputs differ
    v0, t0 = g.val_data[:, 0, 8:13], g.train_data[:32, 0, 8:13]
    assert (np.abs(v0 - t0).max(1) > 1e-3).all()
    assert (np.abs(g.val_data[:, :, :5] - g.test_data_dict["random"][:, :, :5]).max((1, 2)) > 1e-3).all()
    assert np.abs(g.test_data_dict["sin"][:, :, :5] - g.test_data_dict["chirp"][:, :, :5]).max() > 1e-3
    mt = {n: os.path.getmtime(os.path.join(d, n)) for n in names}
    g2 = SOARM101DataGenerator(a)
    g2.generate_and_save_data()  # resumes from the cache
    assert {n: os.path.getmtime(os.path.join(d, n)) for n in names} == mt
    np.testing.assert_array_equal(g2.train_data, g.train_data)
    tr, va = g2.get_train_loader()
    b = next(iter(tr))
    assert tuple(b["x"].shape) == (16, 6, 8) and tuple(b["u"].shape) == (16, 6, 5)
    tb = next(iter(g2.get_test_loader("chirp")))
    assert tuple(tb["x"].shape) == (8, 8, 8)


def test_cube_rests_gpu(gpu_lib, cube_model):
    cm = cube_model
    n = 256
    S = make_sim(cm, n)
    S.reset(extra_qpos=cube_qpos(cm, n, RNG).astype(np.float32))
    for _ in range(50):
        S.step(np.zeros((n, 5), np.float32))
    q = to_np(S.qpos).T
    v = to_np(S.qvel).T
    assert np.abs(q[:, 8] - (-0.0009 + 0.015)).max() < 2e-3   # resting height
    assert np.abs(v[:, 6:]).max() < 1e-2
    assert (to_np(S.ncon) > 0).all()


def test_ik_matches_oracle(gpu_lib, arm_model):
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import cartesian_targets
    n = 600
    tp = 1.6 + 0.02 * RNG.uniform(0, 300, n)
    tgt = np.concatenate([cartesian_targets("Fig8", tp[:300]), cartesian_targets("Circle", tp[300:], idx=0)])
    tgt = tgt.astype(np.float32)
    S, orc = make_sim(arm_model, n), Oracle(arm_model)
    q0 = np.zeros((n, 6), np.float32)
    q0[:, :5] = RNG.uniform(-0.3, 0.3, (n, 5))
    import torch
    qg, okg, itg = S.ik(tgt, q=torch.as_tensor(q0.T.copy(), device=S.device))
    qg, okg = to_np(qg).T, to_np(okg).astype(bool)
    qc, okc, itc = orc.ik(tgt.astype(np.float64), q0.astype(np.float64))
    assert okc.mean() > 0.95
    assert (okg == okc).mean() > 0.98
    both = okg & okc
    np.testing.assert_allclose(qg[both][:, :5], qc[both][:, :5], atol=2e-3)
    from lerobot_mujoco_sim2real_amd import mjcf
    for e in np.nonzero(both)[0][:50]:
        ee = mjcf.NumpyKinematics(arm_model).forward_position(qg[e]).site_xpos(arm_model.desc.obs_site)
        assert np.linalg.norm(ee - tgt[e]) < 1e-5


def test_pose_ik_matches_oracle(gpu_lib, arm_model):
    """qpos_from_site_pose with target_quat (TrajectoryGenerator.py:96-107, rot_weight 0.5): reachable
    poses from perturbed starts, and the reference's default orientation [1, 0, 0, 0] over Fig8."""
    import torch
    from lerobot_mujoco_sim2real_amd import mjcf
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import cartesian_targets
    cm = arm_model
    kin = mjcf.NumpyKinematics(cm)
    s = cm.desc.obs_site
    n = 512
    qt = np.zeros((n, 6))
    qt[:, :5] = RNG.uniform(-0.8, 0.8, (n, 5))
    tp = np.array([kin.forward_position(q).site_xpos(s) for q in qt]).astype(np.float32)
    tq = np.array([kin.forward_position(q).site_xquat(s) for q in qt]).astype(np.float32)
    q0 = (qt + np.c_[RNG.uniform(-0.15, 0.15, (n, 5)), np.zeros(n)]).astype(np.float32)
    S, orc = make_sim(cm, n), Oracle(cm)
    qg, okg, _ = S.ik(tp, q=torch.as_tensor(q0.T.copy(), device=S.device), target_quat=tq)
    qg, okg = to_np(qg).T, to_np(okg).astype(bool)
    qc, okc, _ = orc.ik(tp.astype(np.float64), q0.astype(np.float64), target_quat=tq.astype(np.float64))
    assert okc.mean() > 0.9 and (okg == okc).mean() > 0.9, (okg.mean(), okc.mean(), (okg == okc).mean())
    both = okg & okc
    np.testing.assert_allclose(qg[both][:, :5], qc[both][:, :5], atol=2e-3)
    # the default orientation over the reference's Fig8 path (a 5-dof arm: some points fail)
    tpf = cartesian_targets("Fig8", 1.6 + 0.02 * np.linspace(0, 300, 300)).astype(np.float32)
    S2 = make_sim(cm, 300)
    qf, okf, _ = S2.ik(tpf, q=None, target_quat=np.array([1.0, 0, 0, 0], np.float32))
    qcf, okcf, _ = orc.ik(tpf.astype(np.float64), np.zeros((300, 6)), target_quat=np.array([1.0, 0, 0, 0]))
    okf = to_np(okf).astype(bool)
    assert (okf == okcf).mean() > 0.95
    b2 = okf & okcf
    np.testing.assert_allclose(to_np(qf).T[b2][:, :5], qcf[b2][:, :5], atol=2e-3)


def test_rand_uniform_matches_host_mirror(gpu_lib, arm_model):
    """sim_rand_uniform (the rollout's keyed input draws) == workloads.keyed_uniform bit for bit."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    n = 1000
    S = make_sim(arm_model, n)
    for seed, ctr, k, lo, hi, off in ((7, 0, 5, -0.5, 0.5, 0), (2 ** 40 + 3, 123, 9, 0.0, 2 * np.pi, 5000)):
        d = S.rand_uniform(seed, ctr, k, lo, hi, env_offset=off).cpu().numpy()
        np.testing.assert_array_equal(d, W.keyed_uniform(seed, np.arange(off, off + n), ctr, k, lo, hi))


def test_sharded_rollouts_bit_identical(gpu_lib, arm_model):
    """§8e: a dataset built as two env shards (ranks 0 and 1 of 2, each its own batch) equals the
    single-batch build bit for bit, for every input type (draws keyed by global trajectory id)."""
    from lerobot_mujoco_sim2real_amd.args import Args
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import SOARM101DataGenerator
    g = SOARM101DataGenerator(Args([]), model=arm_model, max_envs=128)
    for kind in ("random", "sin", "chirp", "ik_fig8"):
        full = g.generate_physics_based_data(301, 6, kind, seed=11)
        parts = [g.generate_physics_based_data(301, 6, kind, seed=11, rank=r, world=2, gather=False) for r in range(2)]
        np.testing.assert_array_equal(np.concatenate(parts), full, err_msg=kind)
        assert full.shape == (301, 7, 13)


def test_bad_state_soft_reset(gpu_lib, arm_model_nocontact):
    import torch
    from lerobot_mujoco_sim2real_amd import abi
    cm = arm_model_nocontact
    S = make_sim(cm, 64)
    S.reset()
    S.qvel[2, 5] = float("nan")
    S.qpos[1, 7] = 1e12
    S.step(torch.zeros((64, 5), device=S.device))
    st = to_np(S.status).astype(int)
    assert st[5] & abi.ST_BADQVEL and st[7] & abi.ST_BADQPOS
    assert np.isfinite(to_np(S.qpos)).all() and (st[[0, 1, 2, 3]] == 0).all()


@pytest.mark.parametrize("rs", ["1", "0"])
def test_soft_reset_contact_scene_limit_at_qpos0(gpu_lib, rs, monkeypatch):
    """mj_checkVel soft resets in the pick scene, on a model whose qpos0 sits inside a joint-limit
    margin (conftest.limit_qpos0_model): the reset envs run mj_forward at qpos0 with the
    cube's 4 resting contacts (DModel c0_*, made at model creation) and the active limit row, in
    waves shared with envs that keep their own contacts; rs = "1" the RS kernel (a reset env's
    limit row sends its wave to the v-form sweeps by a wave-wide vote), "0" the quad kernel."""
    from lerobot_mujoco_sim2real_amd import abi
    monkeypatch.setenv("SOARM_RS", rs)
    cm = limit_qpos0_model()
    orc = Oracle(cm)
    n, bad = 64, [1, 6, 17, 30, 63]
    st = soft_reset_states(cm, orc, n, bad)
    S = make_sim(cm, n)
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    stat = to_np(S.status).astype(int)
    assert all(stat[b] & abi.ST_BADQVEL for b in bad) and (stat == st["status"]).all()
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - st["qvel"]).max(1)
    assert_pct(dv, *QVEL_BARS, what="qvel")
    assert dv[bad].max() < 1e-5, dv[bad]
    assert to_np(S.ncon).sum() == st["ncon"].sum()
    # the same envs go bad again: their status bits are already set (sticky), the reset must still
    # store the qpos0 state, take the contacts at qpos0 (the collide ran on the discarded qpos) and
    # run its own kinematics
    import torch
    st = f32(st)  # (both sides from the same fp32 state again, the device's status bits kept)
    status = S.status.clone()
    load_state(S, st)
    S.status.copy_(status)
    S.qvel[2, bad] = torch.nan
    st["qvel"][bad, 2] = np.nan
    ncon0 = to_np(S.ncon).sum()
    S.substeps(1)
    orc.step(st, None, nsub=1)
    stat = to_np(S.status).astype(int)
    assert (stat == st["status"]).all()
    np.testing.assert_allclose(to_np(S.qpos).T[bad], st["qpos"][bad], atol=5e-6)
    dv = np.abs(to_np(S.qvel).T - st["qvel"]).max(1)
    assert_pct(dv, *QVEL_BARS, what="qvel")
    assert dv[bad].max() < 1e-5, dv[bad]
    assert to_np(S.ncon).sum() - ncon0 == st["ncon"].sum() - ncon0


def test_golden_fixture_gpu(gpu_lib, arm_model_nocontact):
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_arm_random.npz"))
    S = make_sim(arm_model_nocontact, z["init_qpos"].shape[0])
    obs = [to_np(S.reset(init_qpos=z["init_qpos"].astype(np.float32)))]
    for a in z["actions"]:
        obs.append(to_np(S.step(a.astype(np.float32))))
    obs = np.stack(obs)
    np.testing.assert_allclose(obs[:2], z["obs"][:2], atol=1e-4)
    # later steps: the shadowing envelope (test_trajectory_shadowing) of the fixture itself -- the
    # fp64 oracle replaying the fixture's inputs with its state re-rounded to fp32 every env-step
    orc = Oracle(arm_model_nocontact)
    st = orc.new_state(z["init_qpos"].shape[0])
    env = [np.abs(orc.reset(st, init_qpos=z["init_qpos"]) - z["obs"][0])]
    for t, a in enumerate(z["actions"]):
        for k in ("qpos", "qvel", "warm"):
            st[k][:] = st[k].astype(np.float32)
        env.append(np.abs(orc.step(st, a) - z["obs"][t + 1]))
    run = np.maximum.accumulate(np.stack(env).max(axis=(1, 2)))  # running max over steps
    err = np.abs(obs - z["obs"]).max(axis=(1, 2))
    assert (err <= 10 * run + 2e-4).all(), (err, run)


def test_datacollection_layout_and_replay(gpu_lib, arm_model_nocontact):
    """[traj, steps+1, 13] layout, row i = [u_i, s_i]; replaying the same inputs through the oracle."""
    from lerobot_mujoco_sim2real_amd.args import Args
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import SOARM101DataGenerator
    gen = SOARM101DataGenerator(Args([]), model=arm_model_nocontact)
    for kind in ("random", "sin", "chirp"):
        d = gen.generate_physics_based_data(64, 6, kind)
        assert d.shape == (64, 7, 13) and d.dtype == np.float64
        assert np.abs(d[:, :, :5]).max() <= 0.5
    n, T = 128, 3
    iq = RNG.uniform(-0.3, 0.3, (n, 5))
    acts = RNG.uniform(-0.5, 0.5, (T + 1, n, 5)).astype(np.float32)
    r = to_np(gen.rollout_device(n, T, "random", init_qpos=iq, actions=acts))
    orc = Oracle(arm_model_nocontact)
    st = orc.new_state(n)
    s0 = orc.reset(st, init_qpos=iq.astype(np.float32).astype(np.float64))
    np.testing.assert_allclose(r[0, :, 5:], s0, atol=2e-6)
    np.testing.assert_allclose(r[:, :, :5], acts, atol=0)
    s1 = orc.step(st, acts[0].astype(np.float64))
    np.testing.assert_allclose(r[1, :, 5:], s1, atol=5e-4)
    # sin / chirp (SineInputGenerator, :31-74): the device generator's inputs equal the reference
    # formula over t = 0..200 (float32 of the float64 value), and the rows replay on the oracle
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import DeviceSine, SineInputGenerator
    for mode in ("sin", "chirp"):
        sg = SineInputGenerator(n, 5, (0.0025, 0.05), (-0.5, 0.5), mode=mode, rng=np.random.default_rng(3))
        ds = DeviceSine(sg, gen._env(n).sim.device)
        for t in range(201):
            f = sg.freq_table + ((0.05 - 0.0025) * (t / 200) if mode == "chirp" else 0.0)
            ref = sg.amp_table * np.sin(2 * np.pi * f * t + sg.phase_table)  # :57-74
            np.testing.assert_allclose(to_np(ds(t)), ref.astype(np.float32), rtol=0, atol=1e-7)
        r = to_np(gen.rollout_device(n, T, mode, init_qpos=iq, sine=sg, seed=5))
        np.testing.assert_allclose(r[:, :, :5], np.stack([sg.batch(t) for t in range(T + 1)]), atol=1e-7)
        st = orc.new_state(n)
        orc.reset(st, init_qpos=iq.astype(np.float32).astype(np.float64))
        np.testing.assert_allclose(r[1, :, 5:], orc.step(st, r[0, :, :5].astype(np.float64)), atol=5e-4)


def test_vecenv_api(gpu_lib):
    from lerobot_mujoco_sim2real_amd.SOARM101 import SOARM101Env, SOARM101VecEnv
    env = SOARM101Env()
    assert env.frame_skip == 10 and abs(env.dt - 0.02) < 1e-12 and env.joint_ids == [0, 1, 2, 3, 4]
    obs, info = env.reset(seed=0)
    assert obs.shape == (8,) and obs.dtype == np.float32 and info == {}
    assert np.all(np.abs(obs[3:]) <= 0.3)
    obs2, r, term, trunc, info = env.step(np.zeros(5, np.float32))
    assert obs2.shape == (8,) and r == 0.0 and term is False and trunc is False
    obs, _ = env.reset(options={"initial_state": np.r_[np.full(5, 0.1), np.zeros(5)]})
    np.testing.assert_allclose(obs[3:], 0.1, atol=1e-7)
    venv = SOARM101VecEnv(num_envs=32)
    o, _ = venv.reset(seed=3)
    assert tuple(o.shape) == (32, 8)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_config1_single_env_zero_action_1000_steps(gpu_lib, seed):
    """BASELINE.json configs[0]: one SOARM101Env (reference scene: arm + table, contacts on),
    reset from a seeded initial state, zero action, 1000 env-steps (SOARM101_Env.py:77-142),
    every step through the single-env numpy API, against the fp64 oracle run the same way.

    Under zero action the velocity servo only damps: the arm sinks under gravity onto the table
    within ~1 s and then rests on it, still chattering (kv h / M ~ 3) and creeping.  Per step the
    obs must shadow the oracle within 10x the envelope of fp32-sized perturbations of the oracle
    itself (its running max: the single-env envelope dips at random steps) plus 2e-4; the final
    resting pose is held tighter: the gripper's height above the table within 2e-4 of the
    oracle's, and the whole final obs within 10x the envelope of the last 100 steps + 1e-3."""
    from lerobot_mujoco_sim2real_amd.SOARM101 import SOARM101Env
    env = SOARM101Env()
    T = 1000
    init = np.r_[np.random.default_rng(seed).uniform(-0.3, 0.3, 5), np.zeros(5)]
    init = init.astype(np.float32).astype(np.float64)
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
        assert og.dtype == np.float32 and r == 0.0 and not term and not trunc and info == {}
        oa, ob = orc.step(a, np.zeros((1, 5))), orc.step(b, np.zeros((1, 5)))
        for k in ("qpos", "qvel", "warm"):
            b[k][:] = b[k].astype(np.float32)
        err[t] = np.abs(og - oa[0]).max()
        envl[t] = np.abs(oa[0] - ob[0]).max()
    run = np.maximum.accumulate(envl)
    bad = np.nonzero(err > 10 * run + 2e-4)[0]
    assert bad.size == 0, ("shadowing", bad[:5], err[bad[:5]], run[bad[:5]])
    assert abs(float(og[2]) - float(oa[0, 2])) < 2e-4, (og[2], oa[0, 2])   # resting on the table
    assert float(og[2]) < 0.02                                          # (it did come to rest)
    # (the envelope over the last 100 steps, 2 s at rest: over 20 steps it can dip ~4x, e.g. seed 0
    # at 9.7e-3 with the device at 9.8e-3 against 3.9e-2 one build earlier at the same error scale)
    assert np.abs(og - oa[0]).max() < 10 * envl[-100:].max() + 1e-3
    assert int(env.sim.status.cpu().numpy()[0]) == int(a["status"][0]) == 0


def test_full_size_shard_invariance_and_determinism(gpu_lib):
    """The headline workload at its full size (4096 envs, pick scene, chirp inputs, 25
    env-steps), checked through size-independent properties (no oracle at this size):
    * determinism: a second run from the same reset is bit-identical;
    * shard invariance: the same envs as two batches of 2048 (env_offset = the global env id
      base, as a rank of the env-sharded multi-GPU run holds them) give
      bit-identical obs, qpos and qvel — envs never interact, the draws are keyed by global id;
    * validity: every state finite, no soft reset, the cube's resting contacts present."""
    import torch
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    cm = W.model("contact")
    n, T = 4096, 25

    def run(lo, hi):
        ids = np.arange(lo, hi)
        S = BatchSim(cm, hi - lo)
        q0 = W.initial_qpos(cm, ids, 0)
        S.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0, env_offset=lo)
        tab = {k: (torch.as_tensor(v, dtype=torch.float32, device=S.device) if isinstance(v, np.ndarray) else v)
               for k, v in W.chirp_tables(ids, 0).items()}
        for t in range(T):
            S.step(W.chirp_action(tab, float(t), lib=torch))
        torch.cuda.synchronize()
        return {"obs": S.obs.clone(), "qpos": S.qpos.clone(), "qvel": S.qvel.clone(),
                "status": S.status.clone(), "ncon": S.ncon.clone()}

    a, b = run(0, n), run(0, n)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    h0, h1 = run(0, n // 2), run(n // 2, n)
    assert torch.equal(a["obs"], torch.cat([h0["obs"], h1["obs"]]))
    for k in ("qpos", "qvel"):
        assert torch.equal(a[k], torch.cat([h0[k], h1[k]], 1)), k
    assert bool(torch.isfinite(a["qpos"]).all()) and bool(torch.isfinite(a["qvel"]).all())
    assert int((a["status"] != 0).sum()) == 0
    # the cube's 4 resting contacts on (nearly) every env and substep
    assert float(a["ncon"].sum()) / (n * T * 10) > 3.5


def test_shard_invariance_quad_kernel(gpu_lib, monkeypatch):
    """Config 4's partition (8192 envs per GPU) with the PGS kernel held fixed: the quad kernel
    (SOARM_RS=0) on 8192 envs as one batch and as two shards of 4096 (global env ids), DR scene,
    10 env-steps -- bit-identical.  (The default kernel depends on the per-GPU batch: the row-space
    kernel up to rs_cap = 4096 envs on MI355X, the quad kernel above.  Their fp32 summation orders
    differ, so a batch split across rs_cap -- 8192 as 2 x 4096 -- agrees with the unsplit one to the
    parity bars only, not bit for bit)"""
    import torch
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    monkeypatch.setenv("SOARM_RS", "0")
    cm = W.model("dr")
    n, T = 8192, 10

    def run(lo, hi):
        ids = np.arange(lo, hi)
        S = BatchSim(cm, hi - lo)
        q0 = W.initial_qpos(cm, ids, 0)
        S.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0, env_offset=lo)
        S.set_params(**W.dr_params(ids, 0))
        tab = {k: (torch.as_tensor(v, dtype=torch.float32, device=S.device) if isinstance(v, np.ndarray) else v)
               for k, v in W.chirp_tables(ids, 0).items()}
        for t in range(T):
            S.step(W.chirp_action(tab, float(t), lib=torch))
        torch.cuda.synchronize()
        return {"obs": S.obs.clone(), "qpos": S.qpos.clone(), "qvel": S.qvel.clone()}

    a = run(0, n)
    h0, h1 = run(0, n // 2), run(n // 2, n)
    assert torch.equal(a["obs"], torch.cat([h0["obs"], h1["obs"]]))
    for k in ("qpos", "qvel"):
        assert torch.equal(a[k], torch.cat([h0[k], h1[k]], 1)), k


def test_whole_node_batch_on_one_gpu(gpu_lib):
    """The largest size BASELINE.json names -- config 4's 65536 envs, the whole node's count -- as ONE
    batch on one GPU (the [row][env] offsets, the contact buffer and the scratch slab at their largest):
    3 DR env-steps finite, no soft reset, the cube's resting contacts present, and bit-identical to
    the same envs as two batches of 32768 (global env ids; both above rs_cap: the quad kernel)."""
    import torch
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    cm = W.model("dr")
    n, T = 65536, 3

    def run(lo, hi):
        ids = np.arange(lo, hi)
        S = BatchSim(cm, hi - lo)
        q0 = W.initial_qpos(cm, ids, 0)
        S.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0, env_offset=lo)
        S.set_params(**W.dr_params(ids, 0))
        tab = {k: (torch.as_tensor(v, dtype=torch.float32, device=S.device) if isinstance(v, np.ndarray) else v)
               for k, v in W.chirp_tables(ids, 0).items()}
        for t in range(T):
            S.step(W.chirp_action(tab, float(t), lib=torch))
        torch.cuda.synchronize()
        out = {"obs": S.obs.clone(), "qpos": S.qpos.clone(), "qvel": S.qvel.clone(), "status": S.status.clone(),
               "ncon": S.ncon.clone()}
        S.close()
        return out

    a = run(0, n)
    assert bool(torch.isfinite(a["qpos"]).all()) and bool(torch.isfinite(a["qvel"]).all())
    assert int((a["status"] != 0).sum()) == 0
    assert float(a["ncon"].sum()) / (n * T * 10) > 3.5
    h0, h1 = run(0, n // 2), run(n // 2, n)
    assert torch.equal(a["obs"], torch.cat([h0["obs"], h1["obs"]]))
    for k in ("qpos", "qvel"):
        assert torch.equal(a[k], torch.cat([h0[k], h1[k]], 1)), k


def test_rs_choice_switches_on_a_live_batch(gpu_lib, monkeypatch):
    """SOARM_RS is read per env-step call and is part of the step graph's cache key: a
    batch whose graph was captured with the row-space kernel runs the quad kernel once SOARM_RS=0 --
    bit-identical to a fresh batch stepped with the quad kernel from the same state, and not to the
    row-space step (the two kernels' fp32 summation orders differ)."""
    import torch
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    cm = W.model("contact")
    n = 1024
    ids = np.arange(n)
    q0 = W.initial_qpos(cm, ids, 0)
    tab = W.chirp_tables(ids, 0)

    def fresh():
        S = BatchSim(cm, n)
        S.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
        return S

    def copy(dst, src):
        for k in ("qpos", "qvel", "qacc_warmstart", "ctrl", "status"):
            getattr(dst, k).copy_(getattr(src, k))

    a0, a1 = (torch.as_tensor(W.chirp_action(tab, t), dtype=torch.float32) for t in (0, 1))
    monkeypatch.setenv("SOARM_RS", "1")
    A = fresh()
    for _ in range(3):
        A.step(a0.to(A.device))
    B = fresh()
    copy(B, A)
    D = fresh()
    copy(D, A)
    monkeypatch.setenv("SOARM_RS", "0")
    A.step(a1.to(A.device))  # (its cached graph was captured with the RS kernel)
    B.step(a1.to(B.device))
    monkeypatch.setenv("SOARM_RS", "1")
    D.step(a1.to(D.device))
    torch.cuda.synchronize()
    assert torch.equal(A.qvel, B.qvel) and torch.equal(A.qpos, B.qpos)
    assert not torch.equal(A.qvel, D.qvel)


def test_separating_axis_cache_is_exact(gpu_lib):
    """k_collide's separating-axis cache (soarm_collide.h SepCache) only lets a pair skip an MPR
    run whose answer would be "apart": a batch whose cache was warmed over 80 env-steps of the
    headline workload (arm-cube and arm-table contacts present) and a fresh batch (empty cache)
    loaded with the same state find bit-identical contacts and take a bit-identical env-step."""
    import torch
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    cm = W.model("contact")
    n = 4096
    ids = np.arange(n)
    A = BatchSim(cm, n)
    q0 = W.initial_qpos(cm, ids, 0)
    A.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
    tab = {k: (torch.as_tensor(v, dtype=torch.float32, device=A.device) if isinstance(v, np.ndarray) else v)
           for k, v in W.chirp_tables(ids, 0).items()}
    for t in range(80):
        A.step(W.chirp_action(tab, float(t), lib=torch))
    B = BatchSim(cm, n)
    for k in ("qpos", "qvel", "qacc_warmstart", "ctrl", "status", "ncon"):
        getattr(B, k).copy_(getattr(A, k))
    ca, na = A.contacts()
    cb, nb = B.contacts()
    assert torch.equal(na, nb) and torch.equal(ca, cb)
    assert int(na.sum()) > 4 * n, "no arm contacts in the sample"
    act = W.chirp_action(tab, 80.0, lib=torch)
    oa, ob = A.step(act).clone(), B.step(act).clone()
    assert torch.equal(oa, ob)
    for k in ("qpos", "qvel", "ncon"):
        assert torch.equal(getattr(A, k), getattr(B, k)), k


@pytest.mark.parametrize("t0", [20, 60, 100])
def test_contact_env_step_late_states_full_size(gpu_lib, t0):
    """The graph-captured 10-substep contact sim_step (the headline's launch sequence) against one
    oracle env-step, from bench states at t0 = 20 (the driver's window), 60 and 100 (the cube
    resting, arm-table and arm-cube contacts in some envs) at the headline's 4096 envs.  Bars ~10x the measured fp32 / fp64 spread
    (profiles/r03_newton_gap.json env_step pgs_device_vs_pgs_fp64: obs p50 6e-8, p99 1.3e-7, max
    1.2e-5; cube qvel p50 5e-7, p99 4e-5, max 1.4e-4)."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    n = 4096
    cm, orc, st, _ = _bench_states("contact", n, t0, nthreads=16)
    a = W.chirp_action(W.chirp_tables(np.arange(n)), t0).astype(np.float32)
    S = make_sim(cm, n)
    st["ncon"][:] = 0
    load_state(S, st)
    og = to_np(S.step(a))  # graph replay of geom + 10 x (collide, substep)
    env = fp32_noise_envelope(orc, st, a.astype(np.float64), nthreads=16)
    oc = orc.step(st, a.astype(np.float64), nthreads=16)
    assert st["ncon"].sum() > (4 * 10 * n if t0 >= 60 else 3.5 * 10 * n), "contacts in the sample"
    assert_pct(np.abs(og - oc).max(1), 1e-6, 2e-6, 2e-4, what="obs")
    # over 10 substeps an env whose arm pushes the cube can see fp32 / fp64 PGS stop a sweep apart
    # in several substeps (r03 on 4096 envs at t = 100: cube qvel p50 5e-7, p99 4.2e-5, max 2.3e-3)
    dv = np.abs(to_np(S.qvel).T - st["qvel"])
    assert_pct(dv[:, 6:].max(1), 5e-6, 5e-4, CUBE_QVEL_MAX, what="cube qvel")
    # the arm's: r03-r05 one env of 4096 (2624) at 3.2e-2 -- a grazing arm-link contact on the table
    # whose fp32 MPR normal tilted by up to 5 degrees; fixed in r06 (soarm_collide.h mpr: the final
    # depth and normal in fp64; tools/env_diverge.py)
    assert_pct(dv[:, :6].max(1), 5e-6, 5e-5, ARM_QVEL_MAX, what="arm qvel")
    _within_noise_envelope(dv, env)
    np.testing.assert_allclose(to_np(S.qpos).T[:, 6:9], st["qpos"][:, 6:9], atol=5e-6)
    assert int((to_np(S.status) != 0).sum()) == int((st["status"] != 0).sum())
    assert abs(float(to_np(S.ncon).sum()) - float(st["ncon"].sum())) <= 1e-4 * float(st["ncon"].sum())


def _contact_divergence(cm, n, T, t0, rng):
    """Envelope of the pick scene: fp64 oracle vs the same oracle re-rounded to fp32 after every
    env-step, from bench states at t0, chirp inputs."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    _, _, st, _ = _bench_states("contact", n, t0)
    tab = W.chirp_tables(np.arange(n))
    acts = np.stack([W.chirp_action(tab, t0 + t) for t in range(T)]).astype(np.float32).astype(np.float64)
    orc = Oracle(cm)
    a = {k: v.copy() for k, v in st.items()}
    b = {k: v.copy() for k, v in st.items()}
    dev = []
    for t in range(T):
        oa, ob = orc.step(a, acts[t], nthreads=8), orc.step(b, acts[t], nthreads=8)
        for k in ("qpos", "qvel", "warm"):
            b[k][:] = b[k].astype(np.float32)
        dev.append(np.abs(oa - ob))
    return st, acts, np.stack(dev)


def test_contact_trajectory_shadowing(gpu_lib, cube_model):
    """Pick scene, 20 env-steps from t = 60 bench states: the GPU's fp32 trajectory stays within 10x
    the envelope of fp32-sized perturbations of the fp64 oracle (as test_trajectory_shadowing for
    the contact-free scene)."""
    cm = cube_model
    n, T = 512, 20
    st, acts, envelope = _contact_divergence(cm, n, T, 60, np.random.default_rng(11))
    S, orc = make_sim(cm, n), Oracle(cm)
    ref = {k: v.copy() for k, v in st.items()}
    load_state(S, st)
    for t in range(T):
        e = np.abs(to_np(S.step(acts[t].astype(np.float32))) - orc.step(ref, acts[t], nthreads=8))
        env = envelope[t]
        assert np.median(e) <= 10 * np.median(env) + 1e-5, (t, np.median(e), np.median(env))
        assert np.quantile(e, 0.9) <= 10 * np.quantile(env, 0.9) + 2e-4, (t, np.quantile(e, 0.9))
    # the cube stays with its shadow too (not in obs): position after T steps
    assert_pct(np.abs(to_np(S.qpos).T[:, 6:9] - ref["qpos"][:, 6:9]).max(1), 1e-4, 2e-3, 5e-2, what="cube pos")


def _exact_newton_substep(cm, st):
    o = Oracle(cm, solver="newton", tolerance=0.0)
    s = {k: v.copy() for k, v in st.items()}
    o.step(s, None, nsub=1, nthreads=16)
    return s


def test_pgs_vs_reference_newton(gpu_lib):
    """Fidelity to what the reference computes: its scene has no <option>, so mj_step runs MuJoCo's
    default Newton solver (SOARM101/SO101/scene_with_table_v.xml:1-32, SOARM101_Env.py:131-132).
    The device's PGS (north star) against the exact optimum of the same constraint problem (oracle
    Newton, tolerance 0), one substep from bench states at t = 20 and 120: every arm-contact env of
    the 4096 bench envs (oracle census; 3 at t = 20, 13 at t = 120) plus 1024 block envs.  Bars from
    the 4096-env measurement (profiles/r05_rs_bars.json): block envs (cube resting) cube qvel
    p50 1.9e-5 / 3.6e-5, p99 3.6e-5, max 3.7e-5; arm-contact envs cube qvel p99 6.5e-3 / max
    7.1e-3, arm qvel p99 2.3e-4 / max 2.4e-4; arm qvel elsewhere <= 1.2e-7."""
    for t0 in (20, 120):
        cm, orc, st4, _ = _bench_states("contact", 4096, t0, nthreads=16)
        names = cm.geom_names
        table, cube = names.index("table"), names.index("cube")
        arm4 = np.array([any({int(c[7]), int(c[8])} != {table, cube} for c in
                             orc.forward(st4["qpos"][i], st4["qvel"][i], st4["ctrl"][i], st4["warm"][i])["contacts"])
                         for i in range(4096)])
        pick = np.r_[np.flatnonzero(arm4), np.flatnonzero(~arm4)[:1024]]
        st = {k: v[pick].copy() for k, v in st4.items()}
        arm = arm4[pick]
        n = len(pick)
        ref = _exact_newton_substep(cm, st)
        S = make_sim(cm, n)
        load_state(S, st)
        S.substeps(1)
        dv = np.abs(to_np(S.qvel).T - ref["qvel"])
        assert_pct(dv[~arm, 6:].max(1), 4e-5, 5e-5, 1e-4, what=f"t{t0} block envs cube qvel")
        assert_pct(dv[~arm, :6].max(1), 1e-6, 1e-6, 2e-6, what=f"t{t0} block envs arm qvel")
        assert arm.any(), "arm contacts in the 4096 bench states"
        # arm-contact envs: bars at ~2x the measured PGS-vs-exact-optimum gap (r03_newton_gap.json,
        # device PGS: cube qvel p50 3.6e-5 / max 7.1e-3, arm qvel p50 4.5e-6 / max 2.4e-4) -- the PGS
        # algorithm's own distance, identical in the fp64 oracle PGS, which the device PGS must match
        # within QVEL_BARS (with fewer than 8 such envs -- t = 20 -- the median is one env's gap and
        # only the max bars apply).  r05, 4096 envs at t = 120 (tools/rs_bars.py): cube qvel p99
        # 6.5e-3 / max 7.1e-3, arm qvel p99 2.3e-4 / max 2.4e-4 -- the oracle's own PGS is 7.1e-3 /
        # 1.9e-4 from the optimum
        few = arm.sum() < 8
        assert_pct(dv[arm, 6:].max(1), 1.3e-2 if few else 8e-5, 1.3e-2, 1.4e-2,
                   what=f"t{t0} arm-contact envs cube qvel")
        assert_pct(dv[arm, :6].max(1), 5e-4 if few else 1e-5, 5e-4, 5e-4, what=f"t{t0} arm-contact envs arm qvel")
        pgs = {k: v[arm].copy() for k, v in st.items()}
        orc.step(pgs, None, nsub=1)
        dp = np.abs(to_np(S.qvel).T[arm] - pgs["qvel"]).max(1)
        # device PGS against the oracle's mj_solPGS on the same rows (r05 4096 envs: arm-contact
        # envs p99 2.1e-4 / max 2.4e-4 at t = 120, 9.4e-5 / 9.6e-5 at t = 20)
        assert_pct(dp, 1e-4, 3e-4, 5e-4, what=f"t{t0} device PGS vs oracle PGS, arm-contact envs")


@pytest.mark.parametrize("t0", [20, 120])
def test_newton_solver_matches_oracle(gpu_lib, t0):
    """solver="Newton" (MuJoCo's default, what the reference's scene runs; soarm_newton.h) on the
    device against the oracle's Newton (oracle.c orc_solve_newton, exact optimum): one substep
    from bench states of the pick scene, 1024 envs, and one graph-captured env-step."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    cmp, orc, st, _ = _bench_states("contact", 1024, t0, nthreads=16)
    cm = W.model("contact", solver="Newton")
    ref = _exact_newton_substep(cm, st)
    S = make_sim(cm, 1024)
    load_state(S, st)
    S.substeps(1)
    dv = np.abs(to_np(S.qvel).T - ref["qvel"])
    assert_pct(dv.max(1), 1e-5, 5e-5, 5e-4, what="qvel")  # r03: p50 2.5e-6, p99 3.9e-6, max 6.9e-6
    dw = np.abs(to_np(S.qacc_warmstart).T - ref["warm"])  # = qacc
    assert_pct(dw.max(1), 1e-3, 1e-2, 0.25, what="qacc")
    a = W.chirp_action(W.chirp_tables(np.arange(1024)), t0).astype(np.float32)
    load_state(S, st)
    og = to_np(S.step(a))
    s2 = {k: v.copy() for k, v in st.items()}
    oc = Oracle(cm, solver="newton", tolerance=0.0).step(s2, a.astype(np.float64), nthreads=16)
    assert_pct(np.abs(og - oc).max(1), 1e-6, 2e-6, 2e-4, what="obs")


def test_newton_zone_prediction_same_optimum(gpu_lib):
    """The Newton zone prediction (soarm_newton.h: the first iteration takes the frictionloss rows'
    zones of two substeps back when the last two differ) changes the path, not the optimum: after
    4 device substeps from t = 100 bench states (each env's zone history filled), one more substep
    against the oracle's exact Newton from the device's own state, and against a fresh batch
    (empty history) from the same state."""
    from lerobot_mujoco_sim2real_amd import workloads as W
    _, _, st, _ = _bench_states("contact", 1024, 100, nthreads=16)
    cm = W.model("contact", solver="Newton")
    S = make_sim(cm, 1024)
    load_state(S, st)
    S.substeps(4)
    s4 = dict(st)
    s4.update(qpos=to_np(S.qpos).T, qvel=to_np(S.qvel).T, warm=to_np(S.qacc_warmstart).T,
              ctrl=to_np(S.ctrl).T)
    ref = _exact_newton_substep(cm, s4)
    S.substeps(1)
    F = make_sim(cm, 1024)
    load_state(F, s4)
    F.substeps(1)
    v = to_np(S.qvel).T
    assert_pct(np.abs(v - ref["qvel"]).max(1), 1e-5, 5e-5, 5e-4, what="qvel vs oracle")
    assert_pct(np.abs(v - to_np(F.qvel).T).max(1), 1e-5, 5e-5, 5e-4, what="with vs without history")


def test_newton_solver_contact_free(gpu_lib):
    """Newton on the contact-free scene (frictionloss + limits): fused k_step vs the oracle."""
    from lerobot_mujoco_sim2real_amd import mjcf
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML, disable_contact=True, solver="Newton")
    n = 1024
    orc = Oracle(cm, tolerance=0.0)
    st = random_states(cm, orc, n, lo=-1.8, hi=1.8, rng=np.random.default_rng(5))  # limits active too
    S = make_sim(cm, n)
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    np.testing.assert_allclose(to_np(S.qpos).T, st["qpos"], atol=2e-6)
    assert_pct(np.abs(to_np(S.qvel).T - st["qvel"]).max(1), 2e-6, 2e-5, 5e-4, what="qvel")


def test_model_file_runs_identically(gpu_lib, cube_model, tmp_path):
    """A model loaded from its compiled file (sim_model_load, the C caller's from_xml_path) runs
    the pick scene bit-identically to the model compiled in Python: reset + 5 chirp env-steps."""
    import torch
    from lerobot_mujoco_sim2real_amd import abi, workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim, SimModel
    path = tmp_path / "cube.soarm"
    cube_model.save(str(path))
    n = 256
    ids = np.arange(n)
    q0 = W.initial_qpos(cube_model, ids, 0)
    tab = W.chirp_tables(ids, 0)
    out = []
    for h in (None, SimModel.from_file(str(path), abi.load_lib())):
        S = BatchSim(cube_model, n, 0, model_handle=h)
        S.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
        for t in range(5):
            S.step(W.chirp_action(tab, t).astype(np.float32))
        torch.cuda.synchronize()
        out.append((to_np(S.obs), to_np(S.qpos), to_np(S.qvel)))
    for a, b in zip(*out):
        np.testing.assert_array_equal(a, b)


def test_native_ccd_centred_symmetric_overlap_device(gpu_lib, tmp_path):
    """ADVICE r4 on the device: a mesh cube centred inside the table box, axis-aligned, a quarter
    turn and random turns (test_oracle.test_native_ccd_centred_symmetric_overlap).  GJK ends with
    the origin on its simplex; the completion (soarm_collide.h gjk_complete) must give the
    oracle's contact: depth within 2e-6, normal up to sign within 1e-5."""
    from lerobot_mujoco_sim2real_amd import mjcf
    from test_cpu_backend import check_probe_contacts
    from test_oracle import probe_states, write_probe_scene
    cm = mjcf.compile_mjcf(write_probe_scene(tmp_path))
    qs = probe_states(cm)
    check_probe_contacts(cm, make_sim(cm, len(qs)), qs)
