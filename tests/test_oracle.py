"""The float64 CPU oracle pinned by analytic known answers.

MuJoCo is absent and the reference may not be run, so the
oracle's parity with mj_step is unpinned; these tests pin its physics by
independent constructions instead.
"""
import numpy as np
import pytest

from lerobot_mujoco_sim2real_amd import abi, mjcf
from conftest import cube_qpos
from oracle import Oracle

RNG = np.random.default_rng(1234)


def _poses(n, lo=-1.0, hi=1.0):
    q = np.zeros((n, 6))
    q[:, :5] = RNG.uniform(lo, hi, (n, 5))
    return q


def test_mass_matrix_vs_jacobian_sum(arm_model_nocontact):
    """CRBA M == sum_b (m J_p'J_p + J_r' I J_r) + armature, SPD."""
    orc = Oracle(arm_model_nocontact)
    for q in _poses(8):
        M = orc.forward(q)["M"]
        Mn = mjcf.NumpyKinematics(arm_model_nocontact).forward_position(q).mass_matrix()
        np.testing.assert_allclose(M, Mn, atol=1e-14)
        assert np.all(np.linalg.eigvalsh(M) > 0.028 - 1e-9)


def test_gravity_is_potential_gradient(arm_model_nocontact):
    cm = arm_model_nocontact
    orc = Oracle(cm)

    def V(q):
        k = mjcf.NumpyKinematics(cm).forward_position(q)
        return sum(cm.desc.body_mass[b] * 9.81 * k.xipos[b][2] for b in range(cm.desc.nbody))

    for q in _poses(4):
        g = np.array([(V(q + 1e-6 * e) - V(q - 1e-6 * e)) / 2e-6 for e in np.eye(6)])
        np.testing.assert_allclose(orc.forward(q, np.zeros(6))["bias"], g, atol=1e-8)


def test_coriolis_is_lagrangian(arm_model_nocontact):
    """bias(q, v) - g(q) == dM/dt v - 1/2 d(v'Mv)/dq  (Euler-Lagrange)."""
    cm = arm_model_nocontact
    orc = Oracle(cm)
    Mq = lambda q: mjcf.NumpyKinematics(cm).forward_position(q).mass_matrix()
    for q in _poses(3):
        v = RNG.normal(size=6)
        dM = [(Mq(q + 1e-6 * e) - Mq(q - 1e-6 * e)) / 2e-6 for e in np.eye(6)]
        cor = sum(dM[i] * v[i] for i in range(6)) @ v - 0.5 * np.array([v @ dM[i] @ v for i in range(6)])
        b = orc.forward(q, v)["bias"] - orc.forward(q, np.zeros(6))["bias"]
        np.testing.assert_allclose(b, cor, atol=1e-8)


def test_passive_energy_decreases():
    """kv = 0 (no servo): damping + frictionloss only dissipate (ctrl irrelevant)."""
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML, kv=0.0, disable_contact=True)
    orc = Oracle(cm)
    n = 8
    st = orc.new_state(n)
    orc.reset(st, init_qpos=RNG.uniform(-0.5, 0.5, (n, 5)), init_qvel=RNG.uniform(-2, 2, (n, 5)))

    def energy(i):
        q, v = st["qpos"][i], st["qvel"][i]
        k = mjcf.NumpyKinematics(cm).forward_position(q)
        V = sum(cm.desc.body_mass[b] * 9.81 * k.xipos[b][2] for b in range(cm.desc.nbody))
        return 0.5 * v @ k.mass_matrix() @ v + V

    E0 = np.array([energy(i) for i in range(n)])
    for _ in range(5):
        orc.step(st, None, nsub=10)
        E1 = np.array([energy(i) for i in range(n)])
        assert np.all(E1 < E0 + 1e-6)
        E0 = E1


def test_frictionloss_rows_bounded(arm_model_nocontact):
    orc = Oracle(arm_model_nocontact)
    for q in _poses(6):
        out = orc.forward(q, RNG.normal(size=6), ctrl=RNG.uniform(-2, 2, 6))
        f = out["efc_force"][:6]
        assert np.all(np.abs(f) <= 0.052 + 1e-12)


def test_stiction_holds_small_torque():
    """Zero gravity, kv = 0, at rest: a 0.03 N m applied-by-bias torque is below
    frictionloss 0.052 -> the soft friction row cancels most of it."""
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML, kv=0.0, disable_contact=True)
    cm.desc.gravity[:] = [0, 0, 0]
    for a in range(6):  # motor-like: force = gain * ctrl
        cm.desc.actuator_gainprm[a] = 1.0
        cm.desc.actuator_biasprm[a][:] = [0, 0, 0]
    orc = Oracle(cm)
    q = np.zeros(6)
    free = orc.forward(q, np.zeros(6), ctrl=np.r_[0, 0, 0, 0, 0.03, 0])
    cm.desc.dof_frictionloss[4] = 0.0
    nofric = Oracle(cm).forward(q, np.zeros(6), ctrl=np.r_[0, 0, 0, 0, 0.03, 0])
    cm.desc.dof_frictionloss[4] = 0.052
    assert abs(free["qacc"][4]) < 0.15 * abs(nofric["qacc"][4])
    assert abs(free["efc_force"][4]) < 0.052  # not saturated


def test_hill_climb_equals_brute_force(arm_model):
    orc = Oracle(arm_model)
    d = arm_model.desc
    dirs = RNG.normal(size=(400, 3))
    for g in range(d.ngeom):
        if d.geom_type[g] != abi.GEOM_MESH:
            continue
        a = orc.hull_support(g, dirs, True)
        b = orc.hull_support(g, dirs, False)
        v = arm_model.hull_vert[d.geom_hulladr[g]: d.geom_hulladr[g] + d.geom_hullnum[g]].astype(np.float64)
        np.testing.assert_allclose((v[a] * dirs).sum(1), (v[b] * dirs).sum(1), atol=1e-12)


def test_library_support_query_equals_brute_force(cube_model):
    """The kernels' hull support query (soarm_collide.h hull_support: the cube-map cell's record, then
    one-trip climbing records carrying their neighbours' coordinates), compiled for the host through
    the CPU backend's test hook, against the brute-force argmax over every hull vertex: random
    directions, the cube map's face centres / edges / corners and directions just off them (where a
    start cell's vertex is furthest from the answer), for every mesh of the pick scene."""
    import ctypes as C
    from lerobot_mujoco_sim2real_amd import sim as simmod
    lib = abi.load_lib()
    h = simmod.SimModel.of(cube_model, lib)
    d = cube_model.desc
    rng = np.random.default_rng(11)
    axes = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float64)
    special = [s * a for a in axes for s in (1, -1)]
    special += [np.array([sx, sy, sz], np.float64) for sx in (1, -1) for sy in (1, -1) for sz in (1, -1)]
    special += [a + b for i, a in enumerate(special[:6]) for b in special[:6][i + 1:] if np.abs(a + b).sum() > 0]
    special = np.array(special)
    jitter = special[None] + 1e-3 * rng.normal(size=(8, len(special), 3))
    dirs = np.concatenate([rng.normal(size=(4000, 3)), special, jitter.reshape(-1, 3)]).astype(np.float32)
    lib.soarm_test_hull_support.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
    nmesh = 0
    for g in range(d.ngeom):
        if d.geom_type[g] != abi.GEOM_MESH:
            continue
        nmesh += 1
        out = np.zeros_like(dirs)
        abi.check(lib, lib.soarm_test_hull_support(h.ptr, g, dirs.ctypes.data, len(dirs), out.ctypes.data))
        v = cube_model.hull_vert[d.geom_hulladr[g]: d.geom_hulladr[g] + d.geom_hullnum[g]].astype(np.float64)
        # the answer is a hull vertex ...
        ids = np.abs(out[:, None, :].astype(np.float64) - v[None]).sum(2).argmin(1)
        np.testing.assert_array_equal(v[ids].astype(np.float32), out)
        # ... whose support value is the maximum: exact for > 99% of these directions (> 99.8% of random ones), the rest within the
        # fp32 rounding of the climb's dot products (20000 directions per mesh: <= 1.8e-8 m)
        dd = dirs.astype(np.float64)
        best = (dd @ v.T).max(1)
        got = (dd * out).sum(1)
        scale = np.abs(v).max() * np.linalg.norm(dd, axis=1)
        assert np.all(got >= best - 5e-7 * scale), (g, np.max(best - got))
        assert np.mean(got >= best) > 0.99
    assert nmesh >= 10


def test_cube_rests_on_table(cube_model):
    """Cube settles on the table: 4 box-box contacts, sum of normal forces = m g."""
    cm = cube_model
    orc = Oracle(cm)
    n = 1
    st = orc.new_state(n)
    ex = cube_qpos(cm, n, np.random.default_rng(0))
    orc.reset(st, extra_qpos=ex)
    for _ in range(30):
        orc.step(st, np.zeros((n, 5)))
    out = orc.forward(st["qpos"][0], st["qvel"][0], st["ctrl"][0], st["warm"][0])
    cube_g = cm.geom("cube")
    con = [c for c in out["contacts"] if int(c[8]) == cube_g or int(c[7]) == cube_g]
    assert len(con) == 4
    for c in con:
        np.testing.assert_allclose(c[4:7], [0, 0, 1], atol=1e-6)
        assert -2e-3 < c[0] < 0
    nf = len(out["efc_force"]) - 4 * out["ncon"]
    fn = out["efc_force"][nf:].sum()  # every pyramid edge carries its force along the normal
    assert abs(fn - 0.03 * 9.81) < 0.02 * 0.03 * 9.81
    assert np.abs(st["qvel"][0][6:]).max() < 1e-3


def test_table_penetration_depth(arm_model):
    """Gripper pushed into the table: MPR depth == table top - lowest hull point, normal +z."""
    cm = arm_model
    orc = Oracle(cm)
    d = cm.desc
    table = cm.geom("table")
    # fold the arm down until a gripper hull dips into the table top (z = -0.0009)
    q = np.array([0.0, 1.2, 0.2, 1.2, 0.0, 0.0])
    kin = mjcf.NumpyKinematics(cm).forward_position(q)
    found = 0
    for k in range(d.npair):
        if d.pair_geom1[k] != table:
            continue
        g = d.pair_geom2[k]
        p, R = kin.geom_pose(g)
        v = cm.hull_vert[d.geom_hulladr[g]: d.geom_hulladr[g] + d.geom_hullnum[g]].astype(np.float64)
        zmin = (p + v @ R.T)[:, 2].min()
        depth = -0.0009 - zmin
        con = orc.collide(q, table, g)
        if depth > 1e-4:
            assert len(con) == 1
            found += 1
            np.testing.assert_allclose(-con[0][0], depth, rtol=2e-2, atol=1e-5)
            np.testing.assert_allclose(con[0][4:7], [0, 0, 1], atol=3e-2)
        elif depth < -1e-4:
            assert len(con) == 0
    assert found >= 1


def test_ik_converges_on_fig8(arm_model):
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import cartesian_targets
    orc = Oracle(arm_model)
    tp = 1.6 + 0.02 * np.linspace(0, 300, 300)
    xyz = cartesian_targets("Fig8", tp)
    q = np.zeros(6)
    for p in xyz[:40]:
        qn, ok, it = orc.ik(p[None], q[None])
        assert ok[0]
        q = qn[0]
        kin = mjcf.NumpyKinematics(arm_model).forward_position(q)
        assert np.linalg.norm(kin.site_xpos(arm_model.desc.obs_site) - p) < 1e-6


def test_pose_ik_converges(arm_model):
    """dm_control qpos_from_site_pose with target_quat (TrajectoryGenerator.py:96-107, rot_weight 0.5):
    poses the arm itself reaches (5 dofs) are recovered from a perturbed start."""
    orc = Oracle(arm_model)
    s = arm_model.desc.obs_site
    kin = mjcf.NumpyKinematics(arm_model)
    n = 40
    qt = np.zeros((n, 6))
    qt[:, :5] = RNG.uniform(-0.8, 0.8, (n, 5))
    tp = np.array([kin.forward_position(q).site_xpos(s) for q in qt])
    tq = np.array([kin.forward_position(q).site_xquat(s) for q in qt])
    q0 = qt + np.c_[RNG.uniform(-0.15, 0.15, (n, 5)), np.zeros(n)]
    qn, ok, it = orc.ik(tp, q0, target_quat=tq)
    assert ok.mean() > 0.9
    for e in np.nonzero(ok)[0]:
        k = kin.forward_position(qn[e])
        assert np.linalg.norm(k.site_xpos(s) - tp[e]) < 1e-6
        assert min(np.abs(k.site_xquat(s) - tq[e]).max(), np.abs(k.site_xquat(s) + tq[e]).max()) < 4e-6
    # a quaternion target of the opposite sign is the same rotation (quat2vel's > pi branch)
    qm, okm, _ = orc.ik(tp, q0, target_quat=-tq)
    np.testing.assert_array_equal(okm, ok)
    np.testing.assert_allclose(qm[ok], qn[ok], atol=1e-9)


def test_pose_ik_reference_default_orientation(arm_model):
    """generate()'s default target_orientation [1, 0, 0, 0] (TrajectoryGenerator.py:118) over the
    Fig8 path: a 5-dof arm cannot hold an arbitrary orientation, so points fail and generate()
    repeats the last good solution (:193-205); the ones that succeed meet both criteria."""
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_DataCollection import cartesian_targets
    orc = Oracle(arm_model)
    tp = 1.6 + 0.02 * np.linspace(0, 300, 300)
    xyz = cartesian_targets("Fig8", tp)
    q, ok, it = orc.ik(xyz, np.zeros((300, 6)), target_quat=np.array([1.0, 0, 0, 0]))
    kin = mjcf.NumpyKinematics(arm_model)
    s = arm_model.desc.obs_site
    for e in np.nonzero(ok)[0][:20]:
        k = kin.forward_position(q[e])
        assert np.linalg.norm(k.site_xpos(s) - xyz[e]) < 1e-6
    assert (it[~ok] < 100).all() or (~ok).sum() == 0  # failures are progress stalls, not the cap


def test_golden_regression(arm_model_nocontact):
    """Committed fixtures (tests/golden/make_golden.py) — the oracle must keep reproducing them."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_arm_random.npz"))
    orc = Oracle(arm_model_nocontact)
    n = z["init_qpos"].shape[0]
    st = orc.new_state(n)
    obs = [orc.reset(st, init_qpos=z["init_qpos"])]
    for a in z["actions"]:
        obs.append(orc.step(st, a))
    np.testing.assert_allclose(np.stack(obs), z["obs"], atol=1e-9)


def _world_hull(cm, xp, xm, g):
    """World-frame vertices of geom g's convex shape (box corners or mesh hull)."""
    d = cm.desc
    if d.geom_type[g] == abi.GEOM_BOX:
        h = np.array(d.geom_size[g])
        loc = np.array([[sx * h[0], sy * h[1], sz * h[2]] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
    else:
        a, nv = d.geom_hulladr[g], d.geom_hullnum[g]
        loc = cm.hull_vert[a:a + nv].astype(np.float64)
    return xp[g] + loc @ xm[g].T


@pytest.mark.parametrize("xml", ["arm", "cube"])
def test_native_ccd_is_minimum_penetration(xml):
    """The oracle's native GJK/EPA (oracle_collision.c, MuJoCo's nativeccd restated) returns the
    minimum penetration of each convex-convex contact: with h(d) = max_A x.d - min_B x.d the
    Minkowski difference's support, its normal n has h(n) = depth within the EPA tolerance, and no
    sampled direction d has h(d) < depth (the depth is the minimum over directions).  MPR, also
    checked, satisfies h(n) >= depth only (it is not a minimum-depth method).

    Native-CCD parity with MuJoCo itself is unpinned (no MuJoCo nativeccd fixtures exist here; the
    oracle's EPA visibility threshold, stalled-GJK hand-off and gjk_complete follow the kernel's
    choices, r05): this geometric check is what pins it, here on the GPU contact test's poses and
    in test_native_ccd_minimum_penetration_stress_poses on the stress poses of tools/ccd_mismatch.py."""
    _minimum_penetration(xml, 48, None, ("native", "mpr"))


def test_native_ccd_minimum_penetration_stress_poses():
    """The same minimum-penetration check of the oracle's native GJK/EPA over the stress poses that
    drove the r05 EPA / GJK changes (tools/ccd_mismatch.py's generator and seed 7: gripper into the
    table, folded arm), both scenes, 256 poses each (MuJoCo parity unpinned, see above)."""
    for xml in ("arm", "cube"):
        _minimum_penetration(xml, 256, 7, ("native",))


def _minimum_penetration(xml, npose, seed, ccds):
    import test_gpu_parity as T  # (the poses of the GPU contact test)
    path = mjcf.SCENE_XML if xml == "arm" else mjcf.CUBE_SCENE_XML
    rng = np.random.default_rng(5)
    dirs = rng.normal(size=(6000, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    for ccd in ccds:
        cm = mjcf.compile_mjcf(path, ccd=ccd)
        orc = Oracle(cm)
        prng = T.RNG if seed is None else np.random.default_rng(seed)
        q = T._contact_poses(cm, npose, prng)
        full = cube_qpos(cm, npose, np.random.default_rng(3) if seed is None else prng, q) if cm.nq > 6 else q
        n_conv, gaps = 0, []
        for e in range(len(full)):
            xp, xm = orc.geom_frames(full[e])
            for r in orc.forward(full[e])["contacts"]:
                g1, g2 = int(r[7]), int(r[8])
                if not (cm.desc.geom_type[g1] in (abi.GEOM_BOX, abi.GEOM_MESH) and cm.desc.geom_type[g2] == abi.GEOM_MESH):
                    continue
                A, B = _world_hull(cm, xp, xm, g1), _world_hull(cm, xp, xm, g2)
                n, depth = r[4:7], -r[0]
                hn = (A @ n).max() - (B @ n).min()
                assert hn >= depth - 2e-6, (e, g1, g2, hn, depth)  # both: the depth is reached along n
                if ccd == "native":
                    gaps.append(hn - depth)
                    hmin = ((A @ dirs.T).max(0) - (B @ dirs.T).min(0)).min()
                    assert hmin >= depth - 1e-9, (e, g1, g2, hmin, depth)  # never deeper than the minimum
                n_conv += 1
        assert n_conv >= 20, (ccd, n_conv)
        if gaps:
            # converged to the EPA tolerance (h(n) = depth within 2e-6) but for the polytope-budget exits
            # (EPA_KV / EPA_KF full on a deep mesh-mesh self contact: the closest face so far, a lower
            # bound) -- measured on the stress poses: 7 of 1112 (arm) and 4 of 1105 (cube) convex contacts, max 5.2e-6
            g = np.array(gaps)
            assert (g > 2e-6).mean() <= 0.02 and g.max() <= 5e-5, (int((g > 2e-6).sum()), len(g), g.max())


# ---- centred, centrally symmetric convex overlap (GJK ends with the origin ON its simplex)
PROBE_H = 0.03
TABLE_C, TABLE_H = np.array([0.0, 0.0, -0.1009]), np.array([0.61, 0.37, 0.1])


def write_probe_scene(dirpath, h=PROBE_H):
    """The arm, floor and table box plus one free body whose geom is an inline-vertex MESH cube
    of half-size h (MJCF ``<mesh vertex=...>``): the table/probe pair runs the convex-convex
    narrowphase (box vs mesh) instead of box_box."""
    corners = " ".join(f"{sx * h} {sy * h} {sz * h}" for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1))
    xml = f"""<mujoco model="probe">
  <include file="{mjcf.ASSET_DIR}/so101_new_calib_v.xml"/>
  <asset><mesh name="probe" vertex="{corners}"/></asset>
  <worldbody>
    <geom name="floor" size="0 0 0.05" pos="0 0 -.75" type="plane"/>
    <geom name="table" pos="0 0 -0.1009" size="0.61 0.37 0.1" type="box" class="collision"/>
    <body name="probe" pos="0.3 0 0.2">
      <freejoint name="probe_free"/>
      <inertial pos="0 0 0" mass="0.05" diaginertia="2e-5 2e-5 2e-5"/>
      <geom name="probe" type="mesh" mesh="probe"/>
    </body>
  </worldbody>
</mujoco>"""
    path = str(dirpath / "probe_scene.xml")
    with open(path, "w") as f:
        f.write(xml)
    return path


def probe_states(cm, n_random=6, seed=11):
    """qpos with the probe centred on the table box: axis-aligned, a quarter turn, random turns."""
    rng = np.random.default_rng(seed)
    quats = [np.array([1.0, 0, 0, 0]), np.array([np.cos(np.pi / 4), 0, 0, np.sin(np.pi / 4)])]
    quats += [q / np.linalg.norm(q) for q in rng.normal(size=(n_random, 4))]
    qs = np.zeros((len(quats), cm.nq))
    qs[:, 6:9] = TABLE_C
    qs[:, 9:13] = quats
    return qs


def test_native_ccd_centred_symmetric_overlap(tmp_path):
    """a mesh cube centred inside the table box.  A - B is centrally symmetric, so
    GJK's second support point is exactly minus its first and the origin lands ON the segment:
    the old shortcut called that touching and reported no contact.  nativeccd starts EPA from
    such simplices (polytope2 / polytope3; the oracle's gjk_complete): the contact must exist and
    be the minimum penetration -- h(n) = depth and no sampled direction below it; axis-aligned,
    depth = table half-height + h exactly, along z."""
    cm = mjcf.compile_mjcf(write_probe_scene(tmp_path))
    assert cm.desc.ccd == 1
    orc = Oracle(cm)
    gt, gp = cm.geom_names.index("table"), cm.geom_names.index("probe")
    dirs = np.random.default_rng(5).normal(size=(20000, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    for i, q in enumerate(probe_states(cm)):
        rc = [r for r in orc.forward(q)["contacts"] if {int(r[7]), int(r[8])} == {gt, gp}]
        assert len(rc) == 1, (i, rc)
        r = rc[0]
        xp, xm = orc.geom_frames(q)
        A, B = _world_hull(cm, xp, xm, gt), _world_hull(cm, xp, xm, gp)
        n, depth = r[4:7], -r[0]
        assert abs((A @ n).max() - (B @ n).min() - depth) <= 2e-6, (i, depth)
        assert ((A @ dirs.T).max(0) - (B @ dirs.T).min(0)).min() >= depth - 1e-9, (i, depth)
        if i < 2:
            assert abs(depth - (TABLE_H[2] + PROBE_H)) <= 1e-9 and abs(abs(n[2]) - 1) <= 1e-9, (i, r)
