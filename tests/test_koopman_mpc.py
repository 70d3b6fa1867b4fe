"""Batched Koopman-MPC (include/koopman_mpc.h) against the float64 oracle.

The reference solves the MPC with casadi/IPOPT (absent here; running the reference is denied,
SURVEY.md §8c), so the oracle (oracle/koopman_mpc.py) restates the reference's cost loop and
minimises it exactly; these tests first pin that minimiser (zero gradient and positive curvature
of the literal cost), then hold the product to it:

* host gains (control/koopman.condensed_gains, a different construction) == oracle minimiser, 1e-9;
* GPU encoder (f64 MFMA) == numpy float64 MLP, 1e-12 relative;
* GPU control step (encoder + feedforward + gains) == oracle get_control, 1e-9 absolute;
* qfrc_bias / qfrc_applied in the physics == the oracle's, fp32 tolerances as test_gpu_parity;
* the batched tracking loop: every frame's action == the oracle MPC on the GPU's own state.

Weights are random (the reference's checkpoint is not used: DESIGN.md §9 records why), drawn with
the reference's initialisers (control/koopman.py).
"""
import ctypes as C
import json
import math

import numpy as np
import pytest

import koopman_mpc as KO
from oracle import Oracle

import soarm_pkg  # noqa: F401
from lerobot_mujoco_sim2real_amd.utility.ZMQ import ZMQCommunicator, real_targets, sim_to_real

RNG = np.random.default_rng(11)
LAYERS = [8, 64, 64, 64, 64, 24]


class _Args:
    x_dim, u_dim, model, layers = 8, 5, "DKUC", LAYERS

    def __init__(self, kind="delta_mpc"):
        self.MPC_type = kind


def make_net(seed=0):
    import torch
    from lerobot_mujoco_sim2real_amd.control.koopman import Koopmanlinear
    torch.manual_seed(seed)
    return Koopmanlinear(8, 5, LAYERS).double()


def net_mats(net):
    return (net.lA.weight.detach().numpy().astype(np.float64), net.lB.weight.detach().numpy().astype(np.float64),
            net.encoder_layers())


def sample_states(n):
    """[n, 8] plausible SO-ARM101 states: ee xyz, 5 joint angles."""
    return np.concatenate([RNG.uniform([0.1, -0.2, 0.0], [0.45, 0.2, 0.35], (n, 3)),
                           RNG.uniform(-1.0, 1.0, (n, 5))], 1)


# ------------------------------------------------------------------ CPU: oracle + host
@pytest.mark.parametrize("kind", ["delta_mpc", "mpc"])
def test_oracle_minimises_the_reference_cost(kind):
    """The oracle's solution is the minimiser of the reference's cost loop
    (control/MPC_Controler.py:80-86 / :115-127): gradient 0, every perturbation costs more."""
    net = make_net(1)
    A, B, layers = net_mats(net)
    H, nz = 10, 32
    z0 = KO.encode(layers, sample_states(1))[0]
    ref = KO.encode(layers, sample_states(H))
    up = RNG.uniform(-0.5, 0.5, 5)
    v = KO.solve(A, B, z0[None], ref[None], up[None], kind)[0].ravel()
    J0 = KO.cost(A, B, v, z0, ref, up, kind)
    h = 1e-6
    g = np.array([(KO.cost(A, B, v + h * e, z0, ref, up, kind) - KO.cost(A, B, v - h * e, z0, ref, up, kind)) / (2 * h)
                  for e in np.eye(v.size)])
    scale = max(1.0, abs(J0))
    assert np.abs(g).max() < 1e-5 * scale
    for _ in range(20):
        d = RNG.normal(0, 1e-3, v.size)
        assert KO.cost(A, B, v + d, z0, ref, up, kind) > J0


def test_oracle_encoder_matches_torch():
    """x_encoder = cat([x, MLP(x)]) (models/KoopmanBase.py:45-47) in float64."""
    import torch
    net = make_net(2)
    x = sample_states(257)
    want = net.x_encoder(torch.as_tensor(x)).detach().numpy()
    got = KO.encode(net.encoder_layers(), x)
    np.testing.assert_allclose(got, want, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("kind", ["delta_mpc", "mpc"])
def test_condensed_gains_equal_oracle_minimiser(kind):
    """u0 = Gr r + Gz z0 + Gu u_prev (host closed form) == oracle get_control u0."""
    from lerobot_mujoco_sim2real_amd.control.koopman import condensed_gains
    net = make_net(3)
    A, B, layers = net_mats(net)
    n, H = 64, 10
    z0 = KO.encode(layers, sample_states(n))
    ref = KO.encode(layers, sample_states(n * H)).reshape(n, H, -1)
    up = RNG.uniform(-0.5, 0.5, (n, 5))
    Gr, Gz, Gu = condensed_gains(A, B, H, kind)
    u0 = ref.reshape(n, -1) @ Gr.T + z0 @ Gz.T + up @ Gu.T
    want, _ = KO.get_control(A, B, z0, ref, up, kind)
    np.testing.assert_allclose(u0, want, rtol=1e-9, atol=1e-9)


def make_bnet(seed=0, u_z=False, scale=0.02):
    """DBKN (KoopmanBlinear) with a random bilinear layer (the reference zero-initialises it)."""
    import torch
    from lerobot_mujoco_sim2real_amd.control.koopman import KoopmanBlinear
    torch.manual_seed(seed)
    net = KoopmanBlinear(8, 5, LAYERS, u_z).double()
    with torch.no_grad():
        net.H.weight.normal_(0.0, scale)
    return net


@pytest.mark.parametrize("u_z", [False, True])
def test_bilinear_model_is_its_linearisation(u_z):
    """KoopmanBlinear.koopman_operation (KoopmanBase.py:68-80) == A z + (Bd + Σ_j z_j Ĥ_j) u with
    Ĥ_j from get_Hi_numpy (:104-110): the identity linearize_B (MPC_Controler.py:46-63) relies on,
    for both Kronecker orders."""
    import torch
    net = make_bnet(7, u_z)
    A, B, layers = net_mats(net)
    Hhat = net.get_Hi_numpy()
    z = KO.encode(layers, sample_states(16))
    u = RNG.uniform(-0.5, 0.5, (16, 5))
    got = net.koopman_operation(torch.as_tensor(z), torch.as_tensor(u)).detach().numpy()
    want = np.stack([A @ z[i] + KO.b_total(B, Hhat, z[i]) @ u[i] for i in range(16)])
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("kind", ["delta_mpc", "mpc"])
def test_bilinear_first_move_equals_oracle(kind):
    """control/koopman.bilinear_first_move (block-structured batched QP, torch float64; here on the
    CPU as a unit test of its algebra) == the oracle's per-env restatement of the reference's cost
    loop with B_total(z0); the oracle's minimiser is pinned by the literal cost's gradient."""
    import torch
    from lerobot_mujoco_sim2real_amd.control.koopman import bilinear_first_move
    net = make_bnet(8)
    A, B, layers = net_mats(net)
    Hhat = net.get_Hi_numpy()
    n, H = 24, 10
    z0 = KO.encode(layers, sample_states(n))
    ref = KO.encode(layers, sample_states(n * H)).reshape(n, H, -1)
    up = RNG.uniform(-0.5, 0.5, (n, 5))
    u0 = bilinear_first_move(torch.as_tensor(A), torch.as_tensor(B), torch.as_tensor(np.stack(Hhat)),
                             torch.as_tensor(z0.T.copy()), torch.as_tensor(ref.transpose(1, 2, 0).copy()),
                             torch.as_tensor(up.T.copy()), kind, H).numpy().T
    want, _ = KO.get_control_bilinear(A, B, Hhat, z0, ref, up, kind, H)
    np.testing.assert_allclose(u0, want, rtol=1e-9, atol=1e-9)
    # the oracle's answer minimises the reference's cost with env 0's B_total
    Bt = KO.b_total(B, Hhat, z0[0])
    v = KO.solve(A, Bt, z0[:1], ref[:1], up[:1], kind)[0].ravel()
    h = 1e-6
    g = np.array([(KO.cost(A, Bt, v + h * e, z0[0], ref[0], up[0], kind) -
                   KO.cost(A, Bt, v - h * e, z0[0], ref[0], up[0], kind)) / (2 * h) for e in np.eye(v.size)])
    assert np.abs(g).max() < 1e-5 * max(1.0, abs(KO.cost(A, Bt, v, z0[0], ref[0], up[0], kind)))


def _reference_state_dict_layout(layers, x_dim, u_dim, bilinear):
    """{key: shape} of the state_dict the reference's classes save, restated from their source:
    x_encode_net is nn.Sequential(OrderedDict(linear_i, relu_i)) (models/KoopmanBase.py:20-27;
    ReLU has no parameters), lA [Nk, Nk] (:31), lB [Nk, u_dim] (:35), lC [x_dim, Nk] (:38),
    DBKN's H [Nk, Nk*u_dim] (:66); Nk = layers[-1] + x_dim (:16)."""
    nk = layers[-1] + x_dim
    keys = {}
    for i in range(len(layers) - 1):
        keys[f"x_encode_net.linear_{i}.weight"] = (layers[i + 1], layers[i])
        keys[f"x_encode_net.linear_{i}.bias"] = (layers[i + 1],)
    keys["lA.weight"] = (nk, nk)
    keys["lB.weight"] = (nk, u_dim)
    keys["lC.weight"] = (x_dim, nk)
    if bilinear:
        keys["H.weight"] = (nk, nk * u_dim)
    return keys


@pytest.mark.parametrize("model", ["DKUC", "DBKN"])
def test_reference_state_dict_loads_strict(model):
    """Koopman_MPC.py:262-265 — init_model(args); model.double(); model.load_state_dict(sd) —
    runs unchanged against this build's classes with a state_dict of the reference's key set
    (strict loading: no missing or unexpected keys), and the loaded weights are the ones used."""
    import torch
    from lerobot_mujoco_sim2real_amd.args import Args
    from lerobot_mujoco_sim2real_amd.control.koopman import init_model
    args = Args()
    args.model = model
    layout = _reference_state_dict_layout(list(args.layers), args.x_dim, args.u_dim, model == "DBKN")
    g = torch.Generator().manual_seed(5)
    sd = {k: torch.randn(s, generator=g, dtype=torch.float64) for k, s in layout.items()}
    net = init_model(args)
    net.double()
    res = net.load_state_dict(sd)  # strict=True is the default, as in the reference's call
    assert not res.missing_keys and not res.unexpected_keys
    assert {k: tuple(v.shape) for k, v in net.state_dict().items()} == layout
    W0, b0 = net.encoder_layers()[0]
    np.testing.assert_array_equal(W0, sd["x_encode_net.linear_0.weight"].numpy())
    np.testing.assert_array_equal(b0, sd["x_encode_net.linear_0.bias"].numpy())
    x = torch.as_tensor(sample_states(4))
    np.testing.assert_allclose(net.x_encoder(x).detach().numpy(), KO.encode(net.encoder_layers(), x.numpy()),
                               rtol=1e-13, atol=1e-13)


def test_koopman_create_validates_before_device():
    """Bad shapes -> SIM_E_MODEL; a good controller without a GPU -> SIM_E_NODEVICE (no CPU path)."""
    from lerobot_mujoco_sim2real_amd import abi, build
    build.build()
    lib = abi.load_lib()
    d = abi.KoopmanDesc()
    d.x_dim, d.u_dim, d.nlayer, d.horizon, d.u_clip = 8, 5, 5, 10, 0.5
    for i, w in enumerate(LAYERS):
        d.width[i] = w
    w = np.zeros(100000)
    g = np.zeros(5 * (10 * 32 + 32 + 5))
    h = C.c_void_p()
    d.width[2] = 65
    assert lib.sim_koopman_create(C.byref(d), w.ctypes.data_as(C.c_void_p), g.ctypes.data_as(C.c_void_p), 0,
                                  C.byref(h)) == -2
    d.width[2] = 64
    d.horizon = 40
    assert lib.sim_koopman_create(C.byref(d), w.ctypes.data_as(C.c_void_p), g.ctypes.data_as(C.c_void_p), 0,
                                  C.byref(h)) == -2
    d.horizon = 10
    import torch
    if not torch.cuda.is_available():
        rc = lib.sim_koopman_create(C.byref(d), w.ctypes.data_as(C.c_void_p), g.ctypes.data_as(C.c_void_p), 0,
                                    C.byref(h))
        assert rc == -4 and b"no HIP device" in lib.sim_last_error()


# ------------------------------------------------------------------------- GPU
def _ctl(net, kind="delta_mpc"):
    from lerobot_mujoco_sim2real_amd.control.MPC_Controler import MPCController
    return MPCController(net, _Args(kind))


@pytest.mark.gpu
def test_encode_gpu(gpu_lib):
    net = make_net(4)
    ctl = _ctl(net)
    x = sample_states(1000).astype(np.float32)
    z = ctl.encode(x).cpu().numpy().T
    want = KO.encode(net.encoder_layers(), x.astype(np.float64))
    np.testing.assert_allclose(z, want, rtol=1e-12, atol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["delta_mpc", "mpc"])
def test_control_step_gpu(gpu_lib, kind):
    """lift refs -> feedforward -> mpc_step(x) on the GPU == oracle get_control, for every frame
    of a short reference, including the zero-padded tail windows (Koopman_MPC.py:199-205)."""
    import torch
    net = make_net(5)
    ctl = _ctl(net, kind)
    A, B, layers = net_mats(net)
    T, n, H = 14, 300, 10
    sref = sample_states(T * n).reshape(T, n, 8).astype(np.float32)
    zref_dev = ctl.lift_reference(torch.as_tensor(sref, device=ctl.device))
    ff = ctl.feedforward(zref_dev)
    zref = KO.encode(layers, sref.reshape(T * n, 8).astype(np.float64)).reshape(T, n, -1)
    np.testing.assert_allclose(zref_dev.permute(0, 2, 1).cpu().numpy(), zref, rtol=1e-12, atol=1e-13)
    up0 = RNG.uniform(-0.6, 0.6, (n, 5))
    for k in (0, 5, T - 3, T - 1):
        x = sample_states(n).astype(np.float32)
        up = torch.as_tensor(up0.T.copy(), device=ctl.device)
        a = ctl.step(torch.as_tensor(x, device=ctl.device), ff[k], up).cpu().numpy()
        u0, aw = KO.get_control(A, B, KO.encode(layers, x.astype(np.float64)), KO.lifted_window(zref, k, H), up0, kind)
        np.testing.assert_allclose(up.cpu().numpy().T, u0, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(a, aw.astype(np.float32), atol=1e-6)
        assert (np.abs(a) <= 0.5).all()


@pytest.mark.gpu
def test_get_control_single_env(gpu_lib):
    """MPCController.get_control(p) with the reference's p layout (Koopman_MPC.py:199-213)."""
    net = make_net(6)
    ctl = _ctl(net)
    A, B, layers = net_mats(net)
    ref = KO.encode(layers, sample_states(10))
    z0 = KO.encode(layers, sample_states(1))[0]
    ctl.u_prev = RNG.uniform(-0.3, 0.3, 5)
    p = np.concatenate([ref.ravel(), z0, ctl.u_prev]).reshape(-1, 1)
    u0, a = ctl.get_control(p)
    w0, wa = KO.get_control(A, B, z0[None], ref[None], p[-5:, 0][None])
    np.testing.assert_allclose(u0, w0[0], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(a, wa[0], atol=1e-12)
    np.testing.assert_allclose(ctl.u_prev, wa[0])  # delta_mpc keeps a (MPC_Controler.py:150-151)
    psi = ctl.Psi_o(sample_states(1))
    assert psi.shape == (32, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["delta_mpc", "mpc"])
@pytest.mark.parametrize("H", [10, 7])
def test_bilinear_control_gpu(gpu_lib, kind, H):
    """DBKN: step_bilinear for n envs (HIP lift + the per-env float64 QP kernel k_bilinear) and
    get_control(p) == the oracle's per-env restatement of the reference's cost loop.  H = 10 (the
    reference's horizon, u_dim 5) runs the static-shape instantiation, H = 7 the generic one."""
    import torch
    from lerobot_mujoco_sim2real_amd.control.MPC_Controler import MPCController
    net = make_bnet(9)
    ctl = MPCController(net, _Args(kind), horizon=H)
    assert ctl.bilinear
    A, B, layers = net_mats(net)
    Hhat = net.get_Hi_numpy()
    n = 515  # (not a whole number of 8-env workgroups)
    x = sample_states(n).astype(np.float32)
    ref = KO.encode(layers, sample_states(n * H)).reshape(n, H, -1)
    up0 = RNG.uniform(-0.5, 0.5, (n, 5))
    up = torch.as_tensor(up0.T.copy(), device=ctl.device)
    win = torch.as_tensor(ref.transpose(1, 2, 0).copy(), device=ctl.device)
    a = ctl.step_bilinear(torch.as_tensor(x, device=ctl.device), win, up).cpu().numpy()
    u0, aw = KO.get_control_bilinear(A, B, Hhat, KO.encode(layers, x.astype(np.float64)), ref, up0, kind, H)
    np.testing.assert_allclose(up.cpu().numpy().T, u0, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(a, aw.astype(np.float32), atol=1e-6)
    z0 = KO.encode(layers, sample_states(1))[0]
    ctl.u_prev = RNG.uniform(-0.3, 0.3, 5)
    p = np.concatenate([ref[0].ravel(), z0, ctl.u_prev]).reshape(-1, 1)
    g0, _ = ctl.get_control(p)
    w0, _ = KO.get_control_bilinear(A, B, Hhat, z0[None], ref[:1], p[-5:, 0][None], kind, H)
    np.testing.assert_allclose(g0, w0[0], rtol=1e-9, atol=1e-9)


@pytest.mark.gpu
def test_bias_matches_oracle(gpu_lib, arm_model, cube_model):
    from test_gpu_parity import load_state, random_states, to_np, make_sim
    for cm in (arm_model, cube_model):
        n = 256
        S, orc = make_sim(cm, n), Oracle(cm)
        st = random_states(cm, orc, n)
        if cm.nq > 6:  # the free cube spinning: Coriolis terms on the free body too
            st["qvel"][:, 6:] = RNG.uniform(-1, 1, (n, 6))
        load_state(S, st)
        b = to_np(S.bias()).T
        want = orc.bias(st)
        np.testing.assert_allclose(b, want, atol=2e-5, rtol=1e-4)


@pytest.mark.gpu
def test_step_with_applied_force(gpu_lib, arm_model_nocontact, arm_model):
    """qfrc_applied enters the smooth forces of every substep; a reset zeroes it."""
    import torch
    from test_gpu_parity import load_state, random_states, to_np, make_sim
    for cm in (arm_model_nocontact, arm_model):
        n = 512
        S, orc = make_sim(cm, n), Oracle(cm)
        rng = np.random.default_rng(17)  # its own stream: independent of the other tests' draws
        st = random_states(cm, orc, n, rng=rng)
        load_state(S, st)
        app = rng.uniform(-0.5, 0.5, (n, cm.nv))
        S.enable_qfrc_applied().copy_(torch.as_tensor(app.T, dtype=torch.float32, device=S.device))
        a = rng.uniform(-0.5, 0.5, (n, 5)).astype(np.float32)
        og = to_np(S.step(a))
        app64 = app.astype(np.float32).astype(np.float64)
        st0 = {k: v.copy() for k, v in st.items()}  # (Oracle.step advances st in place)
        oc = orc.step(st, a.astype(np.float64), applied=app64)
        err = np.abs(og - oc).max(1)  # per env
        # a missing or mis-scaled applied force moves every env by ~h^2 |f| / M ~ 1e-3; the bulk is
        # at fp32 resolution.  A few envs whose wrist servo chatters (h kv / M ~ 3, see
        # test_gpu_parity's shadowing tests) amplify fp32 rounding within one env-step: they are
        # held to the oracle's own sensitivity there -- the same env-step from the state with qvel
        # perturbed by one fp32 ulp (the shadowing envelope) -- and p99.9 to 5e-4.
        pert = {k: v.copy() for k, v in st0.items()}  # the same env-step, from the perturbed start state
        pert["qvel"] = np.nextafter(pert["qvel"].astype(np.float32), np.float32(np.inf)).astype(np.float64)
        env = np.abs(orc.step(pert, a.astype(np.float64), applied=app64) - oc).max(1)
        assert np.median(err) < 1e-6 and np.percentile(err, 99) < 5e-5 and np.percentile(err, 99.9) < 5e-4, \
            (np.median(err), np.percentile(err, 99), np.percentile(err, 99.9))
        bad = err > 10 * env + 1e-5
        assert bad.sum() == 0, (np.nonzero(bad)[0], err[bad], env[bad])
        S.reset(init_qpos=np.zeros((n, 5), np.float32))
        assert float(S.qfrc_applied.abs().max()) == 0.0


@pytest.mark.gpu
def test_tracking_loop_matches_oracle(gpu_lib, arm_model):
    """KoopmanMPCTracking: frame by frame, the GPU's action equals the oracle MPC applied to the
    GPU's own state and u_prev (1e-6, the action is float32), and the GPU's next state equals one
    oracle env-step with qfrc_applied = qfrc_bias from that state (fp32 step tolerances)."""
    import torch
    from lerobot_mujoco_sim2real_amd.Koopman_MPC import KoopmanMPCTracking
    net = make_net(7)
    ctl = _ctl(net)
    A, B, layers = net_mats(net)
    T, n = 30, 64
    t = np.linspace(0, 2 * np.pi, T)
    phase = RNG.uniform(0, 2 * np.pi, n)
    cart = np.stack([0.3 + 0.0 * t[:, None] + 0 * phase, 0.1 * np.cos(t[:, None] + phase),
                     0.15 + 0.05 * np.sin(t[:, None] + phase)], -1)
    jq = RNG.uniform(-0.3, 0.3, (1, n, 5)) + 0.1 * np.sin(t[:, None, None] + phase[None, :, None])
    sent = _Sink()
    run = KoopmanMPCTracking(ctl, arm_model, cart, jq, communicator=ZMQCommunicator(socket=sent), stream_env_id=3)
    sref = run.state_all_ref.cpu().numpy().astype(np.float64)
    zref = KO.encode(layers, sref.reshape(T * n, 8)).reshape(T, n, -1)
    orc = Oracle(arm_model)
    run.runBefore()
    for k in range(T):
        x = run.state.cpu().numpy().astype(np.float64)
        up = run.u_prev.cpu().numpy().T.copy()
        c64 = lambda t: np.ascontiguousarray(t.cpu().numpy().T, dtype=np.float64)  # oracle: C order
        st = {"qpos": c64(run.sim.qpos), "qvel": c64(run.sim.qvel), "warm": c64(run.sim.qacc_warmstart),
              "ctrl": c64(run.sim.ctrl),
              "status": run.sim.status.cpu().numpy().copy(), "ncon": np.zeros(n)}
        obs = run.runFunc().cpu().numpy()
        u0, aw = KO.get_control(A, B, KO.encode(layers, x), KO.lifted_window(zref, k, 10), up)
        np.testing.assert_allclose(run.action.cpu().numpy(), aw.astype(np.float32), atol=1e-6)
        np.testing.assert_allclose(run.u_prev.cpu().numpy().T, u0, rtol=1e-9, atol=1e-9)
        applied = orc.bias(st)
        oc = orc.step(st, run.action.cpu().numpy().astype(np.float64), applied=applied)
        err = np.abs(obs - oc)
        assert np.median(err) < 2e-6 and err.max() < 1e-3, (k, np.median(err), err.max())
        # sim -> real: env 3's qpos[:6] after the step, degrees minus joint_offsets (:186-190)
        q = run.sim.qpos[:6, 3].double().cpu().numpy()
        assert json.loads(sent.msgs[-1]) == real_targets(q) and len(sent.msgs) == k + 1
    assert int(run.sim.status.abs().sum()) == 0
    # past the last frame: the reference's return to the "home" keyframe (Koopman_MPC.py:148-183).
    # Frame T builds the 20-point path (no step); frames T+1..T+20 set qpos[:nj] along it and step
    # with home_ctrl; later frames hold home.  Each checked against the oracle doing the same.
    home = np.asarray(arm_model.keyframes["home"]["qpos"], np.float64)
    hctrl = np.asarray(arm_model.keyframes["home"]["ctrl"], np.float64)[:5]
    before = run.sim.qpos.cpu().numpy().copy()
    run.runFunc()
    np.testing.assert_array_equal(run.sim.qpos.cpu().numpy(), before)  # path built, no step
    path = np.linspace(jq[-1].astype(np.float32).astype(np.float64), np.broadcast_to(home[:5], (n, 5)), 20)
    for i in range(24):
        c64 = lambda t: np.ascontiguousarray(t.cpu().numpy().T, dtype=np.float64)  # noqa: E731
        st = {"qpos": c64(run.sim.qpos), "qvel": c64(run.sim.qvel), "warm": c64(run.sim.qacc_warmstart),
              "ctrl": c64(run.sim.ctrl), "status": run.sim.status.cpu().numpy().copy(), "ncon": np.zeros(n)}
        applied = orc.bias(st)  # qfrc_applied = qfrc_bias before qpos is overwritten (:119)
        st["qpos"][:, :5] = (path[i] if i < 20 else np.broadcast_to(home[:5], (n, 5))).astype(np.float32)
        obs = run.runFunc().cpu().numpy()
        oc = orc.step(st, np.broadcast_to(hctrl, (n, 5)).copy(), applied=applied)
        err = np.abs(obs - oc)
        assert np.median(err) < 2e-6 and err.max() < 1e-3, (i, np.median(err), err.max())
    assert len(sent.msgs) == T + 25


@pytest.mark.gpu
def test_bilinear_tracking_loop(gpu_lib, arm_model):
    """KoopmanMPCTracking with a DBKN model: every frame's action equals the oracle's bilinear MPC
    on the GPU's own state and u_prev (its QP linearised at that frame's lifted state)."""
    import torch
    from lerobot_mujoco_sim2real_amd.Koopman_MPC import KoopmanMPCTracking
    net = make_bnet(10)
    ctl = _ctl(net)
    A, B, layers = net_mats(net)
    Hhat = net.get_Hi_numpy()
    T, n = 12, 32
    t = np.linspace(0, 2 * np.pi, T)
    phase = RNG.uniform(0, 2 * np.pi, n)
    cart = np.stack([0.3 + 0.0 * t[:, None] + 0 * phase, 0.1 * np.cos(t[:, None] + phase),
                     0.15 + 0.05 * np.sin(t[:, None] + phase)], -1)
    jq = RNG.uniform(-0.3, 0.3, (1, n, 5)) + 0.1 * np.sin(t[:, None, None] + phase[None, :, None])
    run = KoopmanMPCTracking(ctl, arm_model, cart, jq)
    sref = run.state_all_ref.cpu().numpy().astype(np.float64)
    zref = KO.encode(layers, sref.reshape(T * n, 8)).reshape(T, n, -1)
    run.runBefore()
    for k in range(T):
        x = run.state.cpu().numpy().astype(np.float64)
        up = run.u_prev.cpu().numpy().T.copy()
        run.runFunc()
        u0, aw = KO.get_control_bilinear(A, B, Hhat, KO.encode(layers, x), KO.lifted_window(zref, k, 10), up)
        np.testing.assert_allclose(run.u_prev.cpu().numpy().T, u0, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(run.action.cpu().numpy(), aw.astype(np.float32), atol=1e-6)
    assert torch.isfinite(run.sim.qpos).all()


class _Sink:
    """Stands in for the PUB socket: records what would be published."""

    def __init__(self):
        self.msgs = []

    def send_string(self, s):
        self.msgs.append(s)


def test_sim_to_real_payload():
    """The published list equals the reference's conversion (Koopman_MPC.py:16-27,186-189):
    degrees(qpos[:6]) - joint_offsets, JSON-encoded by send_data (utility/ZMQ.py:36-51)."""
    q = [0.1, -0.2, 0.3, 0.0, 1.0, -0.5]
    expect = [math.degrees(v) - o for v, o in zip(q, [0, 0, 0, 0, 0, -41.97])]
    assert real_targets(q) == expect
    assert sim_to_real([10.0, 0, 0, 0, 0, 0.0]) == [10.0, 0, 0, 0, 0, 41.97]
    sink = _Sink()
    c = ZMQCommunicator(socket=sink)
    c.send_data(expect)
    assert sink.msgs == [json.dumps(expect)]
    c.cleanup()
    c.send_data(expect)  # no socket: nothing sent (the reference prints and returns)
    assert len(sink.msgs) == 1


def test_zmq_transport_fails_loudly_without_pyzmq():
    try:
        import zmq  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError, match="pyzmq"):
            ZMQCommunicator("tcp://127.0.0.1:5555")
    else:
        pytest.skip("pyzmq present")
