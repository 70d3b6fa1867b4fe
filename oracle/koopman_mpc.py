"""Float64 restatement of the reference's Koopman-MPC tracking path.

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` (and nothing in the product) as the
checker of ``sim_koopman_*`` (include/koopman_mpc.h).

What it restates, following the reference's own code order:

* ``Koopmanlinear.x_encoder`` (``models/KoopmanBase.py:20-25,45-47``): Linear layers with a
  ReLU between consecutive layers (none after the last), output ``cat([x, feat])``;
  ``MPCController.Psi_o`` (``control/MPC_Controler.py:154-167``) returns it as a column.
* ``MPCController.setup_mpc`` / ``setup_delta_mpc`` (``control/MPC_Controler.py:65-141``) with
  ``state_full = True`` (``:35-40``: the test ``args.model == 'IBKN' or 'IKN'`` is always true,
  so Q = 50 I_Nkoopman and R = 0.5 I_u); for the linear model (DKUC: no ``H`` layer)
  ``B_total = Bd``, for the bilinear DBKN ``B_total = Bd + sum_j z0_j H_hat_j`` at the frame's
  lifted state (``linearize_B``, ``:46-63``; :func:`get_control_bilinear`).  The cost loop is restated literally: z and u_t are carried
  as affine functions of the decision vector through ``z_next = Ad z + B u_t`` in the loop's
  order, and the quadratic it builds is minimised exactly (normal equations).  ``nlpsol`` is
  called with no bounds (``:145``), so this minimiser is the point IPOPT converges to.
* ``get_control`` (``:143-152``): ``u0 = u_opt[0] + u_eso + u_prev``, ``a = clip(u0, +-0.5)``.
* ``Test.runMPC`` / ``runFunc`` (``Koopman_MPC.py:114-136,197-222``): lifted references
  ``Psi_o(state_all_ref[k+1 .. k+H])`` with zero rows past the end (``:199-205``), ``z0 =
  Psi_o(state)`` where state is ``state_all_ref[0]`` on the first frame (``:91``) and the last
  observation afterwards (``:221``), ``u_prev <- u0`` (``:219``), gravity compensation
  ``qfrc_applied = qfrc_bias`` before every env.step (``:119``).

Parity of this restatement against casadi/IPOPT itself is unpinned (casadi is absent and the
reference cannot be run here); it is pinned by the optimality test in
``tests/test_koopman_mpc.py`` (zero gradient of the literal cost, positive curvature) and by
torch's own ``nn.Linear``/``ReLU`` forward for the encoder.
"""
import numpy as np

Q_STATE_FULL = 50.0  # control/MPC_Controler.py:39
R_STATE_FULL = 0.5   # control/MPC_Controler.py:40
U_CLIP = 0.5         # control/MPC_Controler.py:149


def encode(layers, x):
    """z = [x, MLP(x)]; layers = [(W [out, in], b [out]), ...] float64; x [m, x_dim]."""
    h = np.asarray(x, np.float64)
    for i, (W, b) in enumerate(layers):
        h = h @ np.asarray(W, np.float64).T + np.asarray(b, np.float64)
        if i + 1 < len(layers):
            h = np.maximum(h, 0.0)
    return np.concatenate([np.asarray(x, np.float64), h], axis=-1)


def _quadratic(A, B, H, kind, Q, R):
    """Hessian and the affine pieces of the reference's cost loop in the decision vector v.

    Returns (Hess [Hu, Hu], terms) where terms lists per step t the affine map of z_{t+1}:
    z_{t+1} = Mz_t v + Pz_t z0 + Pu_t u_prev (the loop keeps z0 and u_prev symbolic too)."""
    nz, nu = B.shape
    nv = H * nu
    Mz, Pz, Pu = np.zeros((nz, nv)), np.eye(nz), np.zeros((nz, nu))  # z = z0
    Mu, Cu = np.zeros((nu, nv)), np.eye(nu)                           # u_t = u_prev (delta form)
    Hs = np.zeros((nv, nv))
    terms = []
    for t in range(H):
        E = np.zeros((nu, nv))
        E[:, t * nu:(t + 1) * nu] = np.eye(nu)
        if kind == "delta_mpc":          # u_t = u_t + delta_u_t   (:117)
            Mu = Mu + E
            Mut, Cut = Mu, Cu
            Mpen = E                     # cost term delta_u_t' R delta_u_t   (:126)
        else:                            # u_t = u[t]   (:83)
            Mut, Cut = E, np.zeros((nu, nu))
            Mpen = E                     # cost term u_t' R u_t   (:85)
        # z_next = Ad z + B_total u_t   (:84 / :118)
        Mz = A @ Mz + B @ Mut
        Pz = A @ Pz
        Pu = A @ Pu + B @ Cut
        terms.append((Mz.copy(), Pz.copy(), Pu.copy()))
        Hs += 2 * Q * (Mz.T @ Mz) + 2 * R * (Mpen.T @ Mpen)
    return Hs, terms


def prepare(A, B, H=10, kind="delta_mpc", Q=Q_STATE_FULL, R=R_STATE_FULL):
    """The cost's quadratic for (A, B, H, kind), reusable across calls (it depends on nothing else)."""
    A, B = np.asarray(A, np.float64), np.asarray(B, np.float64)
    return (A, B, H, kind, Q) + _quadratic(A, B, H, kind, Q, R)


def solve(A, B, z0, ref, u_prev, kind="delta_mpc", H=10, Q=Q_STATE_FULL, R=R_STATE_FULL, qp=None):
    """Minimiser of the reference's MPC cost for each env.

    z0 [n, nz], ref [n, H, nz] (lifted, zero rows past the trajectory end), u_prev [n, nu].
    Returns the decision vector reshaped [n, H, nu] (u_opt of get_control, :146).
    qp: prepare(A, B, H, kind) to skip rebuilding the quadratic."""
    if qp is None:
        qp = prepare(A, B, H, kind, Q, R)
    A, B, H, kind, Q, Hs, terms = qp
    nz, nu = B.shape
    z0 = np.atleast_2d(z0)
    n = z0.shape[0]
    ref = np.asarray(ref, np.float64).reshape(n, H, nz)
    u_prev = np.atleast_2d(u_prev).reshape(n, nu)
    g = np.zeros((n, H * nu))
    for t, (Mz, Pz, Pu) in enumerate(terms):
        c = z0 @ Pz.T + u_prev @ Pu.T - ref[:, t]   # z_{t+1} - ref_t at v = 0
        g += 2 * Q * c @ Mz
    v = np.linalg.solve(Hs, -g.T).T
    return v.reshape(n, H, nu)


def cost(A, B, v, z0, ref, u_prev, kind="delta_mpc", H=10, Q=Q_STATE_FULL, R=R_STATE_FULL):
    """The reference's cost (control/MPC_Controler.py:80-86 / :115-127) evaluated by its own loop
    at decision vector v [H*nu] for ONE env (used to pin `solve`)."""
    A, B = np.asarray(A, np.float64), np.asarray(B, np.float64)
    nu = B.shape[1]
    z = np.asarray(z0, np.float64).copy()
    u_t = np.asarray(u_prev, np.float64).copy()
    J = 0.0
    for t in range(H):
        d = v[t * nu:(t + 1) * nu]
        if kind == "delta_mpc":
            u_t = u_t + d
        else:
            u_t = d
        z = A @ z + B @ u_t
        e = z - ref[t]
        J += Q * e @ e + R * d @ d
    return J


def get_control(A, B, z0, ref, u_prev, kind="delta_mpc", H=10, u_eso=None, qp=None):
    """(u0, a) of MPCController.get_control (:143-152) for n envs."""
    v = solve(A, B, z0, ref, u_prev, kind, H, qp=qp)
    u0 = v[:, 0] + np.atleast_2d(u_prev) + (0.0 if u_eso is None else u_eso)
    return u0, np.clip(u0, -U_CLIP, U_CLIP)


def b_total(B, Hhat, z0):
    """linearize_B (MPC_Controler.py:46-63): B_total = Bd + sum_j z0[j] * H_hat_j for ONE env.
    Hhat: the DBKN model's get_Hi_numpy() list (KoopmanBase.py:104-110), z0 [nz]."""
    Bt = np.asarray(B, np.float64).copy()
    for j, Hj in enumerate(Hhat):
        Bt += float(z0[j]) * np.asarray(Hj, np.float64)
    return Bt


def get_control_bilinear(A, B, Hhat, z0, ref, u_prev, kind="delta_mpc", H=10):
    """(u0, a) of get_control for a DBKN model, n envs: each env's QP is built by the reference's
    cost loop with its own B_total(z0) (setup_mpc / setup_delta_mpc pass z0 as a parameter and
    linearise B at it once, :72-73 / :107-108)."""
    z0 = np.atleast_2d(z0)
    n = z0.shape[0]
    ref = np.asarray(ref, np.float64).reshape(n, H, -1)
    u_prev = np.atleast_2d(u_prev)
    u0 = np.zeros((n, np.asarray(B).shape[1]))
    for e in range(n):
        Bt = b_total(B, Hhat, z0[e])
        v = solve(A, Bt, z0[e:e + 1], ref[e:e + 1], u_prev[e:e + 1], kind, H)
        u0[e] = v[0, 0] + u_prev[e]
    return u0, np.clip(u0, -U_CLIP, U_CLIP)


def lifted_window(zref, k, H):
    """Lifted reference rows k+1 .. k+H of zref [T, n, nz], zero past the end (Koopman_MPC.py:199-205)."""
    T, n, nz = zref.shape
    out = np.zeros((n, H, nz))
    for t in range(H):
        if k + 1 + t < T:
            out[:, t] = zref[k + 1 + t]
    return out


def closed_loop(orc, layers, A, B, state_ref, frames, kind="delta_mpc", H=10, init_q=None):
    """Test.runBefore + `frames` x runFunc/runMPC (Koopman_MPC.py:84-136,197-222) for n envs on
    the float64 physics oracle.  state_ref [T, n, 8] = [cartesian xyz, joint angles] per frame.
    Returns (obs [frames, n, 8], actions [frames, n, nu])."""
    T, n, _ = state_ref.shape
    zref = encode(layers, state_ref.reshape(T * n, -1)).reshape(T, n, -1)
    st = orc.new_state(n)
    q0 = state_ref[0, :, 3:8] if init_q is None else init_q
    orc.reset(st, init_qpos=q0)
    x = state_ref[0]
    u_prev = np.zeros((n, B.shape[1]))
    obs_out, act_out = [], []
    for k in range(frames):
        applied = orc.bias(st)                                 # qfrc_applied = qfrc_bias (:119)
        z0 = encode(layers, x)
        u0, a = get_control(A, B, z0, lifted_window(zref, k, H), u_prev, kind, H)
        u_prev = u0                                            # :219
        obs = orc.step(st, a, applied=applied)
        x = obs.astype(np.float32).astype(np.float64)          # obs is float32 (SOARM101_Env.py:75)
        obs_out.append(obs)
        act_out.append(a)
    return np.stack(obs_out), np.stack(act_out)
