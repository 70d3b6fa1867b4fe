"""The Koopman model the MPC controller lifts states with.

Reference: ``models/KoopmanBase.py:12-60`` (``Koopmanlinear``, the ``DKUC`` model that
``init_model`` builds, ``models/init_model.py:4-10``) with ``encode_layers = [x_dim, 64, 64, 64,
64, 24]`` (``args.py:103``), so ``Nkoopman = 24 + x_dim = 32``.  Only what the controller needs
is kept: the encoder ``x_encoder(x) = cat([x, MLP(x)])``, the Koopman matrices ``lA``
(Nkoopman x Nkoopman, initialised as 0.9 x an orthogonalised Gaussian draw) and ``lB``
(Nkoopman x u_dim), and the fixed decoder ``lC = [I | 0]``.  Training the model (``train.py``,
``models/losses.py``) is out of scope.  Parameter names are the reference's
(``x_encode_net.linear_{i}``, ``lA``, ``lB``, ``lC``, DBKN's ``H``), so a state_dict the reference
saved loads with ``load_state_dict(..., strict=True)`` (``tests/test_koopman_mpc.py``).

The bilinear ``DBKN`` model (``KoopmanBlinear``, ``:62-110``) adds ``H (z ⊗ u)`` to the step;
the MPC linearises it at the frame's lifted state, ``B_total = Bd + Σ_j z0_j Ĥ_j``
(``MPC_Controler.py:46-63``), so its QP differs per env and frame: :func:`bilinear_first_move`
solves those QPs batched in float64 on the device.
"""
from collections import OrderedDict

import numpy as np
import torch
from torch import nn


class Koopmanlinear(nn.Module):
    """DKUC: z_{k+1} = lA z_k + lB u_k with z = [x, MLP(x)]."""

    def __init__(self, x_dim, u_dim, encode_layers):
        super().__init__()
        self.x_dim, self.u_dim = x_dim, u_dim
        self.Nkoopman = encode_layers[-1] + x_dim
        # named modules linear_{i} / relu_{i} as KoopmanBase.py:20-27, so the reference's saved
        # state_dict (x_encode_net.linear_0.weight, ...) loads strictly (Koopman_MPC.py:262-265)
        mods = OrderedDict()
        for i, (a, b) in enumerate(zip(encode_layers[:-1], encode_layers[1:])):
            mods[f"linear_{i}"] = nn.Linear(a, b)
            if i + 2 < len(encode_layers):
                mods[f"relu_{i}"] = nn.ReLU()
        self.x_encode_net = nn.Sequential(mods)
        self.u_encode_net = nn.Identity()
        nk = self.Nkoopman
        self.lA = nn.Linear(nk, nk, bias=False)
        g = torch.randn(nk, nk) / nk  # N(0, (1/nk)^2) as gaussian_init_ (KoopmanBase.py:7-10)
        U, _, V = torch.svd(g)
        self.lA.weight.data = (U @ V.t()) * 0.9
        self.lB = nn.Linear(u_dim, nk, bias=False)
        self.lC = nn.Linear(nk, x_dim, bias=False)
        with torch.no_grad():
            self.lC.weight.zero_()
            self.lC.weight[:, :x_dim] = torch.eye(x_dim)
        self.lC.weight.requires_grad = False

    def x_encoder(self, x):
        return torch.cat([x, self.x_encode_net(x)], dim=-1)

    def x_decoder(self, x_emb):
        return self.lC(x_emb)

    def koopman_operation(self, x_emb, u_emb):
        return self.lA(x_emb) + self.lB(u_emb)

    def u_encoder(self, x, u):
        return self.u_encode_net(u)

    def u_decoder(self, u_emb):
        return u_emb

    def encoder_layers(self):
        """[(W [out, in], b [out]) float64 numpy] of x_encode_net, in order."""
        return [(m.weight.detach().double().cpu().numpy(), m.bias.detach().double().cpu().numpy())
                for m in self.x_encode_net if isinstance(m, nn.Linear)]


class KoopmanBlinear(Koopmanlinear):
    """DBKN (``KoopmanBase.py:62-110``): z_{k+1} = lA z + lB u + H vec(z ⊗ u) (``u_z``: vec(u ⊗ z)),
    H: Linear(Nkoopman * u_dim -> Nkoopman), zero-initialised."""

    def __init__(self, x_dim, u_dim, encode_layers, u_z=False):
        super().__init__(x_dim, u_dim, encode_layers)
        self.H = nn.Linear(self.Nkoopman * self.u_dim, self.Nkoopman, bias=False)
        nn.init.zeros_(self.H.weight)
        self.u_z = u_z

    def koopman_operation(self, x_emb, u_emb):
        lin = self.lA(x_emb) + self.lB(u_emb)
        if self.u_z:
            kron = torch.einsum("bi,bj->bij", u_emb, x_emb).reshape(x_emb.shape[0], -1)
        else:
            kron = torch.einsum("bi,bj->bij", x_emb, u_emb).reshape(x_emb.shape[0], -1)
        return lin + self.H(kron)

    def build_permutation_matrix(self, n, m):
        """P with P vec(u ⊗ z) = vec(z ⊗ u) when u_z (identity otherwise), ``:84-95``."""
        if not self.u_z:
            return np.eye(n * m)
        P = np.zeros((n * m, n * m))
        for i in range(n):
            for j in range(m):
                P[j * n + i, i * m + j] = 1
        return P

    def get_Hi_numpy(self):
        """[Ĥ_j (Nkoopman x u_dim) for j < Nkoopman]: H vec(z ⊗ u) = Σ_j z_j Ĥ_j u (``:104-110``)."""
        P = self.build_permutation_matrix(self.u_dim, self.Nkoopman)
        Hd = self.H.weight.detach().double().cpu().numpy() @ P.T
        return [Hd[:, j * self.u_dim:(j + 1) * self.u_dim].copy() for j in range(self.Nkoopman)]


def init_model(args):
    """``models/init_model.py:2-21``: DKUC (linear) or DBKN (bilinear, ``args.u_z``)."""
    if args.model == "DKUC":
        return Koopmanlinear(args.x_dim, args.u_dim, args.layers)
    if args.model == "DBKN":
        return KoopmanBlinear(args.x_dim, args.u_dim, args.layers, bool(getattr(args, "u_z", False)))
    raise ValueError(f"Model {args.model} not implemented!")


_TOEPLITZ = {}


def _toeplitz_index(H, device):
    """Index tensors of bilinear_first_move's block sums (cached per H and device)."""
    import torch

    key = (H, str(device))
    if key not in _TOEPLITZ:
        D = 2 * H - 1
        da = np.zeros((D, H), np.int64)
        db = np.zeros((D, H), np.int64)
        dm = np.zeros((D, H))
        for di, d in enumerate(range(-(H - 1), H)):
            for a in range(H):
                b = a - d
                if 0 <= b < H:
                    da[di, a], db[di, a], dm[di, a] = a, b, 1.0
        hd = np.zeros((H, H), np.int64)
        ha = np.zeros((H, H), np.int64)
        for s1 in range(H):
            for s2 in range(H):
                hd[s1, s2] = (s2 - s1) + H - 1
                ha[s1, s2] = H - 1 - s1  # (terms with a < max(0, d) are zero-masked)
        ra = np.zeros((H, H), np.int64)
        rt = np.zeros((H, H), np.int64)
        rm = np.zeros((H, H))
        for s in range(H):
            for j, t in enumerate(range(s, H)):
                ra[s, j], rt[s, j], rm[s, j] = t - s, t, 1.0
        T = lambda x: torch.as_tensor(x, device=device)  # noqa: E731
        _TOEPLITZ[key] = {"da": T(da), "db": T(db), "dm": T(dm).double()[None, :, :, None, None],
                          "hd": T(hd), "ha": T(ha), "ra": T(ra), "rt": T(rt),
                          "rm": T(rm).double()[None, :, :, None]}
    return _TOEPLITZ[key]


def bilinear_first_move(A, B, Hhat, z0, window, u_prev, kind, H, q=50.0, r=0.5):
    """First move u0 of the DBKN MPC for n envs (``MPC_Controler.py:46-141``, state_full), float64
    torch tensors on one device: B_total = B + Σ_j z0_j Ĥ_j per env (the reference's
    linearize_B), then the unconstrained QP of the condensed prediction solved exactly.

    A [nz, nz], B [nz, nu], Hhat [nz(j), nz, nu], z0 [nz, n], window [H, nz, n] (lifted reference
    rows k+1 .. k+H, zero past the end), u_prev [nu, n].  Returns u0 = v*_0 + u_prev [nu, n].

    Block structure (no [H nz, H nu] matrix per env): with M_k = A^k B_total, the prediction's
    input blocks are X_{t-s} (X = M for 'mpc', the running sums C_k = Σ_{i<=k} M_i for
    'delta_mpc'), so Hess[s1, s2] = q Σ_{t >= max(s1, s2)} X_{t-s1}' X_{t-s2} + r I and
    rhs[s] = q Σ_{t >= s} X_{t-s}' e_t with e_t = ref_t - A^{t+1} z0 - c_t u_prev (c_t = C_t for
    'delta_mpc': u_prev held, else 0)."""
    import torch

    nz, nu = B.shape
    n = z0.shape[1]
    Bt = B.unsqueeze(0) + torch.einsum("jn,jrk->nrk", z0, Hhat)           # [n, nz, nu]
    P = [torch.eye(nz, dtype=A.dtype, device=A.device)]
    for _ in range(H):
        P.append(A @ P[-1])
    P = torch.stack(P)                                                   # A^0 .. A^H
    M = torch.einsum("kab,nbc->nkac", P[:H], Bt)                         # [n, H, nz, nu]
    C = torch.cumsum(M, dim=1)
    if kind == "delta_mpc":
        X, cu = C, C
    elif kind == "mpc":
        X, cu = M, None
    else:
        raise ValueError(f"MPC_type {kind!r}: 'mpc' or 'delta_mpc'")
    idx = _toeplitz_index(H, A.device)
    W = torch.einsum("nkab,nlac->nklbc", X, X)                           # X_k' X_l [n, H, H, nu, nu]
    # Hess[s1, s2] = q Σ_{t >= max(s1, s2)} W[t - s1, t - s2]: running sums along each diagonal
    # d = s2 - s1 of W (a = t - s1 runs from max(0, d) to H - 1 - s1), gathered per block
    Wd = W[:, idx["da"], idx["db"]] * idx["dm"]                          # [n, 2H-1, H, nu, nu]
    Sd = torch.cumsum(Wd, dim=2)
    Hs = q * Sd[:, idx["hd"], idx["ha"]]                                 # [n, H, H, nu, nu] (s1, s2)
    Hs = Hs.permute(0, 1, 3, 2, 4).reshape(n, H * nu, H * nu)
    Hs = Hs + r * torch.eye(H * nu, dtype=A.dtype, device=A.device)
    Az = torch.einsum("tab,bn->nta", P[1:H + 1], z0)                    # A^{t+1} z0 [n, H, nz]
    e = window.permute(2, 0, 1) - Az                                     # [n, H, nz]
    if cu is not None:
        e = e - torch.einsum("ntab,bn->nta", cu, u_prev)
    # rhs[s] = q Σ_{t >= s} X_{t-s}' e_t
    Y = torch.einsum("nkab,nta->nktb", X, e)                             # X_k' e_t [n, H(k), H(t), nu]
    rhs = q * (Y[:, idx["ra"], idx["rt"]] * idx["rm"]).sum(2)            # [n, H(s), nu]
    rhs = rhs.reshape(n, H * nu)
    L = torch.linalg.cholesky(Hs)
    v = torch.cholesky_solve(rhs.unsqueeze(-1), L)[..., 0]
    return v[:, :nu].T + u_prev


def condensed_gains(A, B, H, kind, q=50.0, r=0.5):
    """Closed-form first move of the unconstrained MPC QP (MPC_Controler.py:65-141, state_full).

    Stacked prediction over t = 0..H-1:  Z = Phi z0 + Gamma U,  Phi = [A; A^2; ...; A^H],
    Gamma[t, s] = A^(t-s) B (s <= t).  'mpc': U are the inputs; 'delta_mpc': U = u_prev 1 + S dU
    with S the block lower-triangular identity.  Minimising
    (Z - Rbar)' (q I) (Z - Rbar) + V' (r I) V  (V = U or dU) gives V* = K (Rbar - Phi z0 - c u_prev)
    and the applied input u0 = V*_0 + u_prev (get_control, :147).  Returns (Gr [nu, H nz],
    Gz [nu, nz], Gu [nu, nu]) with u0 = Gr Rbar + Gz z0 + Gu u_prev."""
    A, B = np.asarray(A, np.float64), np.asarray(B, np.float64)
    nz, nu = B.shape
    P = [np.eye(nz)]
    for _ in range(H):
        P.append(A @ P[-1])
    Phi = np.vstack(P[1:])
    Gam = np.zeros((H * nz, H * nu))
    for t in range(H):
        for s in range(t + 1):
            Gam[t * nz:(t + 1) * nz, s * nu:(s + 1) * nu] = P[t - s] @ B
    if kind == "delta_mpc":
        S = np.kron(np.tril(np.ones((H, H))), np.eye(nu))
        Gd = Gam @ S
        cu = Gam @ np.kron(np.ones((H, 1)), np.eye(nu))  # response to u_prev held
    elif kind == "mpc":
        Gd = Gam
        cu = np.zeros((H * nz, nu))
    else:
        raise ValueError(f"MPC_type {kind!r}: 'mpc' or 'delta_mpc'")
    Hs = q * Gd.T @ Gd + r * np.eye(H * nu)
    K = np.linalg.solve(Hs, q * Gd.T)[:nu]  # first move only
    Gr = K
    Gz = -K @ Phi
    Gu = np.eye(nu) - K @ cu
    return Gr, Gz, Gu
