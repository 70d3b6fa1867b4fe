"""The Koopman model the MPC controller lifts states with.

Reference: ``models/KoopmanBase.py:12-60`` (``Koopmanlinear``, the ``DKUC`` model that
``init_model`` builds, ``models/init_model.py:4-10``) with ``encode_layers = [x_dim, 64, 64, 64,
64, 24]`` (``args.py:103``), so ``Nkoopman = 24 + x_dim = 32``.  Only what the controller needs
is kept: the encoder ``x_encoder(x) = cat([x, MLP(x)])``, the Koopman matrices ``lA``
(Nkoopman x Nkoopman, initialised as 0.9 x an orthogonalised Gaussian draw) and ``lB``
(Nkoopman x u_dim), and the fixed decoder ``lC = [I | 0]``.  Training the model (``train.py``,
``models/losses.py``) is out of scope; a user's own trained state_dict loads with
``load_state_dict`` as usual.

The bilinear ``DBKN`` model (``KoopmanBlinear``, ``:62-110``) makes the MPC's input matrix depend
on the lifted state (``MPC_Controler.py:46-63``), i.e. a different QP Hessian per env and frame;
it is not built here.
"""
import numpy as np
import torch
from torch import nn


class Koopmanlinear(nn.Module):
    """DKUC: z_{k+1} = lA z_k + lB u_k with z = [x, MLP(x)]."""

    def __init__(self, x_dim, u_dim, encode_layers):
        super().__init__()
        self.x_dim, self.u_dim = x_dim, u_dim
        self.Nkoopman = encode_layers[-1] + x_dim
        mods = []
        for i, (a, b) in enumerate(zip(encode_layers[:-1], encode_layers[1:])):
            mods.append(nn.Linear(a, b))
            if i + 2 < len(encode_layers):
                mods.append(nn.ReLU())
        self.x_encode_net = nn.Sequential(*mods)
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


def init_model(args):
    """``models/init_model.py:2-21``: DKUC only (see the module docstring for DBKN)."""
    if args.model == "DKUC":
        return Koopmanlinear(args.x_dim, args.u_dim, args.layers)
    if args.model == "DBKN":
        raise NotImplementedError("DBKN (bilinear Koopman): the MPC's input matrix depends on z0 "
                                  "(MPC_Controler.py:46-63); only the linear DKUC model is built")
    raise ValueError(f"Model {args.model} not implemented!")


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
