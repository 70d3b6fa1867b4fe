"""MPCController: the reference's Koopman-MPC, batched on the GPU.

Reference: ``control/MPC_Controler.py:5-167``.  Same constructor ``MPCController(net, args)``,
attributes (``Ad``, ``Bd``, ``Nkoopman``, ``H``, ``MPC_type``, ``u_prev``, ``u_eso``,
``state_full``) and single-env calls ``Psi_o(s)`` / ``get_control(p) -> (u0, a)``.  casadi/IPOPT
is replaced by the closed form of the same unconstrained QP (``control/koopman.condensed_gains``,
computed once on the host in float64) and every per-env evaluation runs in the HIP library
(``include/koopman_mpc.h``, float64 MFMA):

* :meth:`encode`       — Psi_o for a batch of states (``sim_koopman_encode``)
* :meth:`feedforward`  — Gr · lifted reference window for every frame (``sim_koopman_feedforward``)
* :meth:`step`         — one control step for n envs (``sim_koopman_mpc_step``)

A bilinear DBKN model (``net.H``, ``KoopmanBase.py:62-110``) linearises its input matrix at each
frame's lifted state (``linearize_B``, ``:46-63``), so the QP differs per env and frame:
:meth:`step_bilinear` lifts the state in the HIP library and solves the n QPs in float64 on the
device, one wave per env (``sim_koopman_bilinear_step``, ``koopman_mpc.hip`` ``k_bilinear``;
``control/koopman.bilinear_first_move`` is the same algebra in torch, kept as its CPU cross-check).

There is no CPU path: without the library or a GPU, construction raises.
"""
import ctypes as C

import numpy as np

from .. import abi
from .koopman import condensed_gains

Q_WEIGHT, R_WEIGHT = 50.0, 0.5  # state_full weights (MPC_Controler.py:39-40)


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class MPCController:
    def __init__(self, net, args, device=0, horizon=10, u_clip=0.5):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("MPCController needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.bilinear = isinstance(getattr(net, "H", None), torch.nn.Module)
        self.torch = torch
        self.in_dim, self.u_dim = args.x_dim, args.u_dim
        self.net = net
        self.args = args
        self.device = torch.device("cuda", device)
        self.Ad = net.lA.weight.detach().double().cpu().numpy()
        self.Bd = net.lB.weight.detach().double().cpu().numpy()
        self.Nkoopman = self.Ad.shape[0]
        self.H = horizon
        self.u_clip = u_clip
        self.u_eso = np.zeros(self.u_dim)
        self.u_prev = np.zeros(self.u_dim)
        self.MPC_type = getattr(args, "MPC_type", "delta_mpc")
        # MPC_Controler.py:35-40: `args.model == 'IBKN' or 'IKN'` is always true, so the
        # reference always tracks the full lifted state with Q = 50 I, R = 0.5 I
        self.state_full = True
        self.Q = Q_WEIGHT * np.eye(self.Nkoopman)
        self.R = R_WEIGHT * np.eye(self.u_dim)
        self.Gr, self.Gz, self.Gu = condensed_gains(self.Ad, self.Bd, self.H, self.MPC_type, Q_WEIGHT, R_WEIGHT)
        if self.bilinear:  # (the gains above are the z0 = 0 linearisation; step_bilinear does not use them)
            self.H_hat_list = net.get_Hi_numpy()

        layers = net.encoder_layers()
        widths = [layers[0][0].shape[1]] + [W.shape[0] for W, _ in layers]
        if widths[0] != self.in_dim or self.in_dim + widths[-1] != self.Nkoopman:
            raise ValueError(f"encoder widths {widths} do not match x_dim {self.in_dim} / Nkoopman {self.Nkoopman}")
        d = abi.KoopmanDesc()
        d.x_dim, d.u_dim, d.nlayer, d.horizon, d.u_clip = self.in_dim, self.u_dim, len(layers), self.H, u_clip
        for i, w in enumerate(widths):
            d.width[i] = w
        self._w = np.ascontiguousarray(np.concatenate([np.concatenate([W.ravel(), b]) for W, b in layers]))
        self._g = np.ascontiguousarray(np.hstack([self.Gr, self.Gz, self.Gu]))
        self.lib = abi.load_lib()
        self._h = C.c_void_p()
        abi.check(self.lib, self.lib.sim_koopman_create(C.byref(d), self._w.ctypes.data_as(C.c_void_p),
                                                        self._g.ctypes.data_as(C.c_void_p), device,
                                                        C.byref(self._h)))
        if self.bilinear:  # the per-env QP kernel (koopman_mpc.hip k_bilinear)
            self._Ah = np.ascontiguousarray(self.Ad, np.float64)
            self._Bh = np.ascontiguousarray(self.Bd, np.float64)
            self._Hh = np.ascontiguousarray(np.stack(self.H_hat_list), np.float64)  # [j][nz][nu]
            abi.check(self.lib, self.lib.sim_koopman_set_bilinear(
                self._h, self._Ah.ctypes.data_as(C.c_void_p), self._Bh.ctypes.data_as(C.c_void_p),
                self._Hh.ctypes.data_as(C.c_void_p), int(self.MPC_type == "delta_mpc"), Q_WEIGHT, R_WEIGHT))

    def __del__(self):
        try:
            if self._h:
                self.lib.sim_koopman_free(self._h)
                self._h = None
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _f32(self, x, cols):
        t = self.torch.as_tensor(x, dtype=self.torch.float32, device=self.device)
        return t.reshape(-1, cols).contiguous()

    # ------------------------------------------------------------- batched device API
    def encode(self, x):
        """Psi_o of m states x [m, x_dim] -> z [Nkoopman, m] float64 (device)."""
        x = self._f32(x, self.in_dim)
        z = self.torch.empty((self.Nkoopman, x.shape[0]), dtype=self.torch.float64, device=self.device)
        abi.check(self.lib, self.lib.sim_koopman_encode(self._h, x.shape[0], _ptr(x), _ptr(z), self._stream()))
        return z

    def lift_reference(self, state_ref):
        """state_ref [T, n, x_dim] -> lifted zref [T, Nkoopman, n] float64 (device)."""
        T, n = state_ref.shape[0], state_ref.shape[1]
        z = self.encode(self.torch.as_tensor(state_ref).reshape(T * n, self.in_dim))
        return z.view(self.Nkoopman, T, n).permute(1, 0, 2).contiguous()

    def feedforward(self, zref, nframe=None):
        """ff [nframe, u_dim, n] = Gr · (zref rows f+1 .. f+H, zero past the end)."""
        nref, nz, n = zref.shape
        nframe = nref if nframe is None else nframe
        zref = zref.contiguous()
        ff = self.torch.empty((nframe, self.u_dim, n), dtype=self.torch.float64, device=self.device)
        abi.check(self.lib, self.lib.sim_koopman_feedforward(self._h, nframe, nref, n, _ptr(zref), _ptr(ff),
                                                             self._stream()))
        return ff

    def step(self, x, ff, u_prev, action=None, z0=None):
        """One control step for n envs (in place): u0 = ff + Gz Psi_o(x) + Gu u_prev;
        u_prev <- u0; returns action = clip(u0) [n, u_dim] float32 (device)."""
        n = u_prev.shape[1]
        xx = None if x is None else self._f32(x, self.in_dim)
        if action is None:
            action = self.torch.empty((n, self.u_dim), dtype=self.torch.float32, device=self.device)
        abi.check(self.lib, self.lib.sim_koopman_mpc_step(self._h, n, _ptr(xx), _ptr(z0), _ptr(ff), _ptr(u_prev),
                                                          _ptr(action), self._stream()))
        return action

    def step_bilinear(self, x, window, u_prev, action=None, z0=None):
        """DBKN control step for n envs (in place): z0 = Psi_o(x) (or given [nz, n]), the QP of
        each env with B_total = Bd + Σ_j z0_j Ĥ_j solved exactly; u_prev <- u0; returns
        action = clip(u0) [n, u_dim] float32.  window [H, nz, n]: lifted reference rows."""
        torch = self.torch
        if self.MPC_type not in ("mpc", "delta_mpc"):
            raise ValueError(f"MPC_type {self.MPC_type!r}: 'mpc' or 'delta_mpc'")
        if z0 is None:
            z0 = self.encode(x)
        n = u_prev.shape[1]
        if action is None:
            action = torch.empty((n, self.u_dim), dtype=torch.float32, device=self.device)
        z0 = z0.contiguous()
        window = window.contiguous()
        # k_bilinear reads raw pointers: float64 z0 [nz, n], a window of exactly H rows [H, nz, n]
        # (short tails are zero-padded by the caller, lifted_window), float64 u_prev [u_dim, n] and a
        # float32 action [n, u_dim], all contiguous on this device -- anything else is refused here
        dev = torch.device(self.device) if not isinstance(self.device, torch.device) else self.device
        want = {"z0": (z0, torch.float64, (self.Nkoopman, n)), "window": (window, torch.float64, (self.H, self.Nkoopman, n)),
                "u_prev": (u_prev, torch.float64, (self.u_dim, n)), "action": (action, torch.float32, (n, self.u_dim))}
        for name, (t, dt, shape) in want.items():
            if t.dtype != dt or tuple(t.shape) != shape or not t.is_contiguous() or t.device.type != "cuda" or \
                    (dev.index is not None and t.device.index != dev.index):
                raise ValueError(f"step_bilinear: {name} must be a contiguous {dt} tensor of shape {shape} on {dev}; "
                                 f"got {t.dtype} {tuple(t.shape)} on {t.device} (contiguous: {t.is_contiguous()})")
        abi.check(self.lib, self.lib.sim_koopman_bilinear_step(self._h, n, _ptr(z0), _ptr(window), _ptr(u_prev),
                                                               _ptr(action), self._stream()))
        return action

    # ------------------------------------------------------- reference single-env API
    def Psi_o(self, s):
        """Lifted state of s ([1, x_dim] tensor or array) as a (Nkoopman, 1) numpy column (:154-167)."""
        x = s.detach().cpu().numpy() if hasattr(s, "detach") else np.asarray(s)
        z = self.encode(x.reshape(-1, self.in_dim)).cpu().numpy()
        psi = z[:, :1].copy()
        self.z0 = psi
        return psi

    def get_control(self, p):
        """(u0, a) for p = [lifted ref (H*Nkoopman, row-major); z0 (Nkoopman); u_prev (u_dim, delta_mpc)]
        (:143-152); updates u_prev like the reference (delta_mpc: u_prev = a)."""
        torch = self.torch
        p = np.asarray(p, np.float64).reshape(-1)
        nz, H = self.Nkoopman, self.H
        ref = p[:H * nz].reshape(H, nz)
        z0 = p[H * nz:H * nz + nz]
        u_prev = p[H * nz + nz:H * nz + nz + self.u_dim] if self.MPC_type == "delta_mpc" else self.u_prev
        dev = dict(dtype=torch.float64, device=self.device)
        up = torch.as_tensor(np.asarray(u_prev, np.float64).reshape(self.u_dim, 1), **dev).contiguous()
        zc = torch.as_tensor(z0.reshape(nz, 1), **dev).contiguous()
        if self.bilinear:
            self.step_bilinear(None, torch.as_tensor(ref, **dev).reshape(H, nz, 1), up, z0=zc)
        else:
            zref = torch.zeros((H + 1, nz, 1), **dev)  # frame 0 unused: the window starts at f + 1
            zref[1:, :, 0] = torch.as_tensor(ref, **dev)
            ff = self.feedforward(zref, nframe=1)[0]
            self.step(None, ff, up, z0=zc)
        u0 = up[:, 0].cpu().numpy() + self.u_eso
        a = np.clip(u0, -self.u_clip, self.u_clip)  # float64, as :149 (the device action is its f32 copy)
        if self.MPC_type == "delta_mpc":
            self.u_prev = a.copy()
        return u0, a
