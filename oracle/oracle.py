"""ctypes wrapper of the float64 CPU oracle (``oracle/liboracle.so``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s cpu_baseline leg as the checker.  The product path never
imports this module.  Parity against MuJoCo itself is *unpinned* (MuJoCo is
absent and running the reference is denied); the oracle is
pinned by analytic known-answer tests and the survey's FK anchors.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_fp = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")


def build(force=False):
    """make is a no-op when liboracle.so is newer than its sources."""
    subprocess.check_call(["make", "-s", "-C", HERE] + (["-B"] if force else []))
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        vp = C.c_void_p
        L.orc_batch_reset.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
        L.orc_batch_reset.restype = None
        L.orc_batch_step.argtypes = [vp, vp, vp, vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, vp, vp,
                                     vp, vp, C.c_int, vp, vp]
        L.orc_batch_bias.argtypes = [vp, C.c_int, vp, vp, vp, vp]
        L.orc_batch_bias.restype = None
        L.orc_batch_step.restype = None
        L.orc_debug_forward.argtypes = [vp] * 4 + [vp] * 4 + [vp] * 8
        L.orc_debug_forward.restype = C.c_int
        L.orc_collide_geoms.argtypes = [vp] * 5 + [C.c_int, C.c_int, vp, C.c_int]
        L.orc_collide_geoms.restype = C.c_int
        L.orc_geom_frames.argtypes = [vp] * 4
        L.orc_geom_frames.restype = None
        L.orc_ik_dls.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp] + [C.c_double] * 6 + [C.c_int] * 3
        L.orc_ik_dls.restype = None
        L.orc_hull_support_flat.argtypes = [vp] * 4 + [C.c_int, vp, C.c_int, C.c_int, vp]
        L.orc_hull_support_flat.restype = C.c_int
        L.orc_newton_stats.argtypes = [vp, C.c_int]
        L.orc_newton_stats.restype = None
        L.orc_solver_stats.argtypes = [vp, C.c_int]
        L.orc_solver_stats.restype = None
        _lib = L
    return _lib


def solver_stats(reset=True):
    """(PGS calls, sweeps, rows), (Newton calls, iterations, line searches) since the last reset
    (single-threaded oracle calls only: the counters are not atomic)."""
    a, b = np.zeros(3), np.zeros(3)
    lib().orc_solver_stats(_p(a), int(reset))
    lib().orc_newton_stats(_p(b), int(reset))
    return a, b


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Oracle:
    """Batched float64 oracle over a compiled model (row-major [n][...] state)."""

    def __init__(self, cm, solver=None, tolerance=None):
        """solver: None (the compiled model's, PGS) or "PGS" / "Newton" (MuJoCo's default, the
        solver the reference's scene runs); tolerance: override (Newton with tolerance 0
        iterates to the exact optimum of the constraint problem)."""
        self.cm = cm
        self.desc = cm.desc
        if solver is not None or tolerance is not None:
            from lerobot_mujoco_sim2real_amd import abi
            self.desc = type(cm.desc).from_buffer_copy(cm.desc)
            if solver is not None:
                self.desc.solver = {"pgs": abi.SOL_PGS, "newton": abi.SOL_NEWTON}[solver.lower()]
            if tolerance is not None:
                self.desc.tolerance = tolerance
        self._desc_p = C.cast(C.pointer(self.desc), C.c_void_p)
        self.hv = np.ascontiguousarray(cm.hull_vert, np.float32)
        self.hadr = np.ascontiguousarray(cm.hull_adr, np.int32)
        self.hadj = np.ascontiguousarray(cm.hull_adj, np.int32)
        lib()

    def new_state(self, n):
        d = self.desc
        return dict(qpos=np.zeros((n, d.nq)), qvel=np.zeros((n, d.nv)), warm=np.zeros((n, d.nv)),
                    ctrl=np.zeros((n, d.nu)), status=np.zeros(n, np.int32), ncon=np.zeros(n))

    def reset(self, st, init_qpos=None, init_qvel=None, extra_qpos=None):
        n = st["qpos"].shape[0]
        d = self.desc
        obs = np.zeros((n, 3 + d.obs_nq))
        iq = None if init_qpos is None else np.ascontiguousarray(init_qpos, np.float64)
        iv = None if init_qvel is None else np.ascontiguousarray(init_qvel, np.float64)
        ex = None if extra_qpos is None else np.ascontiguousarray(extra_qpos, np.float64)
        lib().orc_batch_reset(self._desc_p, n, _p(st["qpos"]), _p(st["qvel"]), _p(st["warm"]),
                              _p(st["ctrl"]), _p(iq), _p(iv), _p(ex), _p(obs))
        st["status"][:] = 0
        st["ncon"][:] = 0
        return obs

    def step(self, st, action=None, nsub=10, params=None, nthreads=1, applied=None):
        """applied: [n, nv] qfrc_applied (float64, modified in place: a soft reset zeroes its row)."""
        n = st["qpos"].shape[0]
        d = self.desc
        obs = np.zeros((n, 3 + d.obs_nq))
        a = None if action is None else np.ascontiguousarray(action, np.float64)
        pr = None if params is None else np.ascontiguousarray(params, np.float64)
        fl = np.zeros(2)
        lib().orc_batch_step(self._desc_p, _p(self.hv), _p(self.hadr), _p(self.hadj), n,
                             _p(st["qpos"]), _p(st["qvel"]), _p(st["warm"]), _p(st["ctrl"]), _p(a),
                             nsub, _p(obs), _p(st["status"]), _p(st["ncon"]), _p(pr), nthreads,
                             _p(fl), _p(applied))
        self.last_flops = float(fl[0])
        self.last_collision_flops = float(fl[1])
        return obs

    def bias(self, st, params=None):
        """qfrc_bias [n, nv] at the states of `st` (gravity + Coriolis, as mj_forward leaves it)."""
        n = st["qpos"].shape[0]
        out = np.zeros((n, self.desc.nv))
        pr = None if params is None else np.ascontiguousarray(params, np.float64)
        lib().orc_batch_bias(self._desc_p, n, _p(np.ascontiguousarray(st["qpos"])),
                             _p(np.ascontiguousarray(st["qvel"])), _p(pr), _p(out))
        return out

    def forward(self, qpos, qvel=None, ctrl=None, warm=None):
        d = self.desc
        nv = d.nv
        M = np.zeros(nv * nv)
        bias, qacc = np.zeros(nv), np.zeros(nv)
        con = np.zeros(9 * 16)
        site = np.zeros(3 * max(d.nsite, 1))
        gx = np.zeros(3 * max(d.ngeom, 1))
        efc = np.zeros(2 * 16 + 4 * 16)
        nefc = C.c_int(0)
        f = lambda a: None if a is None else np.ascontiguousarray(a, np.float64)
        q, v, c, w = f(qpos), f(qvel), f(ctrl), f(warm)
        ncon = lib().orc_debug_forward(self._desc_p, _p(self.hv), _p(self.hadr), _p(self.hadj),
                                       _p(q), _p(v), _p(c), _p(w), _p(M), _p(bias), _p(qacc),
                                       _p(con), _p(site), _p(gx), _p(efc), C.byref(nefc))
        return dict(M=M.reshape(nv, nv), bias=bias, qacc=qacc, ncon=ncon,
                    contacts=con.reshape(16, 9)[:ncon], site_xpos=site.reshape(-1, 3)[: d.nsite],
                    geom_xpos=gx.reshape(-1, 3)[: d.ngeom], efc_force=efc[: nefc.value])

    def ik(self, target, q, tol=1e-6, regularization_threshold=0.1, regularization_strength=1e-2,
           max_update_norm=2.0, progress_thresh=20.0, max_steps=100, ndof=5, target_quat=None,
           rot_weight=0.5):
        """dm_control qpos_from_site_pose restated; target [n,3], target_quat [n,4] (w,x,y,z) or
        None (position only), q [n,nq] (copied)."""
        t = np.ascontiguousarray(target, np.float64).reshape(-1, 3)
        tq = None if target_quat is None else np.ascontiguousarray(
            np.broadcast_to(np.asarray(target_quat, np.float64), (len(t), 4)))
        q = np.array(q, dtype=np.float64, order="C").reshape(len(t), -1)
        ok = np.zeros(len(t), np.int32)
        it = np.zeros(len(t), np.int32)
        lib().orc_ik_dls(self._desc_p, len(t), _p(t), _p(tq), _p(q), _p(ok), _p(it), tol, rot_weight,
                         regularization_threshold, regularization_strength, max_update_norm,
                         progress_thresh, max_steps, int(self.desc.obs_site), ndof)
        return q, ok.astype(bool), it

    def hull_support(self, g, dirs, use_graph=True):
        d = np.ascontiguousarray(dirs, np.float64).reshape(-1, 3)
        out = np.zeros(len(d), np.int32)
        lib().orc_hull_support_flat(self._desc_p, _p(self.hv), _p(self.hadr), _p(self.hadj), g,
                                    _p(d), len(d), int(use_graph), _p(out))
        return out

    def geom_frames(self, qpos):
        """World (xpos [ngeom, 3], xmat [ngeom, 3, 3]) of every geom at qpos."""
        ng = self.desc.ngeom
        xp, xm = np.zeros(3 * ng), np.zeros(9 * ng)
        lib().orc_geom_frames(self._desc_p, _p(np.ascontiguousarray(qpos, np.float64)), _p(xp), _p(xm))
        return xp.reshape(ng, 3), xm.reshape(ng, 3, 3)

    def collide(self, qpos, g1, g2, maxout=8):
        out = np.zeros(7 * 8)
        q = np.ascontiguousarray(qpos, np.float64)
        n = lib().orc_collide_geoms(self._desc_p, _p(self.hv), _p(self.hadr), _p(self.hadj),
                                    _p(q), g1, g2, _p(out), maxout)
        return out.reshape(8, 7)[:n]
