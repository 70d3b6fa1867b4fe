"""Host-side batch simulator over the C ABI (``include/soarm_sim.h``).

:class:`BatchSim` owns one ``sim_batch`` (sharing its model's cached ``sim_model``,
:class:`SimModel`) and the env state as
caller-owned torch tensors on the GPU (SoA ``[field][env]``).  It is the single
object the reference-shaped APIs (``SOARM101Env``, ``SOARM101VecEnv``,
``SOARM101DataGenerator``, ``CartesianTrajectoryGenerator``) drive.  Every call
is asynchronous on torch's current stream; nothing here falls back to a CPU
path — if the HIP library or the GPU is missing, construction raises.

``device=-1`` selects the library's CPU backend explicitly (``sim_batch_create(...,
-1, ...)``): the same per-env physics compiled for the host, with the
state as CPU torch tensors and synchronous calls.  It is never chosen implicitly.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .mjcf import SCENE_XML, compile_mjcf


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def philox4x32(ctr, key):
    """Philox4x32-10 on uint32 arrays ctr [n, 4], key (k0, k1) -> [n, 4] (mirror of the device RNG)."""
    c = np.array(ctr, dtype=np.uint64) & 0xFFFFFFFF
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    m = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[:, 0]
        p1 = np.uint64(0xCD9E8D57) * c[:, 2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & m
        hi1, lo1 = p1 >> np.uint64(32), p1 & m
        c = np.stack([hi1 ^ c[:, 1] ^ k0, lo1, hi0 ^ c[:, 3] ^ k1, lo0], 1)
        k0 = (k0 + np.uint64(0x9E3779B9)) & m
        k1 = (k1 + np.uint64(0xBB67AE85)) & m
    return c.astype(np.uint32)


def reset_qpos_draw(seed, env_ids, nobs=5):
    """The U(-0.3, 0.3) initial joint angles sim_reset draws on device for env ids (float32)."""
    ids = np.asarray(env_ids, dtype=np.uint64)
    k = (int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF)
    out = []
    for blk in range(2):
        ctr = np.stack([ids & 0xFFFFFFFF, ids >> np.uint64(32), np.full_like(ids, blk), np.zeros_like(ids)], 1)
        out.append(philox4x32(ctr, k))
    r = np.concatenate(out, 1)[:, :nobs]
    u = (r >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return np.float32(-0.3) + np.float32(0.6) * u


class SimModel:
    """One ``sim_model`` (MJCF constants + hull records + support LUT) per compiled model.

    Building the hull support LUT is the expensive part of model creation (exact
    argmax over every hull vertex for 6x96x96 directions per mesh), so it is done
    once per :class:`CompiledModel` and shared: every :class:`BatchSim` of the
    model holds this handle, and the library shares the model's device copy
    among the batches on one GPU.  The handle outlives its batches (they keep a
    reference), as ``sim_model_free`` requires."""

    def __init__(self, cm, lib):
        self.lib = lib
        d = cm.desc
        self.key = bytes(d)
        self._hv = np.ascontiguousarray(cm.hull_vert, np.float32)
        self._hadr = np.ascontiguousarray(cm.hull_adr, np.int32)
        self._hadj = np.ascontiguousarray(cm.hull_adj, np.int32)
        self.ptr = C.c_void_p()
        abi.check(lib, lib.sim_model_create(
            C.byref(d), self._hv.ctypes.data_as(C.c_void_p), self._hadr.ctypes.data_as(C.c_void_p),
            self._hadj.ctypes.data_as(C.c_void_p), C.byref(self.ptr)))

    @classmethod
    def from_file(cls, path, lib):
        """A handle loaded from a compiled model file (`sim_model_load`; CompiledModel.save)."""
        h = cls.__new__(cls)
        h.lib, h.key = lib, None
        h.ptr = C.c_void_p()
        abi.check(lib, lib.sim_model_load(os.fsencode(path), C.byref(h.ptr)))
        return h

    @classmethod
    def of(cls, cm, lib):
        """The cached handle of `cm` (rebuilt if its desc was edited since)."""
        h = getattr(cm, "_sim_model", None)
        if h is None or h.key != bytes(cm.desc):
            h = cls(cm, lib)
            cm._sim_model = h
        return h

    def __del__(self):
        try:
            if self.ptr:
                self.lib.sim_model_free(self.ptr)
                self.ptr = None
        except Exception:
            pass


class BatchSim:
    """`n_envs` SO-ARM101 environments stepped in lockstep on one GPU (device = HIP ordinal), or
    on the host threads (device = -1: the CPU backend)."""

    def __init__(self, model=None, n_envs=1, device=0, model_handle=None, **compile_kw):
        """model: a CompiledModel (sizes, names); model_handle: a SimModel to run instead of the
        model's own (e.g. SimModel.from_file of the same model's saved file)."""
        import torch

        self.cpu = device == -1
        if not self.cpu and not torch.cuda.is_available():
            raise RuntimeError("BatchSim needs a ROCm GPU (torch.cuda.is_available() is False); "
                               "device=-1 selects the CPU backend explicitly")
        self.torch = torch
        self.cm = model if model is not None else compile_mjcf(SCENE_XML, **compile_kw)
        self.lib = abi.load_lib()
        d = self.cm.desc
        self.n = int(n_envs)
        self.device = torch.device("cpu") if self.cpu else torch.device("cuda", device)
        self.nq, self.nv, self.nu = d.nq, d.nv, d.nu
        self.nact, self.obs_dim = d.nact, 3 + d.obs_nq
        self.frame_skip = max(1, int(round(0.02 / d.timestep)))
        self._handle = model_handle if model_handle is not None else SimModel.of(self.cm, self.lib)  # kept alive by this batch
        self._model = self._handle.ptr
        self._batch = C.c_void_p()
        abi.check(self.lib, self.lib.sim_batch_create(self._model, self.n, device, C.byref(self._batch)))
        f32 = dict(dtype=torch.float32, device=self.device)
        self.qpos = torch.zeros((self.nq, self.n), **f32)
        self.qvel = torch.zeros((self.nv, self.n), **f32)
        self.qacc_warmstart = torch.zeros((self.nv, self.n), **f32)
        self.ctrl = torch.zeros((self.nu, self.n), **f32)
        self.status = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self.ncon = torch.zeros(self.n, **f32)
        self.obs = torch.zeros((self.n, self.obs_dim), **f32)
        self.qfrc_applied = None  # [nv, n] once enable_qfrc_applied() is called
        self._bind_state()
        self._params = None
        self._act = None

    def _bind_state(self):
        self._state = abi.SimState(_ptr(self.qpos), _ptr(self.qvel), _ptr(self.qacc_warmstart),
                                   _ptr(self.ctrl), _ptr(self.status), _ptr(self.ncon),
                                   _ptr(self.qfrc_applied))

    def enable_qfrc_applied(self):
        """Allocate ``qfrc_applied`` [nv, n] (zeros; MjData.qfrc_applied): from now on every
        substep adds it to the smooth forces, and a reset / soft reset zeroes the env's row
        (``mj_resetData``).  ``Koopman_MPC.py:119`` writes it every frame."""
        if self.qfrc_applied is None:
            self.qfrc_applied = self.torch.zeros((self.nv, self.n), dtype=self.torch.float32, device=self.device)
            self._bind_state()
        return self.qfrc_applied

    # ------------------------------------------------------------------ utils
    def _stream(self):
        if self.cpu:
            return None  # (the CPU backend's calls are synchronous)
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _dev(self, x, shape=None):
        if x is None:
            return None
        t = self.torch.as_tensor(x, dtype=self.torch.float32, device=self.device)
        if shape is not None:
            t = t.reshape(shape)
        return t.contiguous()

    def close(self):
        if getattr(self, "_batch", None):
            self.lib.sim_batch_free(self._batch)
            self._batch = None
        self._handle = None  # the model is freed when its last batch lets go

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------- DR params
    def set_params(self, mass_scale=None, friction=None, damping_scale=None):
        """Per-env domain randomisation ([n] each, None = nominal)."""
        self._pm = [self._dev(x, (self.n,)) for x in (mass_scale, friction, damping_scale)]
        p = abi.SimParams(*[_ptr(x) for x in self._pm])
        self._params = p
        abi.check(self.lib, self.lib.sim_batch_set_params(self._batch, C.byref(p)))

    # --------------------------------------------------------------- API calls
    def reset(self, init_qpos=None, init_qvel=None, extra_qpos=None, seed=0, env_offset=0, mask=None):
        """mj_resetData + init + mj_forward for masked envs; returns obs [n, obs_dim].

        init_qpos / init_qvel: [n, obs_nq] (row per env) or None (U(-0.3,0.3) from
        Philox keyed by (seed, env_offset + i); qvel 0).  extra_qpos: [n, nq]."""
        d = self.cm.desc
        iq = None if init_qpos is None else self._dev(init_qpos, (self.n, d.obs_nq)).T.contiguous()
        iv = None if init_qvel is None else self._dev(init_qvel, (self.n, d.obs_nq)).T.contiguous()
        ex = None if extra_qpos is None else self._dev(extra_qpos, (self.n, self.nq)).T.contiguous()
        mk = None
        if mask is not None:
            mk = self.torch.as_tensor(mask, device=self.device).to(self.torch.uint8).contiguous()
        self._keep = (iq, iv, ex, mk)
        abi.check(self.lib, self.lib.sim_reset(self._batch, C.byref(self._state), _ptr(iq), _ptr(iv),
                                               _ptr(ex), C.c_uint64(seed), C.c_int64(env_offset),
                                               _ptr(mk), _ptr(self.obs), self._stream()))
        return self.obs

    def action_buffer(self):
        """The staging buffer [n, nact] float32 that :meth:`step` reads the action from: a caller
        that writes its actions here directly (``step(sim.action_buffer())``) skips the copy."""
        if self._act is None:
            self._act = self.torch.zeros((self.n, self.nact), dtype=self.torch.float32, device=self.device)
        return self._act

    def step(self, action, frame_skip=None):
        """ctrl[:nact] = action ([n, nact]); frame_skip x mj_step; returns obs [n, obs_dim].

        The action is staged into one persistent device buffer (:meth:`action_buffer`): the
        contact env-step replays a hipGraph keyed by the addresses of the buffers it reads
        (soarm_sim.hip sim_step), so a fresh tensor per call (a strided view, a numpy array,
        a new torch expression) would otherwise recapture the graph."""
        a = self.action_buffer()
        if action is not a:
            src = action if isinstance(action, self.torch.Tensor) else self.torch.as_tensor(
                np.asarray(action, dtype=np.float32))
            a.copy_(src.reshape(self.n, self.nact))
        abi.check(self.lib, self.lib.sim_step(self._batch, C.byref(self._state), _ptr(a),
                                              int(frame_skip or self.frame_skip), _ptr(self.obs),
                                              self._stream()))
        return self.obs

    def rand_uniform(self, seed, counter, k, lo, hi, env_offset=0, out=None):
        """[n, k] float32 U[lo, hi) keyed by (seed, env_offset + i, counter) (sim_rand_uniform;
        host mirror: workloads.keyed_uniform)."""
        if out is None:
            out = self.torch.empty((self.n, k), dtype=self.torch.float32, device=self.device)
        abi.check(self.lib, self.lib.sim_rand_uniform(self._batch, C.c_uint64(seed), C.c_int64(env_offset),
                                                      C.c_uint32(counter & 0xFFFFFFFF), int(k), C.c_float(lo),
                                                      C.c_float(hi), _ptr(out), self._stream()))
        return out

    def substeps(self, nsub):
        abi.check(self.lib, self.lib.sim_substeps(self._batch, C.byref(self._state), int(nsub),
                                                  self._stream()))

    def bias(self, out=None):
        """qfrc_bias [nv, n] at the current state (gravity + Coriolis/centrifugal with the
        current qvel), what ``mj_forward`` leaves in ``d.qfrc_bias`` (``Koopman_MPC.py:119,126``)."""
        if out is None:
            out = self.torch.empty((self.nv, self.n), dtype=self.torch.float32, device=self.device)
        abi.check(self.lib, self.lib.sim_bias(self._batch, C.byref(self._state), _ptr(out), self._stream()))
        return out

    def observe(self):
        abi.check(self.lib, self.lib.sim_observe(self._batch, C.byref(self._state), _ptr(self.obs),
                                                 self._stream()))
        return self.obs

    def profile_begin(self):
        abi.check(self.lib, self.lib.sim_profile_begin(self._batch))

    def profile_end(self):
        """{kind: (total_ms, launches)} for the launches since profile_begin (synchronises)."""
        ms = (C.c_double * 4)()
        cnt = (C.c_int32 * 4)()
        abi.check(self.lib, self.lib.sim_profile_end(self._batch, C.cast(ms, C.c_void_p), C.cast(cnt, C.c_void_p)))
        return {k: (ms[i], cnt[i]) for i, k in enumerate(abi.PROF_KINDS)}

    def contacts(self):
        """Contacts at the current positions: (list [n][MAXCON][8], ncon [n]).
        Fields: dist, pos(3), normal(3) geom1->geom2, pair id (int32 bits)."""
        out = self.torch.zeros((self.n, abi.MAXCON, 8), dtype=self.torch.float32, device=self.device)
        nc = self.torch.zeros(self.n, dtype=self.torch.int32, device=self.device)
        abi.check(self.lib, self.lib.sim_contacts(self._batch, C.byref(self._state), _ptr(out), _ptr(nc),
                                                  self._stream()))
        return out, nc

    def collide_profile(self, with_max=False):
        """Per candidate pair, summed wave cycles of one collide pass (numpy [npair]); with_max:
        also the largest single wave's cycles per pair (the pass's critical path)."""
        npair = self.cm.desc.npair
        cyc = np.zeros(2 * max(npair, 1), dtype=np.float64)
        abi.check(self.lib, self.lib.sim_collide_profile(self._batch, C.byref(self._state),
                                                         cyc.ctypes.data, self._stream()))
        return (cyc[:npair], cyc[npair:2 * npair]) if with_max else cyc[:npair]

    def ik(self, target, q=None, tol=1e-6, regularization_threshold=0.1, regularization_strength=1e-2,
           max_update_norm=2.0, progress_thresh=20.0, max_steps=100, ndof=5, target_quat=None,
           rot_weight=0.5):
        """Batched DLS IK of the observed site (dm_control qpos_from_site_pose).  target [n, 3];
        target_quat [n, 4] or [4] (w, x, y, z; pose IK) or None (position only);
        q [nq, n] warm start (SoA, modified in place) or None (qpos0)."""
        t = self._dev(target, (self.n, 3))
        tq = None
        if target_quat is not None:
            tq = self.torch.as_tensor(np.asarray(target_quat, np.float32) if not isinstance(
                target_quat, self.torch.Tensor) else target_quat, dtype=self.torch.float32, device=self.device)
            tq = tq.expand(self.n, 4).contiguous()
        if q is None:
            q = self.torch.zeros((self.nq, self.n), dtype=self.torch.float32, device=self.device)
            q[:] = self._dev(self.cm.qpos0()).reshape(-1, 1)
        ok = self.torch.zeros(self.n, dtype=self.torch.int32, device=self.device)
        it = self.torch.zeros(self.n, dtype=self.torch.int32, device=self.device)
        o = abi.IkOpts(tol, regularization_threshold, regularization_strength, max_update_norm,
                       progress_thresh, int(max_steps), int(self.cm.desc.obs_site), int(ndof), 0, rot_weight)
        self._keep_ik = (t, tq)
        abi.check(self.lib, self.lib.sim_ik_dls_pose(self._batch, _ptr(t), _ptr(tq), _ptr(q), _ptr(ok), _ptr(it),
                                                     C.byref(o), self._stream()))
        return q, ok, it
