"""CartesianTrajectoryGenerator over the batched DLS-IK kernel.

Reference: ``control/TrajectoryGenerator.py:10-210``.  Same constructor and
``generate(traj_name, target_orientation) -> (xyz [N,3], q [N,num_joints], t [N])``.
The reference solves the N points serially with dm_control's
``qpos_from_site_pose`` (``:96-107``: pose IK with ``rot_weight=0.5`` toward the default
``target_orientation=[1, 0, 0, 0]`` (``:118``); ``None`` — what the ``Koopman_MPC.py:252``
call site passes — is position-only), warm-starting each point from the previous solution
and repeating the last good solution on failure (``:180-205``).  Here the warm-started chain
runs point by point through ``sim_ik_dls`` (one lane), and
:meth:`solve_batch` solves many independent targets at once (one lane each).
"""
import numpy as np

from ..mjcf import SCENE_XML, compile_mjcf
from ..SOARM101.SOARM101_DataCollection import cartesian_targets
from ..sim import BatchSim

IK_DEFAULTS = dict(tol=1e-6, regularization_threshold=0.1, regularization_strength=1e-2,
                   max_update_norm=2.0, progress_thresh=20.0, max_steps=100, rot_weight=0.5)


class CartesianTrajectoryGenerator:
    def __init__(self, model_path: str = SCENE_XML, ee_site_name: str = "gripperframe", num_joints: int = 5,
                 idx=1, time_horizon=60, time_steps_per_sec=5, device=0, model=None):
        self.idx = idx
        self.time_horizon = time_horizon
        self.time_steps = time_steps_per_sec * time_horizon
        self.time_vector = np.linspace(0, self.time_horizon, self.time_steps)
        self.num_joints = num_joints
        self.traj_scale = 0.5
        self.model = model if model is not None else compile_mjcf(model_path, obs_site=ee_site_name)
        self.device = device
        self._sims = {}

    def _sim(self, n):
        """One batch per size, reused across calls (the model's hull LUT and device copy are
        shared by all of them, sim.SimModel)."""
        if n not in self._sims:
            self._sims[n] = BatchSim(self.model, n, self.device)
        return self._sims[n]

    def cartesian_path(self, traj_name="Fig8"):
        t_param = 1.6 + 0.02 * np.linspace(0, self.time_horizon * 5, len(self.time_vector))
        return cartesian_targets(traj_name, t_param, self.idx, self.traj_scale)

    def solve_batch(self, targets, q0=None, target_quat=None, **opts):
        """Independent targets [N,3] (one lane each; target_quat [N,4] / [4] or None = position
        only); returns q [N, nq], ok [N], iters [N]."""
        import torch

        o = dict(IK_DEFAULTS, **opts)
        targets = np.asarray(targets, dtype=np.float32)
        sim = self._sim(len(targets))
        q = None
        if q0 is not None:
            q = torch.as_tensor(np.asarray(q0, np.float32).T.copy(), device=sim.device)
        q, ok, it = sim.ik(targets, q=q, ndof=self.num_joints, target_quat=target_quat, **o)
        return q.T.cpu().numpy(), ok.cpu().numpy().astype(bool), it.cpu().numpy()

    def generate(self, traj_name="Fig8", target_orientation=np.array([1.0, 0.0, 0.0, 0.0])):
        """The reference's default pose target [1, 0, 0, 0] (w, x, y, z) is kept; None = position only."""
        import torch

        tq = None if target_orientation is None else np.asarray(target_orientation, np.float32).reshape(1, 4)

        xyz = self.cartesian_path(traj_name)
        sim = self._sim(1)
        q = torch.as_tensor(self.model.qpos0().astype(np.float32).reshape(-1, 1), device=sim.device).contiguous()
        traj = []
        for i, pos in enumerate(xyz):
            last = q.clone()
            qn, ok, _ = sim.ik(pos[None].astype(np.float32), q=q, ndof=self.num_joints, target_quat=tq,
                               **IK_DEFAULTS)
            if bool(ok[0]):
                traj.append(qn[: self.num_joints, 0].cpu().numpy().copy())
                q = qn
            else:
                if not traj:
                    raise RuntimeError("IK failed on the first trajectory point")
                traj.append(traj[-1])
                q = last
        return xyz, np.array(traj), self.time_vector
