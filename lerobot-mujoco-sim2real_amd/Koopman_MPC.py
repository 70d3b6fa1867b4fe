"""Koopman-MPC trajectory tracking, batched: the reference's ``Test`` loop for n envs at once.

Reference: ``Koopman_MPC.py:29-230`` (one env, a viewer, casadi/IPOPT, ZMQ to the real arm).
Per frame k of a T-frame reference ``state_all_ref = [cartesian xyz, joint angles]``
(``:49``) the reference does (``runFunc`` :110-136, ``runMPC`` :197-222):

1. ``qfrc_applied = qfrc_bias``  (gravity compensation from the last ``mj_forward``, :119)
2. lift the reference window ``state_all_ref[k+1 .. k+H]`` (zero rows past the end, :199-205)
   and the current state (``state_all_ref[0]`` on the first frame, :91; the last observation
   afterwards, :221), solve the MPC, ``u_prev = u0`` (:219)
3. ``env.step(clip(u0, +-0.5))`` (:220), ``mj_forward`` (:126)

:class:`KoopmanMPCTracking` runs that loop for n envs on one GPU with no host round trip:
``sim_bias`` writes ``qfrc_applied`` in place, the reference is lifted and turned into per-frame
feedforward terms once (the reference recomputes the same lifted rows every frame), then each
frame is ``sim_bias`` + ``sim_koopman_mpc_step`` + ``sim_step``.  With a ``communicator``
(``utility.ZMQ.ZMQCommunicator``) each frame also publishes env ``stream_env_id``'s joint angles
as real-robot targets, as the reference does after its step (:186-190).  Past the last frame
``runFunc`` plays the reference's return to the model's ``home`` keyframe (:62-81, :148-183): one
frame builds the 20-point joint-space path from the last reference pose to home, the next 20 set
``qpos`` along it and step with ``home_ctrl``, and every later frame holds ``qpos = home`` and
steps (the last reference pose when the model has no ``home`` key).  The viewer drawing is out of
scope.
"""
from .sim import BatchSim
from .utility.ZMQ import stream_env


class KoopmanMPCTracking:
    """n envs tracking their own reference trajectories with one MPCController."""

    def __init__(self, controller, model, cartesian_points, joint_angle_traj, device=0, sim=None,
                 communicator=None, stream_env_id=0):
        import torch

        self.communicator = communicator
        self.stream_env_id = stream_env_id

        self.torch = torch
        self.ctl = controller
        dev = torch.device("cuda", device)
        cp = torch.as_tensor(cartesian_points, dtype=torch.float32, device=dev)
        jq = torch.as_tensor(joint_angle_traj, dtype=torch.float32, device=dev)
        if cp.ndim == 2:  # one trajectory for every env
            cp, jq = cp[:, None], jq[:, None]
        self.total_frames, self.n = jq.shape[0], jq.shape[1]
        self.num_joints = jq.shape[2]
        # state_all_ref = hstack([cartesian_points, joint_angle_traj]) (Koopman_MPC.py:49)
        self.state_all_ref = torch.cat([cp, jq], -1).contiguous()
        self.sim = sim if sim is not None else BatchSim(model, self.n, device)
        self.sim.enable_qfrc_applied()
        self.H = controller.H
        zref = controller.lift_reference(self.state_all_ref)
        if controller.bilinear:
            # DBKN: the QP depends on each frame's lifted state, so the lifted reference is kept
            # (zero rows past the end, :199-205) and each frame solves its n QPs
            self.zpad = torch.cat([zref, torch.zeros((self.H,) + zref.shape[1:], dtype=zref.dtype, device=dev)])
            self.ff = None
        else:
            self.ff = controller.feedforward(zref)  # [T, u, n]
        self.u_prev = torch.zeros((controller.u_dim, self.n), dtype=torch.float64, device=dev)
        self.action = torch.empty((self.n, controller.u_dim), dtype=torch.float32, device=dev)
        self.traj_index = 0
        # the "home" keyframe (Koopman_MPC.py:62-76) and the return playback state (:78-81)
        home = getattr(model, "keyframes", {}).get("home") if model is not None else None
        self.home_qpos = None if home is None or home["qpos"] is None else \
            torch.as_tensor(home["qpos"], dtype=torch.float32, device=dev)
        nu = controller.u_dim
        hc = home["ctrl"] if home is not None and home["ctrl"] is not None else [0.0] * nu
        self.home_ctrl = torch.as_tensor(hc[:nu], dtype=torch.float32, device=dev).expand(self.n, nu).contiguous()
        self.return_traj = None
        self.return_index = 0
        self.return_duration = 2.0

    def runBefore(self):
        """qpos[:num_joints] = joint_angle_traj[0] on a fresh MjData (qvel, ctrl, warm start 0),
        mj_forward; the first MPC state is state_all_ref[0] (Koopman_MPC.py:83-91)."""
        q0 = self.state_all_ref[0, :, 3:3 + self.num_joints]
        self.sim.reset(init_qpos=q0, init_qvel=self.torch.zeros_like(q0))
        self.state = self.state_all_ref[0]
        self.traj_index = 0
        self.u_prev.zero_()

    def runFunc(self):
        """One frame: gravity compensation, MPC, env.step (Koopman_MPC.py:110-136, 197-222)."""
        k = self.traj_index
        if k >= self.total_frames:
            return self._after_trajectory()
        self.sim.bias(out=self.sim.qfrc_applied)
        if self.ff is None:
            self.ctl.step_bilinear(self.state, self.zpad[k + 1:k + 1 + self.H], self.u_prev, self.action)
        else:
            self.ctl.step(self.state, self.ff[k], self.u_prev, self.action)
        self.state = self.sim.step(self.action)
        if self.communicator is not None:  # sim -> real (Koopman_MPC.py:186-190)
            stream_env(self.sim, self.communicator, self.stream_env_id)
        self.traj_index += 1
        return self.state

    def _after_trajectory(self):
        """Koopman_MPC.py:148-183 for every env: build the return path (one frame, no step), play
        it (qpos[:nj] = path point, mj_forward, step(home_ctrl)), then hold home; gravity
        compensation and the sim -> real stream every frame as in the tracking frames."""
        torch, nj = self.torch, self.num_joints
        self.sim.bias(out=self.sim.qfrc_applied)  # qfrc_applied = qfrc_bias (:119)
        if self.return_traj is None and self.home_qpos is not None:  # phase 2 (:150-165)
            start = self.state_all_ref[-1, :, 3:3 + nj].T                  # joint_angle_traj[-1] [nj, n]
            end = self.home_qpos[:nj, None].expand_as(start)
            steps = int(self.return_duration / 0.1)
            w = torch.linspace(0.0, 1.0, steps, device=start.device, dtype=torch.float64)[:, None, None]
            self.return_traj = ((1 - w) * start.double() + w * end.double()).float()  # np.linspace rows
            self.return_index = 0
        else:
            if self.return_traj is not None and self.return_index < len(self.return_traj):  # phase 3
                self.sim.qpos[:nj] = self.return_traj[self.return_index]
                self.return_index += 1
            else:  # phase 4: hold home (or the last reference pose)
                hold = self.home_qpos[:nj, None] if self.home_qpos is not None else \
                    self.state_all_ref[-1, :, 3:3 + nj].T
                self.sim.qpos[:nj] = hold
            self.state = self.sim.step(self.home_ctrl)  # (mj_forward is inside the step)
        if self.communicator is not None:
            stream_env(self.sim, self.communicator, self.stream_env_id)
        self.traj_index += 1
        return self.state

    def run(self, frames=None, record=True):
        """runBefore + `frames` (default: all) x runFunc; returns the observed states
        [frames, n, 8] (device) as the reference's actual_traj."""
        frames = self.total_frames if frames is None else min(frames, self.total_frames)
        self.runBefore()
        out = self.torch.empty((frames, self.n, self.state_all_ref.shape[2]), dtype=self.torch.float32,
                               device=self.state_all_ref.device) if record else None
        for k in range(frames):
            s = self.runFunc()
            if record:
                out[k] = s
        return out
