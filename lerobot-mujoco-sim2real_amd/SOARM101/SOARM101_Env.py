"""SOARM101Env — drop-in for the reference Gym env, backed by the HIP batch simulator.

Reference: ``SOARM101/SOARM101_Env.py`` (class at :8).  Same constructor
arguments, attributes (``frame_skip``, ``dt``, ``joint_names``, ``joint_ids``,
``ee_site_id``, ``udim``, ``max_speed``, ``xdim``, ``action_space``,
``observation_space``) and return tuples:

* ``reset(seed, options) -> (obs[8] float32, {})``   (:77-106)
* ``step(action[5]) -> (obs[8] float32, 0.0, False, False, {})``   (:108-142)

``obs = [site_xpos[gripperframe] (3), qpos[joint_ids] (5)]`` (:69-75).  As in
MuJoCo, ``site_xpos`` after ``mj_step`` comes from the last substep's forward
pass (before that substep's position update) while ``qpos`` is the new one.

:class:`SOARM101VecEnv` is the batched form of the same API: actions ``[n, 5]``,
observations ``[n, 8]`` (torch tensors on the GPU, or numpy on request).
"""
import os
from typing import Dict, Optional, Tuple

import numpy as np

from ..mjcf import compile_mjcf
from ..sim import BatchSim


class Box:
    """Minimal stand-in for ``gymnasium.spaces.Box`` (gymnasium is not a dependency)."""

    def __init__(self, low, high, shape, dtype):
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)
        self.shape, self.dtype = shape, dtype

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return rng.uniform(self.low, self.high).astype(self.dtype)


class SOARM101VecEnv:
    """`num_envs` SO-ARM101 environments on one GPU (batched SOARM101Env)."""

    metadata = {"render_modes": []}
    joint_names = ["shoulder_pan", "shoulder_lift", "elbow_flex", "wrist_flex", "wrist_roll"]

    def __init__(self, xml_path: Optional[str] = None, num_envs: int = 1, dt: float = 0.02,
                 device: int = 0, model=None, seed: int = 0, env_offset: int = 0, **compile_kw):
        if model is None:
            from ..mjcf import SCENE_XML
            xml_path = xml_path or SCENE_XML
            if not os.path.exists(xml_path):  # SOARM101_Env.py:35-36
                raise FileNotFoundError(f"XML file not found: {xml_path}")
            model = compile_mjcf(xml_path, **compile_kw)
        self.model = model
        try:
            self.ee_site_id = model.site("gripperframe")
        except (KeyError, ValueError):  # SOARM101_Env.py:51-52
            raise ValueError("Site 'gripperframe' not found in model") from None
        self.joint_ids = [model.joint(n) for n in self.joint_names]
        self.sim = BatchSim(model, num_envs, device)
        self.num_envs = num_envs
        # SOARM101_Env.py:39-40
        self.frame_skip = max(1, int(np.round(dt / model.timestep)))
        self.dt = model.timestep * self.frame_skip
        self.udim = 5
        self.max_speed = 0.5
        self.xdim = 8
        self.action_space = Box(-self.max_speed, self.max_speed, (self.udim,), np.float32)
        self.observation_space = Box(-np.inf, np.inf, (self.xdim,), np.float32)
        self._seed = seed
        self._env_offset = env_offset
        self._resets = 0

    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None, mask=None):
        """Reset all (or `mask`ed) envs.  options['initial_state']: [n, 10] = qpos(5), qvel(5)."""
        if seed is not None:
            self._seed, self._resets = seed, 0
        iq = iv = None
        if options and "initial_state" in options:
            s = np.asarray(options["initial_state"], dtype=np.float32).reshape(self.num_envs, -1)
            iq, iv = s[:, :5], s[:, 5:10]
        # fresh Philox stream per reset call: key (seed, call index), counter = env id
        key = (self._seed & 0xFFFFFFFF) | ((self._resets & 0xFFFFFFFF) << 32)
        self._resets += 1
        obs = self.sim.reset(init_qpos=iq, init_qvel=iv, extra_qpos=options.get("qpos") if options else None,
                             seed=key, env_offset=self._env_offset, mask=mask)
        return obs, {}

    def step(self, action):
        obs = self.sim.step(action, self.frame_skip)
        return obs, 0.0, False, False, {}

    def close(self):
        self.sim.close()


class SOARM101Env(SOARM101VecEnv):
    """Single-env API of the reference (numpy in / numpy out)."""

    def __init__(self, xml_path: Optional[str] = None, dt: float = 0.02, render_mode=False, **kw):
        if render_mode:
            raise NotImplementedError("viewer rendering is out of scope (SURVEY.md §2)")
        super().__init__(xml_path, 1, dt, **kw)
        self.render_mode = render_mode
        self.np_random = np.random.default_rng()
        print(f"环境控制步长(dt): {self.dt:.4f}s (执行 {self.frame_skip} 个物理步骤)")

    def reset(self, seed: Optional[int] = None, options: Optional[Dict] = None) -> Tuple[np.ndarray, Dict]:
        if seed is not None:
            self.np_random = np.random.default_rng(seed)
        if options and "initial_state" in options:
            init = np.asarray(options["initial_state"], dtype=np.float64)
            iq, iv = init[:5], init[5:10]
        else:
            iq = self.np_random.uniform(low=-0.3, high=0.3, size=self.udim)
            iv = np.zeros(self.udim)
        obs = self.sim.reset(init_qpos=iq[None], init_qvel=iv[None])
        return obs[0].cpu().numpy().astype(np.float32), {}

    def step(self, action: np.ndarray):
        a = np.asarray(action, dtype=np.float32)[: self.udim]
        obs = self.sim.step(a[None], self.frame_skip)
        return obs[0].cpu().numpy().astype(np.float32), 0.0, False, False, {}

    def render(self):
        return None

    @property
    def data_qpos(self):
        return self.sim.qpos[:, 0].cpu().numpy()

    @property
    def data_qvel(self):
        return self.sim.qvel[:, 0].cpu().numpy()
