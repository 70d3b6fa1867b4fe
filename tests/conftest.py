import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import soarm_pkg  # noqa: E402,F401  (registers lerobot_mujoco_sim2real_amd)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")


@pytest.fixture(scope="session")
def arm_model():
    from lerobot_mujoco_sim2real_amd import mjcf
    return mjcf.compile_mjcf(mjcf.SCENE_XML)


@pytest.fixture(scope="session")
def arm_model_nocontact():
    from lerobot_mujoco_sim2real_amd import mjcf
    return mjcf.compile_mjcf(mjcf.SCENE_XML, disable_contact=True)


@pytest.fixture(scope="session")
def cube_model():
    from lerobot_mujoco_sim2real_amd import mjcf
    return mjcf.compile_mjcf(mjcf.CUBE_SCENE_XML)


@pytest.fixture(scope="session")
def gpu_lib():
    """Build (if stale) and load the HIP library; only for gpu-marked tests."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from lerobot_mujoco_sim2real_amd import abi, build
    build.build()
    return abi.load_lib()


def cube_qpos(cm, n, rng, arm_q=None):
    """Build-defined pick-scene pose: cube on the table near the EE workspace
    at (0.25 +- 0.05, +-0.05, -0.0009 + 0.015)."""
    q = np.tile(cm.qpos0(), (n, 1))
    if arm_q is not None:
        q[:, :arm_q.shape[1]] = arm_q
    q[:, 6] = 0.25 + rng.uniform(-0.05, 0.05, n)
    q[:, 7] = rng.uniform(-0.05, 0.05, n)
    q[:, 8] = -0.0009 + 0.015
    return q
