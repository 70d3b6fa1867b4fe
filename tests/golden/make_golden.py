"""Generate the committed oracle fixtures (run: python tests/golden/make_golden.py).

There are no golden vectors in the reference: the
fixtures here are produced by this repository's float64 oracle and pin it
against regressions; the GPU parity tests compare the HIP path with them.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import mjcf  # noqa: E402
from oracle import Oracle  # noqa: E402


def main():
    rng = np.random.default_rng(20251212)
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML, disable_contact=True)
    orc = Oracle(cm)
    n, T = 8, 12
    iq = rng.uniform(-0.3, 0.3, (n, 5))
    acts = rng.uniform(-0.5, 0.5, (T, n, 5))
    st = orc.new_state(n)
    obs = [orc.reset(st, init_qpos=iq)]
    for a in acts:
        obs.append(orc.step(st, a))
    np.savez_compressed(os.path.join(HERE, "oracle_arm_random.npz"), init_qpos=iq, actions=acts,
                        obs=np.stack(obs))


if __name__ == "__main__":
    main()
