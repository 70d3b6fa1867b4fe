"""MI355X-native batched SO-ARM101 simulator (drop-in for the reference's
SOARM101Env / SOARM101_DataCollection hot path).

The package directory name contains hyphens, so it is imported under the
alias ``lerobot_mujoco_sim2real_amd`` (see ``soarm_pkg.py`` at the repo root).
"""
__version__ = "0.1.0"
