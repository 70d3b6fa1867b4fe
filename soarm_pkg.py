"""Import helper: registers ``lerobot-mujoco-sim2real_amd/`` as the Python
package ``lerobot_mujoco_sim2real_amd`` (a hyphenated directory is not
importable by name)."""
import importlib.util
import os
import sys

NAME = "lerobot_mujoco_sim2real_amd"
ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "lerobot-mujoco-sim2real_amd")


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod


pkg = load()
