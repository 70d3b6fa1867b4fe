"""The float64 oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 race
detection / sanitizers): oracle/selftest.c drives reset, PGS and Newton steps (both scenes), bias,
a diagnostic forward and position / pose IK from a compiled model file."""
import os
import subprocess

import numpy as np
import pytest

from lerobot_mujoco_sim2real_amd import mjcf, workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def write_model(cm, path):
    with open(path, "wb") as f:
        f.write(bytes(cm.desc))
        hv = np.ascontiguousarray(cm.hull_vert, np.float32)
        f.write(np.int32(len(hv)).tobytes())
        f.write(hv.tobytes())
        f.write(np.ascontiguousarray(cm.hull_adr, np.int32).tobytes())
        adj = np.ascontiguousarray(cm.hull_adj, np.int32)
        f.write(np.int32(len(adj)).tobytes())
        f.write(adj.tobytes())


@pytest.mark.parametrize("scene", ["arm", "cube"])
def test_oracle_asan_ubsan(tmp_path, scene):
    subprocess.check_call(["make", "-s", "-C", ORACLE, "selftest_asan"])
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML) if scene == "arm" else W.model("contact")
    p = str(tmp_path / "model.bin")
    write_model(cm, p)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(ORACLE, "selftest_asan"), p], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "selftest ok" in r.stdout and "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
