"""C-ABI boundary: the HIP library loads and exports exactly what include/soarm_sim.h declares.

No compute calls here (no GPU in the CPU suite)."""
import ctypes as C
import os
import re

import pytest

from lerobot_mujoco_sim2real_amd import abi, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = "".join(open(os.path.join(ROOT, "include", h)).read() for h in ("soarm_sim.h", "koopman_mpc.h"))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(sim_\w+)\s*\(", src, flags=re.M)))


def test_header_matches_python_exports():
    assert header_functions() == sorted(abi.EXPORTS)


def test_library_loads_and_exports_everything():
    build.build()
    lib = abi.load_lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.sim_version().decode().startswith("soarm_sim")


def test_no_device_fails_loudly():
    """Without a GPU, batch creation returns an error code (never a CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        return
    import soarm_pkg  # noqa: F401
    from lerobot_mujoco_sim2real_amd import mjcf
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML)
    lib = abi.load_lib()
    import numpy as np
    hv = np.ascontiguousarray(cm.hull_vert)
    ha = np.ascontiguousarray(cm.hull_adr)
    hj = np.ascontiguousarray(cm.hull_adj)
    model = C.c_void_p()
    assert lib.sim_model_create(C.byref(cm.desc), hv.ctypes.data_as(C.c_void_p), ha.ctypes.data_as(C.c_void_p),
                                hj.ctypes.data_as(C.c_void_p), C.byref(model)) == 0
    batch = C.c_void_p()
    rc = lib.sim_batch_create(model, 4, 0, C.byref(batch))
    assert rc == -4 and b"no HIP device" in lib.sim_last_error()
    lib.sim_model_free(model)


def test_model_file_round_trip_and_rejects(tmp_path):
    """sim_model_save / sim_model_load (the C caller's MjModel.from_xml_path): a saved model
    loads (sim_model_create runs on the host: no GPU needed); wrong magic, version, layout or a
    truncated / padded file are rejected with SIM_E_ARG."""
    import numpy as np
    import soarm_pkg  # noqa: F401
    from lerobot_mujoco_sim2real_amd import mjcf
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML)
    lib = abi.load_lib()
    path = tmp_path / "scene.soarm"
    cm.save(str(path))
    raw = path.read_bytes()
    d = cm.desc
    assert len(raw) == 16 + C.sizeof(d) + 12 * d.nhullvert + 4 * (d.nhullvert + 1) + 4 * d.nhulladj
    assert raw[:8] == b"SOARMMDL" and raw[16:16 + C.sizeof(d)] == bytes(d)
    off = 16 + C.sizeof(d)
    np.testing.assert_array_equal(np.frombuffer(raw, np.float32, 3 * d.nhullvert, off).reshape(-1, 3),
                                  cm.hull_vert)
    model = C.c_void_p()
    assert lib.sim_model_load(str(path).encode(), C.byref(model)) == 0 and model
    lib.sim_model_free(model)

    def rejected(data, what):
        bad = tmp_path / "bad.soarm"
        bad.write_bytes(data)
        m = C.c_void_p()
        assert lib.sim_model_load(str(bad).encode(), C.byref(m)) == -1 and not m, what
        return lib.sim_last_error()

    assert b"not a compiled" in rejected(b"XOARMMDL" + raw[8:], "magic")
    assert b"version" in rejected(raw[:8] + (1).to_bytes(4, "little") + raw[12:], "version")
    assert b"version" in rejected(raw[:12] + (C.sizeof(d) + 4).to_bytes(4, "little") + raw[16:], "layout")
    assert b"truncated" in rejected(raw[:-4], "truncated")
    assert b"truncated" in rejected(raw + b"\0", "trailing bytes")
    assert lib.sim_model_load(str(tmp_path / "missing.soarm").encode(), C.byref(model)) == -1


def test_struct_header_is_checked():
    """Every by-pointer struct leads with (struct_size, abi_version) (SIM_ABI_VERSION): a caller
    built against another layout gets SIM_E_ARG from sim_model_create / sim_model_save /
    sim_ik_dls instead of a field-by-field misread."""
    import soarm_pkg  # noqa: F401
    from lerobot_mujoco_sim2real_amd import mjcf
    hdr = open(os.path.join(ROOT, "include", "soarm_sim.h")).read()
    assert f"#define SIM_ABI_VERSION {abi.ABI_VERSION}" in hdr
    lib = abi.load_lib()
    assert f"abi {abi.ABI_VERSION}" in lib.sim_version().decode()
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML)
    assert cm.desc.struct_size == C.sizeof(abi.ModelDesc) and cm.desc.abi_version == abi.ABI_VERSION
    for field, val in (("struct_size", C.sizeof(abi.ModelDesc) - 8), ("abi_version", abi.ABI_VERSION - 1)):
        d = abi.ModelDesc.from_buffer_copy(cm.desc)
        setattr(d, field, val)
        model = C.c_void_p()
        assert lib.sim_model_create(C.byref(d), None, None, None, C.byref(model)) == -1 and not model
        assert b"struct_size / abi_version" in lib.sim_last_error()
        assert lib.sim_model_save(C.byref(d), None, None, None, b"/nonexistent/x") == -1
    o = abi.IkOpts(1e-6, 0.1, 1e-2, 2.0, 20.0, 100, 0, 5, 0, 0.5)
    assert o.struct_size == C.sizeof(abi.IkOpts) and o.tol == 1e-6 and o.rot_weight == 0.5
    o.struct_size -= 8  # the r03 layout (no rot_weight)
    assert lib.sim_ik_dls(None, None, None, None, None, C.byref(o), None) == -1
    assert b"sim_ik_opts" in lib.sim_last_error()


def test_model_validation_rejects_unsupported():
    import soarm_pkg  # noqa: F401
    from lerobot_mujoco_sim2real_amd import mjcf
    cm = mjcf.compile_mjcf(mjcf.SCENE_XML)
    cm.desc.geom_condim[0] = 6
    lib = abi.load_lib()
    model = C.c_void_p()
    rc = lib.sim_model_create(C.byref(cm.desc), None, None, None, C.byref(model))
    assert rc == -2 and b"condim" in lib.sim_last_error()


def test_philox_mirror_known_answer():
    """Philox4x32-10 known-answer vector (Random123 kat_vectors: ctr=0, key=0)."""
    import numpy as np
    from lerobot_mujoco_sim2real_amd.sim import philox4x32
    out = philox4x32(np.zeros((1, 4), np.uint32), (0, 0))[0]
    assert [hex(x) for x in out] == ["0x6627e8d5", "0xe169c58d", "0xbc57ac4c", "0x9b00dbd8"]


def test_env_errors_match_reference():
    """SOARM101_Env.py:35-36 (missing XML) and :51-52 (missing EE site) raise before any GPU use."""
    from lerobot_mujoco_sim2real_amd.SOARM101.SOARM101_Env import SOARM101Env
    from lerobot_mujoco_sim2real_amd.mjcf import compile_mjcf, SCENE_XML
    with pytest.raises(FileNotFoundError):
        SOARM101Env(xml_path="/nonexistent/scene.xml")
    cm = compile_mjcf(SCENE_XML)
    cm.site_names = [n + "_x" for n in cm.site_names]
    with pytest.raises(ValueError):
        SOARM101Env(model=cm)
