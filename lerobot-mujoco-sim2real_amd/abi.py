"""ctypes mirror of ``include/soarm_sim.h`` (the C-ABI boundary).

Only plain C types cross the boundary; this module defines the structures
and loads the in-tree ``libsoarm_sim.so``.  There is deliberately no fallback:
if the HIP library is missing, :func:`load_lib` raises.
"""
import ctypes as C
import os

MAXBODY, MAXJNT, MAXDOF, MAXQ = 12, 12, 16, 20
MAXGEOM, MAXPAIR, MAXSITE, MAXU, MAXOBSQ = 40, 160, 4, 8, 8
MAXCON = 16

JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = 0, 1, 2, 3
SOL_PGS, SOL_CG, SOL_NEWTON = 0, 1, 2
CCD_MPR, CCD_NATIVE = 0, 1
GEOM_PLANE, GEOM_SPHERE, GEOM_BOX, GEOM_MESH = 0, 2, 6, 7

ST_BADQPOS, ST_BADQVEL, ST_BADQACC, ST_CONOVERFLOW = 1, 2, 4, 8

i32, f64 = C.c_int32, C.c_double
ABI_VERSION = 2  # SIM_ABI_VERSION (include/soarm_sim.h)


class _Versioned(C.Structure):
    """A by-pointer ABI struct: leading (struct_size, abi_version), filled on construction."""

    def __init__(self, *args, **kw):
        super().__init__(0, 0, *args, **kw)
        self.struct_size = C.sizeof(type(self))
        self.abi_version = ABI_VERSION


def _a(t, *dims):
    for d in reversed(dims):
        t = t * d
    return t


class ModelDesc(_Versioned):
    _fields_ = [
        ("struct_size", i32), ("abi_version", i32),
        ("nbody", i32), ("njnt", i32), ("nq", i32), ("nv", i32), ("nu", i32),
        ("ngeom", i32), ("nsite", i32), ("npair", i32), ("nhullvert", i32), ("nhulladj", i32),
        ("timestep", f64), ("gravity", _a(f64, 3)), ("impratio", f64), ("tolerance", f64),
        ("meaninertia", f64),
        ("iterations", i32), ("disable_contact", i32), ("disable_eulerdamp", i32), ("solver", i32),
        ("ccd", i32), ("_pad0", i32),
        # bodies
        ("body_parentid", _a(i32, MAXBODY)), ("body_rootid", _a(i32, MAXBODY)),
        ("body_weldid", _a(i32, MAXBODY)), ("body_jntnum", _a(i32, MAXBODY)),
        ("body_jntadr", _a(i32, MAXBODY)), ("body_dofnum", _a(i32, MAXBODY)),
        ("body_dofadr", _a(i32, MAXBODY)),
        ("body_pos", _a(f64, MAXBODY, 3)), ("body_quat", _a(f64, MAXBODY, 4)),
        ("body_ipos", _a(f64, MAXBODY, 3)), ("body_iquat", _a(f64, MAXBODY, 4)),
        ("body_mass", _a(f64, MAXBODY)), ("body_inertia", _a(f64, MAXBODY, 3)),
        ("body_invweight0", _a(f64, MAXBODY, 2)),
        # joints
        ("jnt_type", _a(i32, MAXJNT)), ("jnt_bodyid", _a(i32, MAXJNT)),
        ("jnt_qposadr", _a(i32, MAXJNT)), ("jnt_dofadr", _a(i32, MAXJNT)),
        ("jnt_limited", _a(i32, MAXJNT)), ("_pad1", i32),
        ("jnt_pos", _a(f64, MAXJNT, 3)), ("jnt_axis", _a(f64, MAXJNT, 3)),
        ("jnt_range", _a(f64, MAXJNT, 2)), ("jnt_solref", _a(f64, MAXJNT, 2)),
        ("jnt_solimp", _a(f64, MAXJNT, 5)), ("jnt_margin", _a(f64, MAXJNT)),
        ("qpos0", _a(f64, MAXQ)),
        # dofs
        ("dof_bodyid", _a(i32, MAXDOF)), ("dof_jntid", _a(i32, MAXDOF)),
        ("dof_parentid", _a(i32, MAXDOF)),
        ("dof_armature", _a(f64, MAXDOF)), ("dof_damping", _a(f64, MAXDOF)),
        ("dof_frictionloss", _a(f64, MAXDOF)), ("dof_invweight0", _a(f64, MAXDOF)),
        ("dof_solref", _a(f64, MAXDOF, 2)), ("dof_solimp", _a(f64, MAXDOF, 5)),
        # geoms
        ("geom_type", _a(i32, MAXGEOM)), ("geom_bodyid", _a(i32, MAXGEOM)),
        ("geom_condim", _a(i32, MAXGEOM)), ("geom_hulladr", _a(i32, MAXGEOM)),
        ("geom_hullnum", _a(i32, MAXGEOM)), ("_pad2", i32),
        ("geom_pos", _a(f64, MAXGEOM, 3)), ("geom_quat", _a(f64, MAXGEOM, 4)),
        ("geom_size", _a(f64, MAXGEOM, 3)), ("geom_friction", _a(f64, MAXGEOM, 3)),
        ("geom_solref", _a(f64, MAXGEOM, 2)), ("geom_solimp", _a(f64, MAXGEOM, 5)),
        ("geom_margin", _a(f64, MAXGEOM)), ("geom_rbound", _a(f64, MAXGEOM)),
        ("geom_aabb", _a(f64, MAXGEOM, 6)),
        # pairs
        ("pair_geom1", _a(i32, MAXPAIR)), ("pair_geom2", _a(i32, MAXPAIR)),
        # sites
        ("site_bodyid", _a(i32, MAXSITE)), ("site_pos", _a(f64, MAXSITE, 3)),
        ("site_quat", _a(f64, MAXSITE, 4)),
        # actuators
        ("actuator_trnid", _a(i32, MAXU)), ("actuator_ctrllimited", _a(i32, MAXU)),
        ("actuator_forcelimited", _a(i32, MAXU)),
        ("actuator_gear", _a(f64, MAXU)), ("actuator_gainprm", _a(f64, MAXU)),
        ("actuator_biasprm", _a(f64, MAXU, 3)), ("actuator_ctrlrange", _a(f64, MAXU, 2)),
        ("actuator_forcerange", _a(f64, MAXU, 2)),
        # observation recipe
        ("obs_site", i32), ("obs_nq", i32), ("obs_qadr", _a(i32, MAXOBSQ)),
        ("nact", i32), ("_pad3", i32),
    ]


class IkOpts(_Versioned):
    _fields_ = [
        ("struct_size", i32), ("abi_version", i32),
        ("tol", f64), ("regularization_threshold", f64), ("regularization_strength", f64),
        ("max_update_norm", f64), ("progress_thresh", f64),
        ("max_steps", i32), ("site", i32), ("ndof", i32), ("_pad", i32), ("rot_weight", f64),
    ]


class SimState(C.Structure):
    _fields_ = [
        ("qpos", C.c_void_p), ("qvel", C.c_void_p), ("qacc_warmstart", C.c_void_p),
        ("ctrl", C.c_void_p), ("status", C.c_void_p), ("ncon", C.c_void_p),
        ("qfrc_applied", C.c_void_p),
    ]


KMAXLAYER = 6


class KoopmanDesc(C.Structure):
    """``sim_koopman_desc`` (include/koopman_mpc.h)."""
    _fields_ = [("x_dim", i32), ("u_dim", i32), ("nlayer", i32), ("width", _a(i32, KMAXLAYER + 1)),
                ("horizon", i32), ("_pad", i32), ("u_clip", f64)]


class SimParams(C.Structure):
    _fields_ = [("mass_scale", C.c_void_p), ("friction", C.c_void_p), ("damping_scale", C.c_void_p)]


PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "csrc", "libsoarm_sim.so")

# every symbol include/soarm_sim.h declares
EXPORTS = [
    "sim_last_error", "sim_version", "sim_model_create", "sim_model_free",
    "sim_batch_create", "sim_batch_free", "sim_batch_set_params", "sim_reset",
    "sim_step", "sim_substeps", "sim_bias", "sim_observe", "sim_contacts", "sim_collide_profile", "sim_phase_profile", "sim_ik_dls",
    "sim_profile_begin", "sim_profile_end", "sim_rand_uniform", "sim_ik_dls_pose",
    "sim_model_save", "sim_model_load",
    # include/koopman_mpc.h
    "sim_koopman_create", "sim_koopman_free", "sim_koopman_encode", "sim_koopman_feedforward",
    "sim_koopman_mpc_step", "sim_koopman_set_bilinear", "sim_koopman_bilinear_step",
]
PROF_KINDS = ["step_fused", "collide", "substep", "geom"]

_lib = None


def load_lib(path=None):
    """Load the HIP C-ABI library (raises if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("SOARM_SIM_LIB") or LIB_PATH  # env override: A/B builds (tools/)
    if not os.path.exists(p):
        raise RuntimeError(
            f"HIP library {p} not built; run `python __graft_entry__.py` (build()) first")
    lib = C.CDLL(p)
    vp, ip = C.c_void_p, C.c_int
    lib.sim_last_error.restype = C.c_char_p
    lib.sim_version.restype = C.c_char_p
    lib.sim_model_create.argtypes = [C.POINTER(ModelDesc), vp, vp, vp, C.POINTER(vp)]
    lib.sim_model_free.argtypes = [vp]
    lib.sim_model_free.restype = None
    lib.sim_model_save.argtypes = [C.POINTER(ModelDesc), vp, vp, vp, C.c_char_p]
    lib.sim_model_load.argtypes = [C.c_char_p, C.POINTER(vp)]
    lib.sim_batch_create.argtypes = [vp, ip, ip, C.POINTER(vp)]
    lib.sim_batch_free.argtypes = [vp]
    lib.sim_batch_free.restype = None
    lib.sim_batch_set_params.argtypes = [vp, C.POINTER(SimParams)]
    lib.sim_reset.argtypes = [vp, C.POINTER(SimState), vp, vp, vp, C.c_uint64, C.c_int64, vp, vp, vp]
    lib.sim_step.argtypes = [vp, C.POINTER(SimState), vp, ip, vp, vp]
    lib.sim_substeps.argtypes = [vp, C.POINTER(SimState), ip, vp]
    lib.sim_observe.argtypes = [vp, C.POINTER(SimState), vp, vp]
    lib.sim_bias.argtypes = [vp, C.POINTER(SimState), vp, vp]
    lib.sim_contacts.argtypes = [vp, C.POINTER(SimState), vp, vp, vp]
    lib.sim_collide_profile.argtypes = [vp, C.POINTER(SimState), vp, vp]
    lib.sim_phase_profile.argtypes = [vp, ip]
    lib.sim_profile_begin.argtypes = [vp]
    lib.sim_profile_end.argtypes = [vp, vp, vp]
    lib.sim_ik_dls.argtypes = [vp, vp, vp, vp, vp, C.POINTER(IkOpts), vp]
    lib.sim_ik_dls_pose.argtypes = [vp, vp, vp, vp, vp, vp, C.POINTER(IkOpts), vp]
    lib.sim_rand_uniform.argtypes = [vp, C.c_uint64, C.c_int64, C.c_uint32, ip, C.c_float, C.c_float, vp, vp]
    lib.sim_koopman_create.argtypes = [C.POINTER(KoopmanDesc), vp, vp, ip, C.POINTER(vp)]
    lib.sim_koopman_free.argtypes = [vp]
    lib.sim_koopman_free.restype = None
    lib.sim_koopman_encode.argtypes = [vp, ip, vp, vp, vp]
    lib.sim_koopman_feedforward.argtypes = [vp, ip, ip, ip, vp, vp, vp]
    lib.sim_koopman_mpc_step.argtypes = [vp, ip, vp, vp, vp, vp, vp, vp]
    lib.sim_koopman_set_bilinear.argtypes = [vp, vp, vp, vp, ip, C.c_double, C.c_double]
    lib.sim_koopman_bilinear_step.argtypes = [vp, ip, vp, vp, vp, vp, vp]
    for name in EXPORTS:
        if not hasattr(lib, name):
            raise RuntimeError(f"{p} does not export {name}")
    if path is None:
        _lib = lib
    return lib


def check(lib, rc):
    if rc != 0:
        raise RuntimeError(f"soarm_sim error {rc}: {lib.sim_last_error().decode()}")
