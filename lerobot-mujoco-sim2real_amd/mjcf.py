"""MJCF -> compiled model (``sim_model_desc``) for the batched simulator.

Replaces ``mujoco.MjModel.from_xml_path`` (``SOARM101/SOARM101_Env.py:34``) for
the subset of MJCF the hot-path scene uses (``SOARM101/SO101/scene_with_table_v.xml``
and its include ``so101_new_calib_v.xml``), following MuJoCo's compiler rules
[ext, MuJoCo user/xml docs]:

* ``<include>`` splices the included file's top-level sections; ``<compiler>``
  attributes accumulate in document order (``angle="radian"`` comes from the
  include, ``so101_new_calib_v.xml:5``); ``autolimits`` makes a ``range``
  imply ``limited``.
* default classes nest; an element takes ``class=`` or the enclosing body's
  ``childclass`` (``so101_new_calib_v.xml:34``) or ``main``.
* actuator shortcuts share ONE default actuator per class: ``<position kp=50>``
  in class ``sts3215`` (``so101_new_calib_v.xml:23``) sets its gainprm[0] = 50,
  and a ``<velocity>`` element without ``kv`` (``so101_new_calib_v.xml:160-165``)
  keeps that gain: force = 50*(ctrl - qvel), biasprm[2] = -gainprm[0].  The
  ``kv`` argument of :func:`compile_mjcf` overrides it (MuJoCo's bare default
  would be kv = 1; SURVEY.md §8 keeps this switchable).
* only collidable geoms (contype|conaffinity != 0) are compiled; ``type="mesh"``
  geoms collide as the convex hull of the mesh (``hulls.npz``).
* candidate pairs: contype/conaffinity filter, same-weld-body and
  parent/child filter (world exempt) — 71 pairs for the arm on the table.
  Pairs are ordered by (body1, body2) then geom order, and each pair is
  ordered by geom type (MuJoCo's collision table is upper-triangular), which
  fixes contact indexing deterministically.
* ``body_invweight0`` / ``dof_invweight0`` are computed at qpos0 as in
  ``mj_setConst`` (used by constraint regularisation).

No ``<option>`` element exists in the scene, so MuJoCo defaults apply:
timestep 0.002, gravity (0, 0, -9.81), impratio 1, Euler with implicit damping.
"""
import os
import xml.etree.ElementTree as ET

import numpy as np

from . import abi

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "so101")
SCENE_XML = os.path.join(ASSET_DIR, "scene_with_table_v.xml")
CUBE_SCENE_XML = os.path.join(ASSET_DIR, "scene_with_table_cube_v.xml")
# position-servo scenes (kp = 50 class default, forcerange +-33.5) of the viewer / sim2real scripts
POSITION_SCENE_XML = os.path.join(ASSET_DIR, "scene_with_table.xml")
FLOOR_SCENE_XML = os.path.join(ASSET_DIR, "scene.xml")
# the old calibration's arm on its own (no scene includes it; SO101/so101_old_calib.xml)
OLD_CALIB_XML = os.path.join(ASSET_DIR, "so101_old_calib.xml")

# MuJoCo defaults (mjmodel.h / user_objects docs)
DEF_SOLREF = (0.02, 1.0)
DEF_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)
DEF_FRICTION = (1.0, 0.005, 0.0001)

JOINT_TYPES = {"free": abi.JNT_FREE, "ball": abi.JNT_BALL, "slide": abi.JNT_SLIDE,
               "hinge": abi.JNT_HINGE}
GEOM_TYPES = {"plane": abi.GEOM_PLANE, "sphere": abi.GEOM_SPHERE, "box": abi.GEOM_BOX,
              "mesh": abi.GEOM_MESH}


# ----------------------------------------------------------------- math helpers
def quat_normalize(q):
    q = np.asarray(q, dtype=np.float64)
    return q / np.linalg.norm(q)


def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                     w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def quat2mat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def mat2quat(R):
    """Rotation matrix -> unit quaternion (w >= 0)."""
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = quat_normalize(q)
    return q if q[0] >= 0 else -q


def axisangle_quat(axis, ang):
    axis = np.asarray(axis, dtype=np.float64)
    return np.concatenate([[np.cos(ang / 2)], np.sin(ang / 2) * axis])


# ------------------------------------------------------------------ XML loading
def _floats(s):
    return [float(x) for x in s.split()]


def _load_tree(path, seen=None):
    """Parse `path`, splicing <include> elements recursively."""
    seen = seen or set()
    path = os.path.abspath(path)
    if path in seen:
        raise ValueError(f"recursive include of {path}")
    seen = seen | {path}
    root = ET.parse(path).getroot()
    base = os.path.dirname(path)

    def splice(elem):
        out = []
        for ch in list(elem):
            if ch.tag == "include":
                inc = _load_tree(os.path.join(base, ch.get("file")), seen)
                out.extend(inc)  # top-level sections of the included <mujoco>
            else:
                splice(ch)
                out.append(ch)
        for ch in list(elem):
            elem.remove(ch)
        elem.extend(out)
        return elem

    return splice(root)


class _Defaults:
    """MuJoCo default-class tree: class name -> {element kind -> attrs}."""

    def __init__(self):
        self.classes = {"main": {}}

    def parse(self, elem, parent="main"):
        """Parse a nested ``<default class=...>`` inheriting from `parent`."""
        name = elem.get("class")
        if name is None:
            raise ValueError("nested <default> needs a class attribute")
        base = {k: dict(v) for k, v in self.classes[parent].items()}
        if "actuator" in base and "biasprm" in base["actuator"]:
            base["actuator"]["biasprm"] = list(base["actuator"]["biasprm"])
        self.classes[name] = base
        for ch in elem:
            if ch.tag == "default":
                self.parse(ch, name)
            elif ch.tag in ("position", "velocity", "motor", "general"):
                act = base.setdefault("actuator", {})
                _apply_actuator_shortcut(act, ch.tag, ch.attrib, is_default=True)
            else:
                base.setdefault(ch.tag, {}).update(ch.attrib)

    def get(self, cls, kind):
        return dict(self.classes.get(cls or "main", {}).get(kind, {}))


def _apply_actuator_shortcut(act, kind, attrib, is_default=False):
    """MuJoCo actuator shortcut semantics on a 'general actuator' dict."""
    for k in ("ctrlrange", "forcerange", "ctrllimited", "forcelimited", "gear", "joint"):
        if k in attrib:
            act[k] = attrib[k]
    gain = float(act.get("gainprm0", 1.0))
    if kind == "position":
        kp = float(attrib.get("kp", gain))
        act["gainprm0"] = kp
        # kv / dampratio not given: the actuator keeps its current (class default) value.
        # dampratio is kept as a positive biasprm[2] and turned into -kv once the model's
        # inertia is known (mj_setConst), see _set_dampratio
        b2 = float(act.get("biasprm", [0.0, 0.0, 0.0])[2])
        if "dampratio" in attrib:
            b2 = float(attrib["dampratio"])
        elif "kv" in attrib:
            b2 = -float(attrib["kv"])
        act["biasprm"] = [0.0, -kp, b2]
    elif kind == "velocity":
        kv = float(attrib.get("kv", gain))   # no kv attribute -> class default gain
        act["gainprm0"] = kv
        act["biasprm"] = [0.0, 0.0, -kv]
    elif kind == "motor":
        act["gainprm0"] = 1.0
        act["biasprm"] = [0.0, 0.0, 0.0]
    elif kind == "general":
        if "gainprm" in attrib:
            act["gainprm0"] = _floats(attrib["gainprm"])[0]
        if "biasprm" in attrib:
            act["biasprm"] = (_floats(attrib["biasprm"]) + [0, 0, 0])[:3]


# -------------------------------------------------------------- compiled model
class CompiledModel:
    """Compiled MJCF: the C struct plus names and hull arrays."""

    def __init__(self):
        self.desc = abi.ModelDesc()
        self.body_names, self.joint_names, self.geom_names = [], [], []
        self.site_names, self.actuator_names = [], []
        self.keyframes = {}
        self.hull_vert = np.zeros((0, 3), np.float32)
        self.hull_adr = np.zeros(1, np.int32)
        self.hull_adj = np.zeros(0, np.int32)
        self.source = None

    def save(self, path):
        """Write the compiled model file `sim_model_load` reads (include/soarm_sim.h): a C / C++
        caller then loads the model with no Python at run time (SOARM101_Env.py:34's
        MjModel.from_xml_path).  Names and keyframes are not part of the file."""
        import ctypes as C

        lib = abi.load_lib()
        hv = np.ascontiguousarray(self.hull_vert, np.float32)
        ha = np.ascontiguousarray(self.hull_adr, np.int32)
        hj = np.ascontiguousarray(self.hull_adj, np.int32)
        abi.check(lib, lib.sim_model_save(C.byref(self.desc), hv.ctypes.data_as(C.c_void_p),
                                          ha.ctypes.data_as(C.c_void_p), hj.ctypes.data_as(C.c_void_p),
                                          os.fsencode(path)))

    # name lookup (mj_name2id equivalents)
    def body(self, name):
        return self.body_names.index(name)

    def joint(self, name):
        return self.joint_names.index(name)

    def site(self, name):
        return self.site_names.index(name)

    def geom(self, name):
        return self.geom_names.index(name)

    @property
    def nq(self):
        return self.desc.nq

    @property
    def nv(self):
        return self.desc.nv

    @property
    def nu(self):
        return self.desc.nu

    @property
    def timestep(self):
        return self.desc.timestep

    def qpos0(self):
        return np.array(self.desc.qpos0[: self.desc.nq])


def _orient(attrib, angle_scale):
    if "quat" in attrib:
        return quat_normalize(_floats(attrib["quat"]))
    if "axisangle" in attrib:
        v = _floats(attrib["axisangle"])
        ax = np.asarray(v[:3]) / np.linalg.norm(v[:3])
        return axisangle_quat(ax, v[3] * angle_scale)
    if "euler" in attrib:  # MuJoCo default eulerseq "xyz" (intrinsic)
        e = np.asarray(_floats(attrib["euler"])) * angle_scale
        q = np.array([1.0, 0, 0, 0])
        for k, a in enumerate(e):
            ax = np.zeros(3)
            ax[k] = 1
            q = quat_mul(q, axisangle_quat(ax, a))
        return quat_normalize(q)
    return np.array([1.0, 0.0, 0.0, 0.0])


def _load_hulls(path=None):
    z = np.load(path or os.path.join(ASSET_DIR, "hulls.npz"))
    out = {}
    for k in z.files:
        name, part = k.rsplit("/", 1)
        out.setdefault(name, {})[part] = z[k]
    return out


def hull_with_graph(verts_f32):
    """Convex hull of a vertex cloud plus its vertex adjacency graph (the hill-climbing support
    queries walk it): hull vertices (float32, ascending input order), CSR neighbour lists."""
    from scipy.spatial import ConvexHull
    pts = np.unique(np.asarray(verts_f32, dtype=np.float32), axis=0)
    h = ConvexHull(pts.astype(np.float64))
    hv = np.sort(h.vertices)
    local = -np.ones(len(pts), dtype=np.int64)
    local[hv] = np.arange(len(hv))
    nbr = [set() for _ in range(len(hv))]
    for tri in h.simplices:
        a, b, c = local[tri]
        nbr[a].update((b, c))
        nbr[b].update((a, c))
        nbr[c].update((a, b))
    adr = np.zeros(len(hv) + 1, dtype=np.int32)
    adj = []
    for i, s in enumerate(nbr):
        lst = sorted(s)
        adj.extend(lst)
        adr[i + 1] = adr[i] + len(lst)
    return pts[hv].astype(np.float32), np.asarray(adj, dtype=np.int32), adr


def vertex_hull(verts_f32):
    """hulls.npz-style record of an inline ``<mesh vertex="...">`` asset: MuJoCo makes such a
    mesh the convex hull of its vertices, and its centre the hull's volume centroid."""
    from scipy.spatial import ConvexHull
    v, adj, adr = hull_with_graph(verts_f32)
    p = v.astype(np.float64)
    h = ConvexHull(p)
    o = p.mean(0)
    a, b, c = (p[h.simplices[:, k]] for k in range(3))
    vol = np.abs(np.einsum("ij,ij->i", a - o, np.cross(b - o, c - o))) / 6.0
    com = (vol[:, None] * (a + b + c + o) / 4.0).sum(0) / vol.sum()
    return {"v": v, "adj": adj, "adr": adr, "com": com}


def compile_mjcf(xml_path=SCENE_XML, kv=None, disable_contact=False, iterations=100,
                 tolerance=1e-8, obs_site="gripperframe",
                 obs_joints=("shoulder_pan", "shoulder_lift", "elbow_flex", "wrist_flex", "wrist_roll"),
                 solver="PGS", ccd="native"):
    """Compile an MJCF file into a :class:`CompiledModel`.

    ccd: the convex-convex narrowphase, "native" (MuJoCo's GJK/EPA, the default of current
    releases, and so this compiler's) or "mpr" (libccd MPR, MuJoCo's classic path); an explicit
    ``<option><flag nativeccd="disable"/></option>`` in the MJCF selects MPR.

    solver: "PGS" (the north star's and BASELINE config 3's solver, the headline) or "Newton"
    (MuJoCo's default, which the reference scene's missing <option> selects): both run on the
    device (soarm_pgs.h / soarm_newton.h) and in the oracle; only CG is rejected."""
    if not os.path.exists(xml_path):
        raise FileNotFoundError(f"MuJoCo XML file not found: {xml_path}")
    root = _load_tree(xml_path)
    cm = CompiledModel()
    cm.source = os.path.abspath(xml_path)
    d = cm.desc

    compiler = {}
    for c in root.iter("compiler"):
        compiler.update(c.attrib)
    angle_scale = 1.0 if compiler.get("angle", "degree") == "radian" else np.pi / 180
    autolimits = compiler.get("autolimits", "true") == "true"

    defaults = _Defaults()
    for dsec in root.findall("default"):
        # top-level <default> is class main; its children are nested classes
        for ch in dsec:
            if ch.tag == "default":
                defaults.parse(ch, "main")
            elif ch.tag in ("position", "velocity", "motor", "general"):
                _apply_actuator_shortcut(defaults.classes["main"].setdefault("actuator", {}),
                                         ch.tag, ch.attrib, True)
            else:
                defaults.classes["main"].setdefault(ch.tag, {}).update(ch.attrib)

    # mesh assets: name -> file stem (hull in hulls.npz) or, for an inline ``vertex`` mesh, its
    # own hull computed here
    meshes = {}
    hulls = _load_hulls()
    for asec in root.findall("asset"):
        for m in asec.findall("mesh"):
            f = m.get("file")
            if f is None and m.get("vertex") is not None:
                nm = m.get("name")
                if not nm:
                    raise ValueError("an inline (vertex) mesh needs a name")
                v = np.asarray(_floats(m.get("vertex")), dtype=np.float32).reshape(-1, 3)
                v = v * np.asarray(_floats(m.get("scale", "1 1 1")), dtype=np.float32)
                hulls[nm] = vertex_hull(v)
                meshes[nm] = nm
                continue
            nm = m.get("name") or os.path.splitext(os.path.basename(f))[0]
            meshes[nm] = os.path.splitext(os.path.basename(f))[0]

    # option (none in the reference scene -> MuJoCo defaults)
    opt = {}
    for o in root.iter("option"):
        opt.update(o.attrib)
    d.timestep = float(opt.get("timestep", 0.002))
    g = _floats(opt.get("gravity", "0 0 -9.81"))
    d.gravity[:] = g
    d.impratio = float(opt.get("impratio", 1.0))
    d.tolerance = tolerance
    d.iterations = iterations
    sol = {"pgs": abi.SOL_PGS, "newton": abi.SOL_NEWTON}
    if str(solver).lower() not in sol:
        raise ValueError(f"solver must be PGS or Newton, not {solver!r}")
    d.solver = sol[str(solver).lower()]
    ccds = {"mpr": abi.CCD_MPR, "native": abi.CCD_NATIVE}
    if str(ccd).lower() not in ccds:
        raise ValueError(f"ccd must be 'native' or 'mpr', not {ccd!r}")
    d.ccd = ccds[str(ccd).lower()]
    for o in root.iter("option"):
        for fl in o.iter("flag"):
            if fl.get("nativeccd") == "disable":
                d.ccd = abi.CCD_MPR
    d.disable_contact = int(bool(disable_contact))

    # ---- walk bodies depth-first; worldbody sections merged in order
    bodies = [dict(name="world", parent=-1, pos=np.zeros(3), quat=np.array([1.0, 0, 0, 0]),
                   ipos=np.zeros(3), iquat=np.array([1.0, 0, 0, 0]), mass=0.0, inertia=np.zeros(3),
                   joints=[], geoms_all=[])]
    joints, geoms, sites = [], [], []

    def elem_attrs(el, kind, childclass):
        a = defaults.get(el.get("class") or childclass, kind)
        a.update(el.attrib)
        return a

    def walk(el, bid, childclass):
        for ch in el:
            if ch.tag == "body":
                cc = ch.get("childclass", childclass)
                b = dict(name=ch.get("name", f"body{len(bodies)}"), parent=bid,
                         pos=np.asarray(_floats(ch.get("pos", "0 0 0"))),
                         quat=_orient(ch.attrib, angle_scale), joints=[], geoms_all=[],
                         inertial=None)
                nb = len(bodies)
                bodies.append(b)
                for sub in ch:
                    if sub.tag == "inertial":
                        b["inertial"] = sub.attrib
                walk(ch, nb, cc)
            elif ch.tag in ("joint", "freejoint"):
                a = elem_attrs(ch, "joint", childclass) if ch.tag == "joint" else dict(ch.attrib, type="free")
                joints.append((bid, a))
                bodies[bid]["joints"].append(len(joints) - 1)
            elif ch.tag == "geom":
                a = elem_attrs(ch, "geom", childclass)
                geoms.append((bid, a))
                bodies[bid]["geoms_all"].append(len(geoms) - 1)
            elif ch.tag == "site":
                a = elem_attrs(ch, "site", childclass)
                sites.append((bid, a))

    for wb in root.findall("worldbody"):
        walk(wb, 0, None)

    nbody = len(bodies)
    if nbody > abi.MAXBODY:
        raise ValueError("too many bodies")
    d.nbody = nbody

    # ---- geoms: types, sizes, poses, collidability
    cgeoms = []  # compiled collidable geoms
    hv, hadr, hadj = [], [0], []
    for gi, (bid, a) in enumerate(geoms):
        gtype = a.get("type", "sphere")
        contype = int(a.get("contype", 1))
        conaff = int(a.get("conaffinity", 1))
        info = dict(body=bid, type=gtype, a=a, pos=np.asarray(_floats(a.get("pos", "0 0 0"))),
                    quat=_orient(a, angle_scale), contype=contype, conaff=conaff)
        if gtype == "mesh":
            info["mesh"] = meshes.get(a.get("mesh"), a.get("mesh"))
        geoms[gi] = (bid, a, info)
        if contype == 0 and conaff == 0:
            continue
        if gtype not in GEOM_TYPES:
            raise ValueError(f"geom type {gtype} not supported")
        cgeoms.append(info)

    # ---- body inertials (explicit, else from the body's geoms: boxes only here)
    for b in bodies[1:]:
        ine = b.get("inertial")
        if ine is not None:
            b["ipos"] = np.asarray(_floats(ine.get("pos", "0 0 0")))
            b["mass"] = float(ine["mass"])
            if "fullinertia" in ine:
                xx, yy, zz, xy, xz, yz = _floats(ine["fullinertia"])
                I = np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]])
                iq = _orient(ine, angle_scale)
                I = quat2mat(iq) @ I @ quat2mat(iq).T
                w, V = np.linalg.eigh(I)
                if np.linalg.det(V) < 0:
                    V[:, 2] = -V[:, 2]
                b["inertia"] = w
                b["iquat"] = mat2quat(V)
            else:
                b["inertia"] = np.asarray(_floats(ine["diaginertia"]))
                b["iquat"] = _orient(ine, angle_scale)
        else:
            # inertia from geoms (only boxes/spheres with explicit mass or density 1000)
            mass, ipos, inertia = 0.0, np.zeros(3), np.zeros(3)
            for gidx in b["geoms_all"]:
                _, a, info = geoms[gidx]
                sz = np.asarray(_floats(a.get("size", "0 0 0")))
                if info["type"] == "box":
                    vol = 8 * sz[0] * sz[1] * sz[2]
                    m = float(a["mass"]) if "mass" in a else 1000.0 * vol
                    inertia = m / 3.0 * np.array([sz[1] ** 2 + sz[2] ** 2, sz[0] ** 2 + sz[2] ** 2,
                                                  sz[0] ** 2 + sz[1] ** 2])
                elif info["type"] == "sphere":
                    vol = 4 / 3 * np.pi * sz[0] ** 3
                    m = float(a["mass"]) if "mass" in a else 1000.0 * vol
                    inertia = np.full(3, 0.4 * m * sz[0] ** 2)
                else:
                    raise ValueError("inertia from geoms supports box/sphere only")
                mass = m
                ipos = info["pos"]
            b["mass"], b["ipos"], b["inertia"] = mass, ipos, inertia
            b["iquat"] = np.array([1.0, 0, 0, 0])

    # ---- joints / dofs, in body order
    jorder = []
    for bid, b in enumerate(bodies):
        jorder.extend(b["joints"])
    jmap = {old: new for new, old in enumerate(jorder)}
    nq = nv = 0
    qpos0 = []
    d.njnt = len(jorder)
    if d.njnt > abi.MAXJNT:
        raise ValueError("too many joints")
    dof_info = []
    for new, old in enumerate(jorder):
        bid, a = joints[old]
        jt = a.get("type", "hinge")
        jtype = JOINT_TYPES[jt]
        cm.joint_names.append(a.get("name", f"joint{new}"))
        d.jnt_type[new] = jtype
        d.jnt_bodyid[new] = bid
        d.jnt_qposadr[new] = nq
        d.jnt_dofadr[new] = nv
        d.jnt_pos[new][:] = _floats(a.get("pos", "0 0 0"))
        ax = np.asarray(_floats(a.get("axis", "0 0 1")))
        d.jnt_axis[new][:] = ax / np.linalg.norm(ax)
        rng = _floats(a["range"]) if "range" in a else [0.0, 0.0]
        if jtype in (abi.JNT_HINGE, abi.JNT_BALL):
            rng = [r * angle_scale for r in rng]
        d.jnt_range[new][:] = rng
        lim = a.get("limited", "auto")
        limited = (lim == "true") or (lim == "auto" and autolimits and "range" in a)
        d.jnt_limited[new] = int(limited and jtype != abi.JNT_FREE)
        d.jnt_solref[new][:] = _floats(a["solreflimit"]) if "solreflimit" in a else DEF_SOLREF
        d.jnt_solimp[new][:] = _floats(a["solimplimit"]) if "solimplimit" in a else DEF_SOLIMP
        d.jnt_margin[new] = float(a.get("margin", 0.0))
        ndof = {abi.JNT_FREE: 6, abi.JNT_BALL: 3}.get(jtype, 1)
        if jtype == abi.JNT_FREE:
            b = bodies[bid]
            qpos0.extend(list(b["pos"]) + list(b["quat"]))
            nq += 7
        elif jtype == abi.JNT_BALL:
            qpos0.extend([1.0, 0, 0, 0])
            nq += 4
        else:
            qpos0.append(float(a.get("ref", 0.0)))
            nq += 1
        for k in range(ndof):
            dof_info.append(dict(body=bid, jnt=new,
                                 damping=float(a.get("damping", 0.0)),
                                 armature=float(a.get("armature", 0.0)),
                                 frictionloss=float(a.get("frictionloss", 0.0)),
                                 solref=_floats(a["solreffriction"]) if "solreffriction" in a else DEF_SOLREF,
                                 solimp=_floats(a["solimpfriction"]) if "solimpfriction" in a else DEF_SOLIMP))
        nv += ndof
    if nq > abi.MAXQ or nv > abi.MAXDOF:
        raise ValueError("model too large")
    d.nq, d.nv = nq, nv
    d.qpos0[:nq] = qpos0

    # ---- bodies
    dof_of_body = {}
    for i, di in enumerate(dof_info):
        dof_of_body.setdefault(di["body"], []).append(i)
    for bid, b in enumerate(bodies):
        cm.body_names.append(b["name"])
        d.body_parentid[bid] = max(b["parent"], 0)
        d.body_pos[bid][:] = b["pos"]
        d.body_quat[bid][:] = b["quat"]
        d.body_ipos[bid][:] = b["ipos"]
        d.body_iquat[bid][:] = b["iquat"]
        d.body_mass[bid] = b["mass"]
        d.body_inertia[bid][:] = b["inertia"]
        js = [jmap[j] for j in b["joints"]]
        d.body_jntnum[bid] = len(js)
        d.body_jntadr[bid] = js[0] if js else -1
        ds = dof_of_body.get(bid, [])
        d.body_dofnum[bid] = len(ds)
        d.body_dofadr[bid] = ds[0] if ds else -1
    for bid in range(nbody):
        # root = child of world on the path; weld = nearest ancestor-or-self with dofs
        r = bid
        while r > 0 and d.body_parentid[r] != 0:
            r = d.body_parentid[r]
        d.body_rootid[bid] = r
        w = bid
        while w > 0 and d.body_jntnum[w] == 0:
            w = d.body_parentid[w]
        d.body_weldid[bid] = w

    # dofs
    for i, di in enumerate(dof_info):
        d.dof_bodyid[i] = di["body"]
        d.dof_jntid[i] = di["jnt"]
        d.dof_damping[i] = di["damping"]
        d.dof_armature[i] = di["armature"]
        d.dof_frictionloss[i] = di["frictionloss"]
        d.dof_solref[i][:] = di["solref"]
        d.dof_solimp[i][:] = di["solimp"]
        # parent dof: previous dof of the same joint, else last dof of nearest ancestor body with dofs
        if i > 0 and dof_info[i - 1]["jnt"] == di["jnt"]:
            d.dof_parentid[i] = i - 1
        else:
            p = d.body_parentid[di["body"]]
            while p > 0 and d.body_dofnum[p] == 0:
                p = d.body_parentid[p]
            d.dof_parentid[i] = (d.body_dofadr[p] + d.body_dofnum[p] - 1) if p > 0 else -1

    # ---- collidable geoms
    if len(cgeoms) > abi.MAXGEOM:
        raise ValueError("too many geoms")
    d.ngeom = len(cgeoms)
    for gi, info in enumerate(cgeoms):
        a = info["a"]
        cm.geom_names.append(a.get("name", f"geom{gi}"))
        gt = GEOM_TYPES[info["type"]]
        d.geom_type[gi] = gt
        d.geom_bodyid[gi] = info["body"]
        d.geom_condim[gi] = int(a.get("condim", 3))
        d.geom_pos[gi][:] = info["pos"]
        d.geom_quat[gi][:] = info["quat"]
        d.geom_friction[gi][:] = (_floats(a["friction"]) + list(DEF_FRICTION))[:3] if "friction" in a \
            else DEF_FRICTION
        d.geom_solref[gi][:] = _floats(a["solref"]) if "solref" in a else DEF_SOLREF
        d.geom_solimp[gi][:] = _floats(a["solimp"]) if "solimp" in a else DEF_SOLIMP
        d.geom_margin[gi] = float(a.get("margin", 0.0))
        d.geom_hulladr[gi] = -1
        d.geom_hullnum[gi] = 0
        if gt == abi.GEOM_MESH:
            h = hulls[info["mesh"]]
            d.geom_hulladr[gi] = sum(len(x) for x in hv)
            d.geom_hullnum[gi] = len(h["v"])
            base_adj = sum(len(x) for x in hadj)
            hv.append(h["v"])
            hadj.append(h["adj"])
            hadr.extend(list(h["adr"][1:] + base_adj))
            # collision centre = mesh volume centroid (MuJoCo's re-centred mesh frame)
            c = np.asarray(h["com"], dtype=np.float64)
            half = np.max(np.abs(h["v"].astype(np.float64) - c), axis=0)
            d.geom_aabb[gi][:] = list(c) + list(half)
            d.geom_rbound[gi] = float(np.max(np.linalg.norm(h["v"] - c, axis=1)))
        elif gt == abi.GEOM_BOX:
            sz = _floats(a["size"])
            d.geom_size[gi][:] = sz
            d.geom_aabb[gi][:] = [0, 0, 0] + sz
            d.geom_rbound[gi] = float(np.linalg.norm(sz))
        elif gt == abi.GEOM_SPHERE:
            sz = _floats(a["size"])[:1]
            d.geom_size[gi][0] = sz[0]
            d.geom_aabb[gi][:] = [0, 0, 0] + sz * 3
            d.geom_rbound[gi] = sz[0]
        elif gt == abi.GEOM_PLANE:
            sz = (_floats(a.get("size", "0 0 0")) + [0, 0, 0])[:3]
            d.geom_size[gi][:] = sz
            d.geom_rbound[gi] = 0.0
    if hv:
        cm.hull_vert = np.ascontiguousarray(np.concatenate(hv), dtype=np.float32)
        cm.hull_adj = np.ascontiguousarray(np.concatenate(hadj), dtype=np.int32)
        cm.hull_adr = np.asarray(hadr, dtype=np.int32)
    d.nhullvert = len(cm.hull_vert)
    d.nhulladj = len(cm.hull_adj)

    # ---- candidate pairs (static broadphase filter), deterministic order
    pairs = []
    ng = d.ngeom
    for i in range(ng):
        for j in range(i + 1, ng):
            gi, gj = cgeoms[i], cgeoms[j]
            if not ((gi["contype"] & gj["conaff"]) or (gj["contype"] & gi["conaff"])):
                continue
            bi, bj = gi["body"], gj["body"]
            wi, wj = d.body_weldid[bi], d.body_weldid[bj]
            if wi == wj:
                continue
            pwi, pwj = d.body_weldid[d.body_parentid[wi]], d.body_weldid[d.body_parentid[wj]]
            if wi != 0 and wj != 0 and (wi == pwj or wj == pwi):
                continue
            b1, b2 = (bi, bj) if bi <= bj else (bj, bi)
            g1, g2 = (i, j) if bi <= bj else (j, i)
            pairs.append((b1, b2, g1, g2))
    pairs.sort()
    if len(pairs) > abi.MAXPAIR:
        raise ValueError("too many pairs")
    d.npair = len(pairs)
    for k, (_, _, g1, g2) in enumerate(pairs):
        if d.geom_type[g1] > d.geom_type[g2]:
            g1, g2 = g2, g1
        d.pair_geom1[k], d.pair_geom2[k] = g1, g2

    # ---- sites
    d.nsite = len(sites)
    for si, (bid, a) in enumerate(sites):
        cm.site_names.append(a.get("name", f"site{si}"))
        d.site_bodyid[si] = bid
        d.site_pos[si][:] = _floats(a.get("pos", "0 0 0"))
        d.site_quat[si][:] = _orient(a, angle_scale)

    # ---- actuators
    acts = []
    for asec in root.findall("actuator"):
        for el in asec:
            if el.tag not in ("position", "velocity", "motor", "general"):
                continue
            base = defaults.get(el.get("class"), "actuator")
            if "biasprm" in base:
                base["biasprm"] = list(base["biasprm"])
            _apply_actuator_shortcut(base, el.tag, el.attrib)
            if kv is not None and el.tag == "velocity":
                base["gainprm0"] = kv
                base["biasprm"] = [0.0, 0.0, -kv]
            acts.append((el.get("name", f"act{len(acts)}"), base))
    d.nu = len(acts)
    for ai, (nm, a) in enumerate(acts):
        cm.actuator_names.append(nm)
        d.actuator_trnid[ai] = cm.joint_names.index(a["joint"])
        d.actuator_gear[ai] = _floats(a.get("gear", "1"))[0]
        d.actuator_gainprm[ai] = float(a.get("gainprm0", 1.0))
        d.actuator_biasprm[ai][:] = a.get("biasprm", [0.0, 0.0, 0.0])
        cr = _floats(a["ctrlrange"]) if "ctrlrange" in a else [0.0, 0.0]
        fr = _floats(a["forcerange"]) if "forcerange" in a else [0.0, 0.0]
        d.actuator_ctrlrange[ai][:] = cr
        d.actuator_forcerange[ai][:] = fr
        cl, fl = a.get("ctrllimited", "auto"), a.get("forcelimited", "auto")
        d.actuator_ctrllimited[ai] = int(cl == "true" or (cl == "auto" and autolimits and "ctrlrange" in a))
        d.actuator_forcelimited[ai] = int(fl == "true" or (fl == "auto" and autolimits and "forcerange" in a))

    # ---- keyframes
    for ks in root.findall("keyframe"):
        for k in ks.findall("key"):
            cm.keyframes[k.get("name")] = dict(
                qpos=np.asarray(_floats(k.get("qpos"))) if k.get("qpos") else None,
                ctrl=np.asarray(_floats(k.get("ctrl"))) if k.get("ctrl") else None)

    # ---- observation recipe (SOARM101_Env.py:46-50, 69-75)
    d.obs_site = cm.site(obs_site)
    d.obs_nq = len(obs_joints)
    for k, jn in enumerate(obs_joints):
        d.obs_qadr[k] = d.jnt_qposadr[cm.joint(jn)]
    d.nact = len(obs_joints)

    # ---- invweight0 at qpos0 (mj_setConst)
    kin = NumpyKinematics(cm)
    q0 = cm.qpos0()
    kin.forward_position(q0)
    M = kin.mass_matrix()
    Minv = np.linalg.inv(M) if nv else np.zeros((0, 0))
    # mjStatistic.meaninertia: mean diagonal of M at qpos0 (armature included)
    d.meaninertia = float(np.trace(M) / nv) if nv else 1.0
    for bid in range(1, nbody):
        jp, jr = kin.jac(kin.xipos[bid], bid)
        J = np.vstack([jp, jr])
        A = J @ Minv @ J.T
        d.body_invweight0[bid][0] = max(np.trace(A[:3, :3]) / 3, 0.0)
        d.body_invweight0[bid][1] = max(np.trace(A[3:, 3:]) / 3, 0.0)
    for j in range(d.njnt):
        adr = d.jnt_dofadr[j]
        if d.jnt_type[j] == abi.JNT_FREE:
            t = np.mean([Minv[adr + k, adr + k] for k in range(3)])
            r = np.mean([Minv[adr + 3 + k, adr + 3 + k] for k in range(3)])
            for k in range(3):
                d.dof_invweight0[adr + k] = t
                d.dof_invweight0[adr + 3 + k] = r
        elif d.jnt_type[j] == abi.JNT_BALL:
            r = np.mean([Minv[adr + k, adr + k] for k in range(3)])
            for k in range(3):
                d.dof_invweight0[adr + k] = r
        else:
            d.dof_invweight0[adr] = Minv[adr, adr]
    _set_dampratio(d)
    return cm


def _set_dampratio(d):
    """Position actuators given ``dampratio`` (``so101_new_calib.xml:11,23``) [ext, mj_setConst]:
    a positive biasprm[2] marks a damping ratio; it becomes the velocity gain
    kv = dampratio * 2 * sqrt(kp * m), m = gear^2 / dof_invweight0 the inertia the actuator moves
    at qpos0, stored as biasprm[2] = -kv.  (Only the position-servo scenes use it: the hot-path
    velocity servos override biasprm, so101_new_calib_v.xml:160-165.)"""
    for a in range(d.nu):
        b = d.actuator_biasprm[a]
        kp = d.actuator_gainprm[a]
        if b[2] <= 0.0 or kp != -b[1]:
            continue
        dof = d.jnt_dofadr[d.actuator_trnid[a]]
        m = d.actuator_gear[a] ** 2 / d.dof_invweight0[dof]
        b[2] = -b[2] * 2.0 * np.sqrt(kp * m)


class NumpyKinematics:
    """Small float64 numpy rigid-body pass (FK, Jacobians, CRBA by Σ Jᵀ I J).

    Used by the compiler for invweight0 and, in tests, as an independent
    cross-check of the oracle's recursive algorithms.  Follows MuJoCo
    mj_kinematics: body frame = parent * (pos, quat), hinge rotates about
    its axis through jnt_pos, free joint sets the frame from qpos.
    """

    def __init__(self, cm):
        self.cm, self.d = cm, cm.desc

    def forward_position(self, qpos):
        d = self.d
        nb = d.nbody
        self.xpos = np.zeros((nb, 3))
        self.xquat = np.zeros((nb, 4))
        self.xquat[0] = [1, 0, 0, 0]
        self.xmat = np.zeros((nb, 3, 3))
        self.xmat[0] = np.eye(3)
        self.xanchor = np.zeros((d.njnt, 3))
        self.xaxis = np.zeros((d.njnt, 3))
        for b in range(1, nb):
            p = d.body_parentid[b]
            if d.body_jntnum[b] and d.jnt_type[d.body_jntadr[b]] == abi.JNT_FREE:
                ja = d.body_jntadr[b]
                qa = d.jnt_qposadr[ja]
                pos = np.array(qpos[qa:qa + 3], dtype=np.float64)
                quat = quat_normalize(qpos[qa + 3:qa + 7])
                self.xanchor[ja] = pos
                self.xaxis[ja] = [0, 0, 1]
            else:
                pos = self.xpos[p] + self.xmat[p] @ np.array(d.body_pos[b])
                quat = quat_mul(self.xquat[p], np.array(d.body_quat[b]))
                for k in range(d.body_jntnum[b]):
                    j = d.body_jntadr[b] + k
                    R = quat2mat(quat)
                    anchor = R @ np.array(d.jnt_pos[j]) + pos
                    self.xanchor[j] = anchor
                    self.xaxis[j] = R @ np.array(d.jnt_axis[j])
                    qa = d.jnt_qposadr[j]
                    if d.jnt_type[j] == abi.JNT_HINGE:
                        quat = quat_mul(quat, axisangle_quat(np.array(d.jnt_axis[j]), qpos[qa] - d.qpos0[qa]))
                        pos = anchor - quat2mat(quat) @ np.array(d.jnt_pos[j])
                    elif d.jnt_type[j] == abi.JNT_SLIDE:
                        pos = pos + self.xaxis[j] * (qpos[qa] - d.qpos0[qa])
                    else:
                        raise ValueError("ball joints unsupported")
            quat = quat_normalize(quat)
            self.xpos[b], self.xquat[b], self.xmat[b] = pos, quat, quat2mat(quat)
        self.xipos = np.array([self.xpos[b] + self.xmat[b] @ np.array(d.body_ipos[b]) for b in range(nb)])
        self.ximat = np.array([self.xmat[b] @ quat2mat(np.array(d.body_iquat[b])) if b else np.eye(3)
                               for b in range(nb)])
        return self

    def site_xpos(self, s):
        d = self.d
        b = d.site_bodyid[s]
        return self.xpos[b] + self.xmat[b] @ np.array(d.site_pos[s])

    def site_xquat(self, s):
        """site frame orientation (w, x, y, z) = body quaternion * site quaternion"""
        d = self.d
        return quat_normalize(quat_mul(self.xquat[d.site_bodyid[s]], np.array(d.site_quat[s])))

    def geom_pose(self, g):
        d = self.d
        b = d.geom_bodyid[g]
        return (self.xpos[b] + self.xmat[b] @ np.array(d.geom_pos[g]),
                self.xmat[b] @ quat2mat(np.array(d.geom_quat[g])))

    def is_ancestor(self, a, b):
        while b > 0:
            if a == b:
                return True
            b = self.d.body_parentid[b]
        return a == 0

    def jac(self, point, body):
        """World-frame translational / rotational Jacobian (3 x nv each) of a point on `body`."""
        d = self.d
        nv = d.nv
        jp, jr = np.zeros((3, nv)), np.zeros((3, nv))
        for i in range(nv):
            bi = d.dof_bodyid[i]
            if not self.is_ancestor(bi, body):
                continue
            j = d.dof_jntid[i]
            k = i - d.jnt_dofadr[j]
            t = d.jnt_type[j]
            if t == abi.JNT_HINGE:
                ax = self.xaxis[j]
                jr[:, i] = ax
                jp[:, i] = np.cross(ax, point - self.xanchor[j])
            elif t == abi.JNT_SLIDE:
                jp[:, i] = self.xaxis[j]
            elif t == abi.JNT_FREE:
                if k < 3:
                    jp[k, i] = 1.0
                else:
                    ax = self.xmat[bi][:, k - 3]
                    jr[:, i] = ax
                    jp[:, i] = np.cross(ax, point - self.xanchor[j])
        return jp, jr

    def mass_matrix(self):
        d = self.d
        nv = d.nv
        M = np.diag([d.dof_armature[i] for i in range(nv)]).astype(np.float64)
        for b in range(1, d.nbody):
            if d.body_mass[b] == 0:
                continue
            jp, jr = self.jac(self.xipos[b], b)
            R = self.ximat[b]
            I = R @ np.diag(d.body_inertia[b]) @ R.T
            M += d.body_mass[b] * jp.T @ jp + jr.T @ I @ jr
        return M
