"""Build the committed model assets from the reference robot description.

Run once in the build container (the GPU box has no /root/reference):

    python tools/build_assets.py [/root/reference]

It copies the two MJCF data files the hot path loads
(``SOARM101/SO101/scene_with_table_v.xml`` selected at ``args.py:91`` and the
``so101_new_calib_v.xml`` it includes at ``scene_with_table_v.xml:4``) and
reduces each binary STL collision mesh to its convex hull (the geometry MuJoCo
collides against for ``type="mesh"`` geoms) plus the hull's vertex adjacency
graph (used for hill-climbing support queries).  The STLs themselves (~17 MB)
are not committed; ``hulls.npz`` holds, per mesh name:

* ``<name>/v``    float32 [n, 3]  hull vertices in the mesh file's own frame
* ``<name>/adj``  int32   [k]     concatenated neighbour lists (local indices)
* ``<name>/adr``  int32   [n+1]   CSR offsets into ``adj``
* ``<name>/com``  float64 [3]     volume centroid of the mesh (MuJoCo re-centres
  mesh geoms on it; the geom "centre" used by MPR and the bounding sphere)
"""
import os
import shutil
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd.mjcf import hull_with_graph  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "lerobot-mujoco-sim2real_amd", "assets", "so101")
# the hot path's scene (velocity servos) and, for the position-servo scenes the viewer /
# sim2real scripts load, scene_with_table.xml + scene.xml
XMLS = ["scene_with_table_v.xml", "so101_new_calib_v.xml", "scene_with_table.xml", "so101_new_calib.xml",
        "scene.xml", "so101_old_calib.xml"]


def read_stl(path):
    raw = open(path, "rb").read()
    n = int(np.frombuffer(raw[80:84], dtype="<u4")[0])
    if 84 + 50 * n != len(raw):
        raise ValueError(f"{path}: not a binary STL")
    dt = np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")])
    tri = np.frombuffer(raw[84:84 + 50 * n], dtype=dt)
    return tri["v"].reshape(-1, 3)


def volume_centroid(tri):
    """Centroid of the closed triangle mesh by signed tetrahedra (origin apex)."""
    a, b, c = (tri[:, k].astype(np.float64) for k in range(3))
    vol = np.einsum("ij,ij->i", a, np.cross(b, c)) / 6.0
    return (vol[:, None] * (a + b + c) / 4.0).sum(0) / vol.sum()


def main(ref_root, xml_only=False):
    src = os.path.join(ref_root, "SOARM101", "SO101")
    os.makedirs(OUT, exist_ok=True)
    for x in XMLS:
        shutil.copyfile(os.path.join(src, x), os.path.join(OUT, x))
    if xml_only:
        return
    arrays = {}
    for f in sorted(os.listdir(os.path.join(src, "assets"))):
        if not f.endswith(".stl"):
            continue
        name = f[:-4]
        tri = read_stl(os.path.join(src, "assets", f)).reshape(-1, 3, 3)
        v, adj, adr = hull_with_graph(tri.reshape(-1, 3))
        arrays[f"{name}/com"] = volume_centroid(tri)
        arrays[f"{name}/v"] = v
        arrays[f"{name}/adj"] = adj
        arrays[f"{name}/adr"] = adr
        print(f"{name:40s} hull verts {len(v):5d}  edges {len(adj) // 2:6d}")
    np.savez_compressed(os.path.join(OUT, "hulls.npz"), **arrays)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0] if args else "/root/reference", xml_only="--xml-only" in sys.argv)
