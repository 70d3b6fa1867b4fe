"""MPR vs native GJK/EPA in the fp64 oracle on the contact test poses (arm into the table,
self contacts, cube scene): same contacts?  depth / normal / position distribution of the
differences.  Writes profiles/r04_ccd_mpr_vs_epa.json."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import soarm_pkg  # noqa: F401,E402
from conftest import cube_qpos  # noqa: E402
from oracle import Oracle  # noqa: E402
from lerobot_mujoco_sim2real_amd import mjcf  # noqa: E402

RNG = np.random.default_rng(7)


def poses(n):
    q = np.zeros((n, 6))
    q[:, 0] = RNG.uniform(-1.0, 1.0, n)
    q[:, 1] = RNG.uniform(0.6, 1.6, n)
    q[:, 2] = RNG.uniform(-0.5, 1.0, n)
    q[:, 3] = RNG.uniform(0.3, 1.6, n)
    q[:, 4] = RNG.uniform(-2.0, 2.0, n)
    q[:, 5] = RNG.uniform(0.0, 1.5, n)
    half = n // 2
    q[half:, 1] = RNG.uniform(-1.7, -1.3, n - half)
    q[half:, 2] = RNG.uniform(1.3, 1.69, n - half)
    return q


def main(n=int(sys.argv[1]) if len(sys.argv) > 1 else 1024):
    res = {}
    for name, xml in (("arm_table", mjcf.SCENE_XML), ("pick", mjcf.CUBE_SCENE_XML)):
        cms = {c: mjcf.compile_mjcf(xml, ccd=c) for c in ("mpr", "native")}
        orcs = {c: Oracle(cm) for c, cm in cms.items()}
        q = poses(n)
        cm = cms["mpr"]
        full = cube_qpos(cm, n, RNG, q) if cm.nq > 6 else q
        same = diff = 0
        dd, nn, pp, depths = [], [], [], []
        conv = []  # convex-convex pairs only
        d = cm.desc
        gt = np.array(d.geom_type)
        t = {}
        for c in orcs:
            t0 = time.perf_counter()
            out = [orcs[c].forward(full[e])["contacts"] for e in range(n)]
            t[c] = time.perf_counter() - t0
            res.setdefault(name, {})[f"oracle_s_{c}"] = t[c]
            if c == "mpr":
                A = out
            else:
                B = out
        for e in range(n):
            a, b = A[e], B[e]
            pa = [tuple(map(int, r[7:9])) for r in a]
            pb = [tuple(map(int, r[7:9])) for r in b]
            if pa != pb:
                diff += 1
                continue
            same += 1
            for ra, rb in zip(a, b):
                g1, g2 = int(ra[7]), int(ra[8])
                if gt[g1] in (6, 7) and gt[g2] == 7:
                    dd.append(abs(ra[0] - rb[0]))
                    depths.append(-ra[0])
                    nn.append(np.abs(ra[4:7] - rb[4:7]).max())
                    pp.append(np.abs(ra[1:4] - rb[1:4]).max())
        dd, nn, pp, depths = map(np.array, (dd, nn, pp, depths))
        pct = lambda x: {"p50": float(np.median(x)), "p90": float(np.percentile(x, 90)),  # noqa: E731
                         "p99": float(np.percentile(x, 99)), "max": float(x.max())} if len(x) else None
        sh = depths < 5e-3
        res[name].update({"envs": n, "envs_same_pairs": same, "envs_pair_set_differs": diff,
                          "convex_contacts": int(len(dd)),
                          "depth_absdiff_shallow(<5mm)": pct(dd[sh]), "depth_absdiff_deep": pct(dd[~sh]),
                          "depth_reldiff_deep": pct(dd[~sh] / depths[~sh]) if (~sh).any() else None,
                          "normal_maxabs_diff_shallow": pct(nn[sh]), "normal_maxabs_diff_deep": pct(nn[~sh]),
                          "pos_maxabs_diff": pct(pp)})
        print(name, json.dumps(res[name], indent=1))
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "profiles", "r04_ccd_mpr_vs_epa.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
