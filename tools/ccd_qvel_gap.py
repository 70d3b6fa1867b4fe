"""One-substep qvel difference between the two narrowphases (MPR vs native GJK/EPA) on the
headline's bench states (fp64 oracle, pick scene, chirp inputs, t = 20 and 120): the physical
effect of the narrowphase choice.  Writes profiles/r04_ccd_qvel_gap.json.
    python tools/ccd_qvel_gap.py [n_envs]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import soarm_pkg  # noqa: F401,E402
from oracle import Oracle  # noqa: E402
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402


def pct(x):
    x = np.asarray(x)
    if not len(x):
        return None
    return {"p50": float(np.median(x)), "p99": float(np.percentile(x, 99)), "max": float(x.max()), "n": int(len(x))}


def main(n=int(sys.argv[1]) if len(sys.argv) > 1 else 2048):
    nt = min(16, os.cpu_count() or 1)
    cms = {c: W.model("contact", ccd=c) for c in ("mpr", "native")}
    orc = {c: Oracle(cm) for c, cm in cms.items()}
    ids = np.arange(n)
    q = W.initial_qpos(cms["mpr"], ids, 0)
    tab = W.chirp_tables(ids, 0)
    res = {"n": n, "workload": "contact (pick scene, chirp), states from the MPR oracle"}
    st = orc["mpr"].new_state(n)
    orc["mpr"].reset(st, init_qpos=q[:, :5], extra_qpos=q)
    t = 0
    names = cms["mpr"].geom_names
    table, cube = names.index("table"), names.index("cube")
    for t_stop in (20, 120):
        while t < t_stop:
            orc["mpr"].step(st, W.chirp_action(tab, t), nthreads=nt)
            t += 1
        out = {}
        for c in ("mpr", "native"):
            s2 = {k: v.copy() for k, v in st.items()}
            orc[c].step(s2, None, nsub=1, nthreads=nt)
            out[c] = s2
        dv = np.abs(out["mpr"]["qvel"] - out["native"]["qvel"])
        arm = np.array([any({int(cc[7]), int(cc[8])} != {table, cube} for cc in
                            orc["mpr"].forward(st["qpos"][i], st["qvel"][i], st["ctrl"][i], st["warm"][i])["contacts"])
                        for i in range(n)])
        res[str(t_stop)] = {"arm_contact_envs": int(arm.sum()),
                            "block_envs": {"cube_qvel": pct(dv[~arm, 6:].max(1)), "arm_qvel": pct(dv[~arm, :6].max(1))},
                            "arm_contact_envs_gap": {"cube_qvel": pct(dv[arm, 6:].max(1)) if arm.any() else None,
                                                     "arm_qvel": pct(dv[arm, :6].max(1)) if arm.any() else None}}
        print(t_stop, json.dumps(res[str(t_stop)]), flush=True)
    json.dump(res, open(os.path.join(ROOT, "profiles", "r04_ccd_qvel_gap.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
