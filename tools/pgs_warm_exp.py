#!/usr/bin/env python3
"""Experiment: PGS warm-started from the previous substep's forces vs mj_solPGS's warm start
(forces implied by qacc_warmstart), on the headline workload (pick scene, chirp), oracle fp64.
Reports PGS sweeps per substep and the gap of each substep's PGS qacc to the exact optimum of
the same constraint problem (Newton, tolerance 0) over env-step windows.

    python tools/pgs_warm_exp.py [--n 512 --T 120]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import soarm_pkg  # noqa: E402,F401
import oracle as O  # noqa: E402
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402


def run(cm, n, T, mode, nthreads=8, seed=0):
    orc = O.Oracle(cm)
    ids = np.arange(n)
    st = orc.new_state(n)
    q = W.initial_qpos(cm, ids, seed)
    orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
    tab = W.chirp_tables(ids, seed)
    acts = np.ascontiguousarray(np.stack([W.chirp_action(tab, t) for t in range(T)]), np.float64)
    L = O.lib()
    vp = C.c_void_p
    L.orc_experiment_pgs.argtypes = [vp] * 4 + [C.c_int] + [vp] * 4 + [C.c_int] * 4 + [vp] * 3
    L.orc_experiment_pgs.restype = None
    sw = np.zeros((T, n))
    gap = np.zeros((T, n, 2))
    qo = np.zeros((n, cm.desc.nq))
    L.orc_experiment_pgs(orc._desc_p, O._p(orc.hv), O._p(orc.hadr), O._p(orc.hadj), n, O._p(st["qpos"]),
                         O._p(st["qvel"]), O._p(st["warm"]), O._p(acts), T, 10, mode, nthreads, O._p(sw),
                         O._p(gap), O._p(qo))
    return sw, gap


def summary(sw, gap, lo, hi):
    g = gap[lo:hi]
    return {"sweeps_mean": float(sw[lo:hi].mean()), "sweeps_max_env_mean": float(sw[lo:hi].mean(0).max()),
            "qacc_gap_free": {"p50": float(np.median(g[..., 1])), "p99": float(np.percentile(g[..., 1], 99)),
                              "max": float(g[..., 1].max())},
            "qacc_gap_arm": {"p50": float(np.median(g[..., 0])), "p99": float(np.percentile(g[..., 0], 99)),
                             "max": float(g[..., 0].max())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--T", type=int, default=120)
    a = ap.parse_args()
    cm = W.model("contact")
    out = {}
    for mode, name in ((0, "mj_solPGS warm start (qacc_warmstart)"), (1, "previous forces")):
        sw, gap = run(cm, a.n, a.T, mode)
        out[name] = {"steps 5-25": summary(sw, gap, 5, 25), "steps 20-120": summary(sw, gap, 20, a.T)}
        print(name, json.dumps(out[name]), flush=True)


if __name__ == "__main__":
    main()
