#!/usr/bin/env python3
"""Diagnostic: one substep from oracle bench states (contact workload) on the GPU against
the fp64 oracle; prints the error of the arm's and the cube's velocities (max, 99th pct,
median).  SOARM_SIM_LIB selects the library build for A/B comparisons."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from test_gpu_parity import _bench_states, make_sim, load_state, to_np  # noqa: E402

for t in (20, 120):
    cm, orc, st, _ = _bench_states("contact", 1024, t, nthreads=16)
    S = make_sim(cm, 1024)
    st["ncon"][:] = 0
    load_state(S, st)
    S.substeps(1)
    orc.step(st, None, nsub=1)
    err = np.abs(to_np(S.qvel).T - st["qvel"])
    for nm, sl in (("arm", slice(0, 6)), ("cube", slice(6, 12))):
        e = err[:, sl].max(1)
        print(f"t={t} {nm}: max {e.max():.3e} p99 {np.percentile(e, 99):.3e} median {np.median(e):.3e}", flush=True)
