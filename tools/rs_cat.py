#!/usr/bin/env python3
"""Diagnostic: one substep of the extra-contact sample (test_one_substep_extra_contact_sweeps) on the
device against the fp64 oracle, qvel error percentiles per contact category (block / arm-only extra /
arm-cube extra / both).  Run once with SOARM_RS=1 and once with SOARM_RS=0."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from test_gpu_parity import _bench_states, make_sim, load_state, to_np  # noqa: E402

nb = 4096
cm, orc, st, _ = _bench_states("contact", nb, 100, nthreads=16)
names = cm.geom_names
table, cube = names.index("table"), names.index("cube")
cat = np.full(nb, "", dtype=object)
for i in range(nb):
    g = [(int(c[7]), int(c[8])) for c in orc.forward(st["qpos"][i], st["qvel"][i], st["ctrl"][i], st["warm"][i])["contacts"]]
    ext = [x for x in g if set(x) != {table, cube}]
    cat[i] = "block" if not ext else ("coupled" if cube in ext[0] else "arm") if len(ext) == 1 else \
        ("both" if len(ext) == 2 and cube not in ext[0] else "other")
sub = {k: v.copy() for k, v in st.items()}
S = make_sim(cm, nb)
sub["ncon"][:] = 0
load_state(S, sub)
S.substeps(1)
orc.step(sub, None, nsub=1, nthreads=16)
dv = np.abs(to_np(S.qvel).T - sub["qvel"]).max(1)
print("SOARM_RS", os.environ.get("SOARM_RS", "1"))
for k in ("block", "arm", "coupled", "both", "other"):
    e = dv[cat == k]
    if len(e):
        w = np.nonzero(cat == k)[0][np.argmax(e)]
        print(f"{k:8s} n {len(e):5d} p50 {np.median(e):.2e} p99 {np.percentile(e, 99):.2e} max {e.max():.2e} (env {w})")
