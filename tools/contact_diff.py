#!/usr/bin/env python3
"""Diagnostic: GPU contacts vs the oracle on folded / table-penetrating poses;
prints every contact whose normal or depth disagrees (test infrastructure)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from conftest import cube_qpos  # noqa: E402
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402
from oracle import Oracle  # noqa: E402

rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
if len(sys.argv) > 2:  # compare an alternative build of the library
    import ctypes
    from lerobot_mujoco_sim2real_amd import abi

    class _Tolerant(ctypes.CDLL):  # an older build may lack newer diagnostic symbols
        def __getattr__(self, name):
            try:
                return super().__getattr__(name)
            except AttributeError:
                return ctypes.CFUNCTYPE(ctypes.c_int)(lambda *a: -1)

    _load, _cdll = abi.load_lib, abi.C.CDLL
    abi.C.CDLL = _Tolerant
    _alt = _load(os.path.abspath(sys.argv[2]))
    abi.C.CDLL = _cdll
    abi.load_lib = lambda path=None: _alt
n = 2048
for name in ("arm", "cube"):
    cm = W.model("contact") if name == "cube" else W.compile_mjcf(W.SCENE_XML)
    q = np.zeros((n, 6))
    q[:, 0] = rng.uniform(-1.0, 1.0, n)
    q[:, 1] = rng.uniform(0.6, 1.6, n)
    q[:, 2] = rng.uniform(-0.5, 1.0, n)
    q[:, 3] = rng.uniform(0.3, 1.6, n)
    q[:, 4] = rng.uniform(-2.0, 2.0, n)
    q[:, 5] = rng.uniform(0.0, 1.5, n)
    h = n // 2
    q[h:, 1] = rng.uniform(-1.7, -1.3, n - h)
    q[h:, 2] = rng.uniform(1.3, 1.69, n - h)
    full = cube_qpos(cm, n, rng, q) if cm.nq > 6 else q
    full = full.astype(np.float32).astype(np.float64)
    S, orc = BatchSim(cm, n), Oracle(cm)
    S.qpos.copy_(torch.as_tensor(full.T, dtype=torch.float32, device=S.device))
    out, nc = S.contacts()
    out, nc = out.cpu().numpy(), nc.cpu().numpy()
    pid = out.view(np.int32)[..., 7]
    d = cm.desc
    nbad = tot = 0
    for e in range(n):
        rc = orc.forward(full[e])["contacts"]
        if len(rc) != nc[e]:
            gp = [(cm.geom_names[d.pair_geom1[x]], cm.geom_names[d.pair_geom2[x]], round(float(out[e, k, 0]), 6))
                  for k, x in enumerate(pid[e, :nc[e]])]
            op = [(cm.geom_names[int(a)], cm.geom_names[int(b)], round(float(dd), 6)) for dd, a, b in rc[:, [0, 7, 8]]]
            print(name, e, "count", nc[e], len(rc), "gpu-only", [x for x in gp if x[:2] not in [y[:2] for y in op]],
                  "oracle-only", [y for y in op if y[:2] not in [x[:2] for x in gp]], "q", np.round(full[e], 4).tolist())
            continue
        for k in range(nc[e]):
            tot += 1
            dn = np.abs(out[e, k, 4:7] - rc[k, 4:7]).max()
            dd = abs(out[e, k, 0] - rc[k, 0])
            if dn > 2e-2 or dd > 5e-5 + 2e-2 * abs(rc[k, 0]):
                nbad += 1
                p = pid[e, k]
                print(name, e, k, cm.geom_names[d.pair_geom1[p]], cm.geom_names[d.pair_geom2[p]],
                      "depth gpu %.6f orc %.6f" % (out[e, k, 0], rc[k, 0]),
                      "pos", np.round(out[e, k, 1:4], 5), np.round(rc[k, 1:4], 5),
                      "n", np.round(out[e, k, 4:7], 4), np.round(rc[k, 4:7], 4))
    print(name, "contacts", tot, "disagreeing", nbad, flush=True)
