#!/usr/bin/env python3
"""Diagnostic: device contacts vs the oracle on the GPU parity test's contact poses, both convex
narrowphases; for every env whose contact pairs differ (non-grazing), the same qpos through the
CPU backend (the kernels' per-env code on the host, no midphase mask) and the other narrowphase
on the device.  Mismatching qpos go to gpurun_out/ccd_mismatch.npz."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
import test_gpu_parity as T  # noqa: E402
from conftest import cube_qpos  # noqa: E402
from oracle import Oracle  # noqa: E402
from lerobot_mujoco_sim2real_amd import mjcf  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402


def pairs(cm, out, nc, e):
    pid = out.astype(np.float32).view(np.int32)[e, :nc[e], 7]
    return [(int(cm.desc.pair_geom1[x]), int(cm.desc.pair_geom2[x]), round(float(out[e, k, 0]), 6))
            for k, x in enumerate(pid)]


def run(S, full):
    S.qpos.copy_(torch.as_tensor(full.T, dtype=torch.float32, device=S.device))
    out, nc = S.contacts()
    return out.detach().cpu().numpy().astype(np.float64), nc.detach().cpu().numpy().astype(int)


rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 7)
T.RNG = rng
bad = []
for xml in (mjcf.SCENE_XML, mjcf.CUBE_SCENE_XML):
    cms = {c: mjcf.compile_mjcf(xml, ccd=c) for c in ("native", "mpr")}
    n = 2048
    q = T._contact_poses(cms["native"], n)
    full = cube_qpos(cms["native"], n, rng, q) if cms["native"].nq > 6 else q
    full = full.astype(np.float32).astype(np.float64)
    for ccd, cm in cms.items():
        orc = Oracle(cm)
        out, nc = run(BatchSim(cm, n, 0), full)
        mism = []
        for e in range(n):
            rc = orc.forward(full[e])["contacts"]
            if len(rc) and np.min(np.abs(rc[:, 0])) < 2e-5:
                continue
            if nc[e] != len(rc):
                gd = np.abs(out[e, :nc[e], 0]).min() if nc[e] else 1.0
                if gd >= 1e-4:
                    mism.append(e)
                    op = [(int(a), int(b), round(float(r0), 6)) for r0, a, b in zip(rc[:, 0], rc[:, 7], rc[:, 8])]
                    print(os.path.basename(xml), ccd, "env", e, "device", pairs(cm, out, nc, e), "oracle", op)
        print(os.path.basename(xml), ccd, "mismatching envs", len(mism), flush=True)
        if mism:
            sub = full[mism]
            oc, ncc = run(BatchSim(cm, len(mism), -1), sub)
            other = cms["mpr" if ccd == "native" else "native"]
            oo, nco = run(BatchSim(other, len(mism), 0), sub)
            od, ndd = run(BatchSim(cm, len(mism), 0), sub)
            for i, e in enumerate(mism):
                print("  env", e, "cpu backend", pairs(cm, oc, ncc, i), "| device again (alone)", pairs(cm, od, ndd, i),
                      "| device other ccd", pairs(other, oo, nco, i))
            bad.append(sub)
os.makedirs("gpurun_out", exist_ok=True)
if bad:
    np.savez("gpurun_out/ccd_mismatch.npz", *bad)
