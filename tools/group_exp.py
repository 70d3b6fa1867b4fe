#!/usr/bin/env python3
"""Diagnostic: the contact workload split into G env groups, each its own BatchSim stepped on
its own HIP stream, against one batch of all envs (same envs, same actions).  A launch lasts as
long as its slowest wave; a group's launches wait only for the group's own tail, and the groups
run concurrently on SIMDs the single batch leaves idle.
usage: group_exp.py [G ...]   (env STEPS=a,b windows; default 5-25 and 20-120)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import workloads as W  # noqa: E402
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

n = int(os.environ.get("ENVS", 4096))
cm = W.model("contact")
dev = torch.device("cuda", 0)


def run(G, w0, w1):
    ng = n // G
    sims, tabs, streams = [], [], []
    for g in range(G):
        ids = np.arange(g * ng, (g + 1) * ng)
        s = BatchSim(cm, ng, 0)
        q0 = W.initial_qpos(cm, ids, 0)
        s.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0, env_offset=g * ng)
        sims.append(s)
        tabs.append({k: (torch.as_tensor(v, dtype=torch.float32, device=dev) if isinstance(v, np.ndarray) else v)
                     for k, v in W.chirp_tables(ids, 0).items()})
        streams.append(torch.cuda.Stream(dev) if G > 1 else torch.cuda.current_stream(dev))
    main = torch.cuda.current_stream(dev)

    def step(t):
        ev = torch.cuda.Event()
        ev.record(main)
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                streams[g].wait_event(ev)
                sims[g].step(W.chirp_action(tabs[g], float(t), lib=torch))
        for g in range(G):
            main.wait_stream(streams[g])

    for t in range(w0):
        step(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(w0, w1):
        step(t)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    obs = torch.cat([s.obs for s in sims])
    return n * (w1 - w0) / dt, obs


wins = [tuple(int(x) for x in w.split("-")) for w in os.environ.get("STEPS", "5-25,20-120").split(",")]
Gs = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
for w0, w1 in wins:
    ref = None
    for G in Gs:
        v, obs = run(G, w0, w1)
        same = "" if ref is None else f" obs identical to G={Gs[0]}: {bool(torch.equal(obs, ref))}"
        ref = obs if ref is None else ref
        print(f"steps {w0}-{w1} G={G}: {v / 1e6:.3f} M env-steps/s{same}", flush=True)
