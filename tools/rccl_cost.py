#!/usr/bin/env python3
"""What a live process group costs the step loop, in ONE process on one GPU.

Phases, each timed over the same workload (`--config rollout|contact`, 4096 envs) in windows of
--steps env-steps: no process group; `gloo` group; `nccl` group (eager init with device_id, as
bench.py had it; or lazy with --lazy); after one all_reduce on it; after destroy_process_group.
Per window it also samples every thread of the process (/proc/self/task/*/stat utime+stime), so a
thread that polls while the loop runs shows up by name and CPU share.

    python tools/rccl_cost.py --config rollout --steps 50 --windows 4 [--lazy] [--pin]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def threads():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                s = f.read()
            name = s[s.index("(") + 1:s.rindex(")")]
            f = s[s.rindex(")") + 2:].split()
            out[tid] = (name, int(f[11]) + int(f[12]))
        except (OSError, ValueError):
            pass
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="rollout")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--windows", type=int, default=4)
    p.add_argument("--lazy", action="store_true", help="nccl group without device_id (communicator made at first use)")
    p.add_argument("--pin", action="store_true", help="pin this (launching) thread to its first allowed core")
    p.add_argument("--phases", default="none,gloo,nccl,nccl_used,destroyed")
    p.add_argument("--pg-first", action="store_true",
                   help="init the nccl group (eager, device_id) before the sim and its tensors exist, as bench.py does")
    a = p.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    import soarm_pkg  # noqa: F401
    from lerobot_mujoco_sim2real_amd import shard, workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim

    tick = os.sysconf("SC_CLK_TCK")
    if a.pin:
        cores = sorted(os.sched_getaffinity(0))
        os.sched_setaffinity(0, {cores[0]})
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    if a.pg_first:
        dist.init_process_group("nccl", init_method="env://", device_id=dev)
    cfg = W.CONFIGS[a.config]
    n = cfg.get("envs", 4096)
    ids = np.arange(n)
    cm = W.model(a.config)
    sim = BatchSim(cm, n, 0)
    q0 = W.initial_qpos(cm, ids)
    sim.reset(init_qpos=q0[:, :5], extra_qpos=q0)
    tab = {k: (torch.as_tensor(v, dtype=torch.float32, device=dev) if isinstance(v, np.ndarray) else v)
           for k, v in W.chirp_tables(ids).items()}
    act = sim.action_buffer()
    rollout = cfg["action"] == "ik_fig8"
    phase = torch.as_tensor(W.ik_phase(ids), dtype=torch.float32, device=dev)
    st = {"q": sim.qpos.clone(), "t": 0}

    def step():
        t = st["t"]
        if rollout:
            st["q"], _, _ = sim.ik(W.fig8_targets(float(t % 100), phase, lib=torch), q=st["q"])
            act.copy_(W.ik_action(st["q"][:5].T, sim.obs[:, 3:8], lib=torch))
        else:
            act.copy_(W.chirp_action(tab, float(20 + t % 100), lib=torch))
        sim.step(act)
        st["t"] += 1

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    res = {"config": a.config, "lazy": a.lazy, "pin": a.pin, "phases": {}}
    for ph in a.phases.split(","):
        if ph == "gloo":
            dist.init_process_group("gloo", init_method="env://")
        elif ph == "nccl" and a.pg_first:
            pass
        elif ph == "nccl":
            if dist.is_initialized():
                dist.destroy_process_group()
            if a.lazy:
                dist.init_process_group("nccl", init_method="env://")
            else:
                dist.init_process_group("nccl", init_method="env://", device_id=dev)
        elif ph == "nccl_used":
            x = torch.ones(4, device=dev)
            dist.all_reduce(x)
            rows = torch.zeros((11, n, 13), device=dev)
            shard.gather_rollouts(rows, dst=0)
            torch.cuda.synchronize()
        elif ph == "destroyed":
            dist.destroy_process_group()
        win = []
        cpu = {}
        for _ in range(a.windows):
            th0 = threads()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            th1 = threads()
            win.append(dt / a.steps * 1e3)
            for tid, (name, c1) in th1.items():
                c0 = th0.get(tid, (name, 0))[1]
                share = (c1 - c0) / tick / dt
                if share > 0.02:
                    k = f"{name}:{tid}"
                    cpu[k] = max(cpu.get(k, 0.0), round(share, 3))
        res["phases"][ph] = {"ms_per_step": [round(x, 4) for x in win], "best": round(min(win), 4),
                             "threads_cpu_share": cpu, "nthreads": len(threads())}
        print(ph, res["phases"][ph], file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
