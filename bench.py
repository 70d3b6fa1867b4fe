#!/usr/bin/env python3
"""bench.py — SO-ARM101 batched simulation throughput on MI355X.

Headline (BASELINE.json ``metric``): env-steps/sec (whole node) at 4096
SO-ARM101 envs per GPU with contacts (config 3: the build-defined pick scene,
table + cube, PGS, chirp actions).  One step = one ``SOARM101Env.step()`` for
every env = 10 physics substeps of 2 ms (``SOARM101_Env.py:39-40,131-132``).

    python bench.py [--gpus N --steps K --warmup W --config contact|nocontact|dr|rollout|mpc|mpc_dbkn|plumbing]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; envs shard by global env id (rank r owns
[r*n, (r+1)*n)), there is no per-step collective (``scaling: weak``); the
timed region is bracketed by barrier + synchronize and the max over ranks is
used.  Rank 0 prints one JSON line.  ``--gpus N`` without a torchrun
environment starts the N rank processes itself (before any GPU call) and exits
with their status; under torchrun, ``--gpus`` must equal WORLD_SIZE.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node), 4096 SO-ARM101 envs w/ contacts, 1/2/4/8 MI355X"
PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 vector (= FP32 MFMA) dense peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (default 4096; 8192 for dr)")
    p.add_argument("--config", default="contact",
                   choices=["contact", "nocontact", "dr", "rollout", "mpc", "mpc_dbkn", "plumbing"])
    p.add_argument("--dist-backend", default=None,
                   help="nccl (= RCCL; the default for --gpus > 1) or gloo (rehearsal on one GPU); given with "
                        "--gpus 1 it initialises a one-rank process group, so the rollout gather runs through it")
    p.add_argument("--solver", default="pgs", choices=["pgs", "newton"],
                   help="constraint solver: PGS (BASELINE config 3) or MuJoCo's default Newton")
    p.add_argument("--ccd", default="mpr", choices=["native", "mpr"],
                   help="convex-convex narrowphase: MuJoCo's native GJK/EPA or libccd MPR")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-profile", action="store_true")
    p.add_argument("--no-steady", action="store_true", help="skip the steps 20-120 steady-state window")
    p.add_argument("--no-other-solver", action="store_true",
                   help="skip timing the same workload with the other constraint solver (contact configs)")
    p.add_argument("--launcher-check", action="store_true",
                   help="exercise the rank launcher / process group / max-over-ranks timing with an empty "
                        "timed region (no GPU; CPU tests)")
    return p.parse_args()


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(args):
    """`--gpus N` without a torchrun environment: start N rank processes of this script (one per
    GPU) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, wait, return the worst exit status.
    Called before anything touches the GPU (this process never initialises HIP)."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   SOARM_BENCH_LAUNCHER="bench.py --gpus")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # a rank that fails leaves the others blocked in a collective: stop them (these exact
    # child processes) once one exits with an error
    import time as _t
    rcs = [None] * len(procs)
    while any(rc is None for rc in rcs):
        for i, pr in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = pr.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, pr in enumerate(procs):
                if rcs[i] is None:
                    pr.terminate()
                    try:
                        rcs[i] = pr.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        pr.kill()
                        rcs[i] = pr.wait()
            break
        _t.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def cpu_backend_leg(cm, cfg, seed, n, T, threads, t0=2, min_s=0.0):
    """The library's own CPU backend (sim_batch_create(..., -1, ...): the kernels' per-env code
    compiled for the host, fp32) on `threads` host threads: n envs x T env-steps of the workload
    after t0 untimed env-steps (the steady window: t0 = 20, T = 100), repeated from the reset
    until at least min_s seconds are timed.  A measured side line, not the bench's cpu_baseline
    (the oracle)."""
    import numpy as np
    from lerobot_mujoco_sim2real_amd import workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    old = os.environ.get("SOARM_CPU_THREADS")
    os.environ["SOARM_CPU_THREADS"] = str(threads)
    try:
        ids = np.arange(n)
        S = BatchSim(cm, n, -1)
        q = W.initial_qpos(cm, ids, seed)
        S.reset(init_qpos=q[:, :5], extra_qpos=q, seed=seed)
        tab = W.chirp_tables(ids, seed)
        if cfg["dr"]:
            S.set_params(**W.dr_params(ids, seed))
        rng = np.random.default_rng(seed)
        acts = [np.zeros((n, 5), np.float32) if cfg["action"] == "zero" else
                W.chirp_action(tab, t).astype(np.float32) if cfg["action"] == "chirp" else
                rng.uniform(-0.5, 0.5, (n, 5)).astype(np.float32) for t in range(T + t0)]
        dt, reps = 0.0, 0
        while reps == 0 or dt < min_s:
            if reps:
                S.reset(init_qpos=q[:, :5], extra_qpos=q, seed=seed)
            for t in range(t0):
                S.step(acts[t])
            ts = time.perf_counter()
            for t in range(t0, T + t0):
                S.step(acts[t])
            dt += time.perf_counter() - ts
            reps += 1
        S.close()
    finally:
        if old is None:
            os.environ.pop("SOARM_CPU_THREADS", None)
        else:
            os.environ["SOARM_CPU_THREADS"] = old
    return {"value": reps * n * T / dt, "unit": "env-steps/s", "threads": threads, "dtype": "f32",
            "sample": f"{reps} x {n} envs x env-steps {t0}-{t0 + T} of the library's CPU backend (device = -1), "
                      f"{dt:.2f} s timed"}


def cpu_baseline(cfg_name, seconds, seed, solver="pgs", ccd="mpr"):
    """The float64 oracle (C restatement of mj_step; for `mpc` plus the numpy MPC restatement)
    on the host cores, a bounded sample of the same workload: chunks of envs x T env-steps."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    from oracle import Oracle
    from lerobot_mujoco_sim2real_amd import workloads as W

    cfg = W.CONFIGS[cfg_name]
    cm = W.model(cfg_name, solver=solver, ccd=ccd)
    orc = Oracle(cm)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    # the GPU box gives a job a 16-CPU share (OMP_NUM_THREADS=16 there) whatever the affinity
    # mask shows: at most 16 threads
    cores = max(1, min(affinity, 16))
    mpc = None
    # the sampled window: the steady window of the GPU line (env-steps 20-120: chunks start from the
    # oracle's own states at t = 20, reached untimed); the Koopman-MPC configs: 10 frames from the reset
    T0, T = (0, 10) if cfg["action"] == "koopman_mpc" else (20, 100)
    if cfg["action"] == "koopman_mpc":
        import koopman_mpc as KO
        net, _ = _mpc_net(seed, cfg.get("koopman", "DKUC"))
        A, B = net.lA.weight.detach().numpy(), net.lB.weight.detach().numpy()
        Hhat = net.get_Hi_numpy() if hasattr(net, "get_Hi_numpy") else None
        mpc = (KO, A, B, net.encoder_layers(), KO.prepare(A, B), Hhat)

    def run_chunk(ids, nthreads):
        n = len(ids)
        st = orc.new_state(n)
        q = W.initial_qpos(cm, ids, seed)
        orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
        tab = W.chirp_tables(ids, seed)
        prm = None
        if cfg["dr"]:
            p = W.dr_params(ids, seed)
            prm = np.stack([p["mass_scale"], p["friction"], p["damping_scale"]], 1).astype(np.float64)
        rng = np.random.default_rng(int(ids[0]))
        phase = W.ik_phase(ids, seed)
        qstar = q.astype(np.float64)
        if mpc:  # Koopman_MPC.py loop on the oracle (joint refs: the start pose)
            KO, A, B, layers, qp, Hhat = mpc
            cart = np.stack([W.fig8_targets(t - 1.0, phase) for t in range(T)])
            sref = np.concatenate([cart, np.repeat(q[None, :, :5].astype(np.float64), T, 0)], -1)
            zref = KO.encode(layers, sref.reshape(T * n, 8)).reshape(T, n, -1)
            x, up = sref[0], np.zeros((n, 5))
        ts = None
        for t in range(T0 + T):
            if t == T0:
                ts = time.perf_counter()
            if mpc:
                if Hhat is None:
                    up, a = KO.get_control(A, B, KO.encode(layers, x), KO.lifted_window(zref, t, 10), up, qp=qp)
                else:
                    up, a = KO.get_control_bilinear(A, B, Hhat, KO.encode(layers, x), KO.lifted_window(zref, t, 10), up)
                x = orc.step(st, a, nthreads=nthreads, applied=orc.bias(st)).astype(np.float32).astype(np.float64)
                continue
            if cfg["action"] == "chirp":
                a = W.chirp_action(tab, t)
            elif cfg["action"] == "ik_fig8":
                qstar, _, _ = orc.ik(W.fig8_targets(t, phase), qstar)
                a = W.ik_action(qstar[:, :5], st["qpos"][:, :5])
            else:
                a = rng.uniform(-0.5, 0.5, (n, 5))
            orc.step(st, a, params=prm, nthreads=nthreads)
        return n * T, time.perf_counter() - ts

    if cfg_name == "plumbing":  # config 1: one env, zero action, 1000 env-steps on one core
        t0 = time.perf_counter()
        st = orc.new_state(1)
        q = W.initial_qpos(cm, np.arange(1), seed)
        orc.reset(st, init_qpos=q[:, :5], extra_qpos=q)
        for _ in range(1000):
            orc.step(st, np.zeros((1, 5)), nthreads=1)
        dt = time.perf_counter() - t0
        return {"value": 1000 / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
                "sample": f"1 env x 1000 env-steps (zero action) of the float64 C oracle on 1 thread, {dt:.2f} s",
                "nproc": os.cpu_count(), "fp32_cpu_backend": cpu_backend_leg(cm, cfg, seed, 1, 1000, 1)}
    n = 256
    done, chunk, dt, tw = 0, 0, 0.0, time.perf_counter()
    while chunk == 0 or time.perf_counter() - tw < seconds:
        k, d = run_chunk(np.arange(chunk * n, (chunk + 1) * n), cores)
        done, dt, chunk = done + k, dt + d, chunk + 1
    # every core of the affinity mask (SURVEY 8d "all host cores"), beside the 16-thread value: on the
    # GPU box the mask shows the whole machine (256) while the job's CPU share is 16, so this leg
    # oversubscribes it -- a shorter sample of 256-env chunks, one env per thread at 256
    da, ca, ta, tw = 0, 0, 0.0, time.perf_counter()
    while ca == 0 or time.perf_counter() - tw < max(1.0, seconds / 4):
        k, d = run_chunk(np.arange(ca * n, (ca + 1) * n), max(1, affinity))
        da, ta, ca = da + k, ta + d, ca + 1
    # the same workload on ONE core (SURVEY 8d asks for both), a shorter sample of 32-env chunks
    d1, c1, t1, tw = 0, 0, 0.0, time.perf_counter()
    while c1 == 0 or time.perf_counter() - tw < max(1.0, seconds / 4):
        k, d = run_chunk(np.arange(c1 * 32, (c1 + 1) * 32), 1)
        d1, t1, c1 = d1 + k, t1 + d, c1 + 1
    cpu_name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_name = next(ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    import importlib.util
    mj = "available (not used)" if importlib.util.find_spec("mujoco") else "MuJoCo unavailable"
    what = "float64 C oracle" + (" + numpy MPC restatement" if mpc else "")
    fp32 = None
    if cfg["action"] in ("chirp", "random"):  # the library's CPU backend on the same workload
        fp32 = cpu_backend_leg(cm, cfg, seed, 512, T, cores, t0=T0, min_s=1.0)
        fp32["single_core"] = cpu_backend_leg(cm, cfg, seed, 32, T, 1, t0=T0, min_s=1.0)
    return {"value": done / dt, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "fp32_cpu_backend": fp32,
            "sample": f"{done} env-steps ({chunk} chunks of {n} envs x env-steps {T0}-{T0 + T}, {cfg_name} "
                      f"workload, each chunk from the oracle's own states at t = {T0}) of the {what}, "
                      f"threads over envs, {dt:.1f} s timed",
            "single_core": {"value": d1 / t1, "sample": f"{d1} env-steps ({c1} chunks of 32 envs x env-steps "
                                                         f"{T0}-{T0 + T}) on 1 thread, {t1:.1f} s timed"},
            "all_affinity_cores": {"value": da / ta, "threads": max(1, affinity),
                                   "sample": f"{da} env-steps ({ca} chunks of {n} envs x env-steps {T0}-{T0 + T}) on "
                                             f"{max(1, affinity)} threads, {ta:.1f} s timed"},
            "affinity_cores": affinity, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cpu_model": cpu_name, "nproc": os.cpu_count(), "mujoco": mj}


def _mpc_net(seed, kind="DKUC"):
    """Random-init Koopman model of the reference's architecture (control/koopman.py): DKUC, or
    DBKN with its bilinear layer drawn N(0, 0.02^2) (the reference zero-initialises it, which
    would make the bilinear MPC the linear one)."""
    import torch
    from lerobot_mujoco_sim2real_amd.args import Args
    from lerobot_mujoco_sim2real_amd.control.koopman import init_model
    torch.manual_seed(seed)
    a = Args(["--model", kind])
    net = init_model(a).double()
    if kind == "DBKN":
        with torch.no_grad():
            net.H.weight.normal_(0.0, 0.02)
    return net, a


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    launcher = os.environ.get("SOARM_BENCH_LAUNCHER", "torchrun" if world > 1 else "single process")
    import numpy as np
    import torch
    import torch.distributed as dist

    if args.launcher_check:
        return launcher_check(args, rank, world, launcher)

    import soarm_pkg  # noqa: F401
    from lerobot_mujoco_sim2real_amd import build, shard, workloads as W
    from lerobot_mujoco_sim2real_amd.sim import BatchSim

    build.ensure_built(local)
    gpu = local % max(torch.cuda.device_count(), 1)  # > 1 rank per GPU only in gloo rehearsals
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    backend = args.dist_backend or "nccl"
    use_pg = world > 1 or args.dist_backend is not None  # one rank: only when asked (the RCCL path on one GPU)
    if use_pg:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", init_method="env://", device_id=dev)
        else:
            dist.init_process_group(backend, init_method="env://")
        if dist.get_world_size() != args.gpus:
            print(f"bench: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}", file=sys.stderr)
            sys.exit(2)

    name = args.config
    cfg = W.CONFIGS[name]
    n = args.envs or cfg.get("envs", 4096)
    ids = np.arange(rank * n, (rank + 1) * n)
    cm = W.model(name, solver=args.solver, ccd=args.ccd)
    sim = BatchSim(cm, n, gpu)
    q0 = W.initial_qpos(cm, ids, args.seed)
    sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=args.seed, env_offset=rank * n)
    if cfg["dr"]:
        sim.set_params(**W.dr_params(ids, args.seed))
    tab = {k: (torch.as_tensor(v, dtype=torch.float32, device=dev) if isinstance(v, np.ndarray) else v)
           for k, v in W.chirp_tables(ids, args.seed).items()}
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed * 1000003 + rank)
    act = sim.action_buffer()  # the step reads its action from here (stable address: graph replay)
    # the synthetic input streams (chirp / random actions) of every step the run touches -- the
    # timed window, its profiled replay, the steady window -- are generated before any timing and
    # stay resident in HBM; a step then stages its row into the action buffer (one copy)
    acts = None
    if cfg["action"] in ("chirp", "random"):
        t_in = max(args.warmup + args.steps, 120)
        if cfg["action"] == "chirp":
            acts = torch.stack([W.chirp_action(tab, float(t), lib=torch) for t in range(t_in)]).contiguous()
        else:
            acts = torch.rand((t_in, n, 5), generator=gen, device=dev) - 0.5

    mpc = cfg["action"] == "koopman_mpc"
    if mpc:
        # Koopman_MPC.py loop for every env: Fig8 reference per env (warm-started DLS IK for
        # its joint angles), lifted and turned into per-frame feedforward once, then per frame
        # sim_bias -> qfrc_applied, k_mpc_step, sim_step (all on device)
        from lerobot_mujoco_sim2real_amd.control.MPC_Controler import MPCController
        from lerobot_mujoco_sim2real_amd.Koopman_MPC import KoopmanMPCTracking
        net, margs = _mpc_net(args.seed, cfg.get("koopman", "DKUC"))
        ctl = MPCController(net, margs, device=gpu)
        phase = torch.as_tensor(W.ik_phase(ids, args.seed), dtype=torch.float32, device=dev)
        cart, jq = W.reference_trajectory(sim, phase, args.warmup + args.steps)
        run = KoopmanMPCTracking(ctl, cm, cart, jq, device=gpu, sim=sim)
        run.runBefore()

    rollout = cfg["action"] == "ik_fig8"
    qstar = None
    if rollout:
        # config 5: DLS-IK toward each env's Fig8 target, action = clip((q* - q)/dt), rows
        # [u | obs] recorded on device for every timed step, gathered to rank 0 at the end
        phase = torch.as_tensor(W.ik_phase(ids, args.seed), dtype=torch.float32, device=dev)
        qstar = sim.qpos.clone()
        rows = torch.empty((args.steps + 1, n, 13), dtype=torch.float32, device=dev)
    rec = {"i": -1}

    def one_step(t):
        nonlocal qstar
        if mpc:
            run.runFunc()
            return
        if rollout:
            qstar, _, _ = sim.ik(W.fig8_targets(float(t), phase, lib=torch), q=qstar)
            act.copy_(W.ik_action(qstar[:5].T, sim.obs[:, 3:8], lib=torch))
        elif acts is not None and t < acts.shape[0]:
            act.copy_(acts[t])
        elif cfg["action"] == "chirp":
            act.copy_(W.chirp_action(tab, float(t), lib=torch))
        elif cfg["action"] == "zero":
            act.zero_()
        else:
            torch.rand((n, 5), generator=gen, device=dev, out=act)
            act.sub_(0.5)
        obs = sim.step(act)
        if rollout and rec["i"] >= 0:
            rows[rec["i"], :, :5] = act
            rows[rec["i"] + 1, :, 5:] = obs
            rec["i"] += 1

    def snapshot():
        """Everything the step loop reads; restore() replays from this point exactly."""
        st = [x.clone() for x in (sim.qpos, sim.qvel, sim.qacc_warmstart, sim.ctrl, sim.status, sim.obs)]
        g = gen.get_state()
        qs = qstar.clone() if rollout else None
        mp_ = (run.u_prev.clone(), run.traj_index, run.state is sim.obs) if mpc else None

        def restore():
            nonlocal qstar
            for dst, src in zip((sim.qpos, sim.qvel, sim.qacc_warmstart, sim.ctrl, sim.status, sim.obs), st):
                dst.copy_(src)
            gen.set_state(g)
            if rollout:
                qstar = qs.clone()
            if mpc:
                run.u_prev.copy_(mp_[0])
                run.traj_index = mp_[1]
                run.state = sim.obs if mp_[2] else run.state_all_ref[0]
        return restore

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def max_over_ranks(*vals):
        if world == 1:
            return vals
        x = torch.tensor(vals, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        return tuple(float(v) for v in x)

    def sum_over_ranks(*vals):
        if world == 1:
            return vals
        x = torch.tensor(vals, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
        return tuple(float(v) for v in x)

    restore_t0 = snapshot()
    t = 0
    for _ in range(args.warmup):
        one_step(t)
        t += 1
    sim.ncon.zero_()
    snap_t, restore_timed = t, snapshot()
    sync()
    t0 = time.perf_counter()
    if rollout:
        rows[0, :, 5:] = sim.obs
        rec["i"] = 0
    for _ in range(args.steps):
        one_step(t)
        t += 1
    gather_s, gather_exact = None, None
    if rollout:
        rec["i"] = -1
        if use_pg:  # rollout rows of every rank to rank 0 (RCCL gather over xGMI)
            torch.cuda.synchronize()
            tg = time.perf_counter()
            got = shard.gather_rollouts(rows if backend == "nccl" else rows.cpu(), dst=0)
            torch.cuda.synchronize()
            gather_s = time.perf_counter() - tg
    sync()
    dt = time.perf_counter() - t0
    if rollout and use_pg and world == 1:
        # one rank: the gathered rows are this rank's, bit for bit (checked after the clock stops: the
        # first torch.equal of a run loads its kernels, ~20 ms, which r05 timed as "RCCL overhead")
        gather_exact = bool(torch.equal(got.to(rows.device), rows))
    (dt,) = max_over_ranks(dt)
    if gather_s is not None:
        (gather_s,) = max_over_ranks(gather_s)
    (ncon,) = sum_over_ranks(float(sim.ncon.sum().item()))
    # validity of what was timed: states finite, soft resets (mj_checkPos/Vel/Acc status bits) counted
    finite = bool(torch.isfinite(sim.obs).all() and torch.isfinite(sim.qpos).all() and torch.isfinite(sim.qvel).all())
    nbad = int((sim.status != 0).sum().item())
    nonfinite, nbad = sum_over_ranks(0.0 if finite else 1.0, float(nbad))
    finite, nbad = nonfinite == 0, int(nbad)
    total_envs = n * world
    value = total_envs * args.steps / dt
    contacts = ncon / (total_envs * args.steps * 10)

    # dominant kernel: HIP events (on the sim's stream) around every launch of a replay of
    # the timed region -- state, action stream and step index restored from the snapshot
    roof = None
    costs = json.load(open(os.path.join(ROOT, "profiles", "algorithmic_cost.json")))
    base = name if name in costs else "mpc"  # (mpc_dbkn: the same physics per env-step as mpc)
    cost = costs.get(name if args.solver == "pgs" else f"{name}_newton", costs[base])
    if not args.no_profile:
        kp = args.steps
        restore_timed()
        t = snap_t
        sync()
        sim.profile_begin()
        for _ in range(kp):
            one_step(t)
            t += 1
        prof = sim.profile_end()
        kind, (ms, cnt) = max(prof.items(), key=lambda kv: kv[1][0])
        avg_ms = ms / max(cnt, 1)
        per_launch = {"step_fused": cost["flops_per_env_step"],
                      "collide": cost["flops_per_env_substep_collision"],
                      "substep": cost["flops_per_env_substep_dynamics"],
                      "geom": 0.0}[kind] * n
        achieved = per_launch / (avg_ms * 1e-3) / 1e12
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tpath):
            tr = json.load(open(tpath))
            key = name if args.solver == "pgs" else f"{name}_newton"
            key = f"{name}_native" if args.ccd == "native" and args.solver == "pgs" else key
            traffic = tr.get(key, {}).get(kind)
        # 64-lane waves, one lane per env (k_substep: four per env in quad mode, soarm_pgs.h lpe();
        # sixteen in the row-space PGS kernel, which the library runs for PGS on the free-body scene
        # up to 4 envs per SIMD, soarm_sim.hip rs_cap): the kernel can occupy at most that many of
        # the chip's 1024 SIMDs; the VALU peak those SIMDs can issue bounds it first
        rs = (kind == "substep" and args.solver == "pgs" and sim.nv == 12 and  # (arm + one free body)
              os.environ.get("SOARM_RS", "1") != "0" and
              n <= 16 * torch.cuda.get_device_properties(dev).multi_processor_count)
        lanes = (16 if rs else 4) if kind == "substep" else 1
        waves = -(-n * lanes // 64)
        capped = PEAK_FP32_TFLOPS * min(1.0, waves / 1024)
        roof = {"bound": "valu", "achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP32_TFLOPS, "traffic": traffic,
                "traffic_source": ("copied from profiles/pmc_traffic.json (rocprofv3 PMC passes of this "
                                   "workload, guide-corrected); not measured in this run") if traffic else None,
                "lanes_per_env": lanes, "waves_per_launch": waves, "occupancy_capped_peak": capped,
                "frac_of_capped": achieved / capped,
                "kernel": kind, "avg_launch_ms": avg_ms, "launches": cnt,
                "flops_per_launch": per_launch,
                "kernel_ms_per_step": {k: v[0] / kp for k, v in prof.items()},
                "hbm_gbs_algorithmic": cost["hbm_bytes_per_env_step"] * n * world / (dt / args.steps) / 1e9,
                "hbm_peak_gbs": PEAK_HBM_GBS,
                "note": "bound = FP32 VALU (per-env 6x6 / 12-dof algebra, no MFMA, HBM < 0.1% of peak); "
                        "peak = MI355X FP32 vector rate; the kernel is latency-bound on each env's "
                        "Gauss-Seidel chain (DESIGN.md §4)"}

    # steady state: the same workload timed over env-steps 20..120 (from the reset), the window
    # where arm-cube / arm-table contacts are present (the driver's short window is not)
    steady = None
    if not args.no_steady and not (rollout or mpc) and (args.warmup, args.steps) != (20, 100):
        restore_t0()
        t = 0
        for _ in range(20):
            one_step(t)
            t += 1
        sync()
        ts = time.perf_counter()
        for _ in range(100):
            one_step(t)
            t += 1
        sync()
        (dts,) = max_over_ranks(time.perf_counter() - ts)
        steady = {"window": "env-steps 20-120", "value": total_envs * 100 / dts, "ms_per_step": dts / 100 * 1e3}
    elif (args.warmup, args.steps) == (20, 100):
        steady = {"window": "env-steps 20-120", "value": value, "ms_per_step": dt / args.steps * 1e3,
                  "note": "= the timed window"}

    # the other constraint solver on the same workload (contact configs): PGS is the configured
    # solver (BASELINE.json configs[2]); Newton is what the reference's MuJoCo runs by default
    # (its scene has no <option>), so both numbers are reported -- value is always --solver's
    other_solver = None
    if not args.no_other_solver and name in ("contact", "dr"):
        other = "newton" if args.solver == "pgs" else "pgs"
        cm2 = W.model(name, solver=other, ccd=args.ccd)
        sim2 = BatchSim(cm2, n, gpu)
        sim2.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=args.seed, env_offset=rank * n)
        if cfg["dr"]:
            sim2.set_params(**W.dr_params(ids, args.seed))
        act2 = sim2.action_buffer()
        gen2 = torch.Generator(device=dev)
        gen2.manual_seed(args.seed * 1000003 + rank)

        def step2(t):
            if acts is not None and t < acts.shape[0]:
                act2.copy_(acts[t])
            elif cfg["action"] == "chirp":
                act2.copy_(W.chirp_action(tab, float(t), lib=torch))
            else:
                torch.rand((n, 5), generator=gen2, device=dev, out=act2)
                act2.sub_(0.5)
            sim2.step(act2)

        windows = [(args.warmup, args.steps)] + ([(20, 100)] if steady is not None and (args.warmup, args.steps) != (20, 100) else [])
        res = {}
        t = 0
        for w0, ns in windows:
            while t < w0:
                step2(t)
                t += 1
            if t > w0:  # the second window starts before the first ended: replay from the reset
                sim2.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=args.seed, env_offset=rank * n)
                gen2.manual_seed(args.seed * 1000003 + rank)
                t = 0
                while t < w0:
                    step2(t)
                    t += 1
            sync()
            ts = time.perf_counter()
            for _ in range(ns):
                step2(t)
                t += 1
            sync()
            (dto,) = max_over_ranks(time.perf_counter() - ts)
            res[f"env-steps {w0}-{w0 + ns}"] = {"value": total_envs * ns / dto, "ms_per_step": dto / ns * 1e3}
        other_solver = {"solver": other, "windows": res}
        del sim2, cm2

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(name, args.cpu_seconds, args.seed, args.solver, args.ccd)

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (Philox-keyed initial states / chirp inputs per global env id)",
            "config": {"workload": (cfg["desc"] if args.solver == "pgs" else
                                    cfg["desc"].replace("PGS (config 3", "Newton (config 3 scene")),
                       "config": name, "envs_per_gpu": n, "global_envs": total_envs,
                       "frame_skip": 10, "substeps_per_s": value * 10,
                       "contacts_per_env_substep": contacts,
                       "solver": ("PGS (iterations 100, tol 1e-8, scale 1/(meaninertia nv))" if args.solver == "pgs"
                                  else "Newton (MuJoCo's default: iterations 100, tol 1e-8, exact line search)"),
                       "narrowphase": ("native GJK/EPA (MuJoCo nativeccd)" if args.ccd == "native"
                                       else "MPR (libccd)"),
                       "parallelism": f"env-sharded x{world} (no per-step collective)"},
            "steady_state": steady,
            "other_solver": other_solver,
            "dist": {"world_size": world, "backend": (backend if use_pg else None),
                     "launcher": launcher, "rollout_gather_s": gather_s,
                     "rollout_gather_bytes": (int(rows.numel() * rows.element_size() * world) if gather_s is not None
                                              else None),
                     "rollout_gather_exact": gather_exact},
            "roofline": roof, "cpu_baseline": cpu,
            "validity": {"state_finite": finite, "envs_status_nonzero": nbad,
                         "library": build.library_info()},
        }
        print(json.dumps(line), flush=True)
        if not finite:
            print("bench: non-finite simulation state after the timed region", file=sys.stderr)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()
    if not finite:
        sys.exit(3)


def launcher_check(args, rank, world, launcher):
    """The multi-rank plumbing of main() with an empty timed region (no GPU, no simulator)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
        assert dist.get_world_size() == args.gpus
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    if world > 1:
        dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "steps": args.steps,
                          "ms_per_step": float(dt[0]) * 1e3, "dist": {"world_size": world, "backend": "gloo",
                                                                       "launcher": launcher},
                          "launcher_check": True}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
