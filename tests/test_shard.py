"""Multi-GPU path on CPU: world-size-2 gloo process group."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import soarm_pkg  # noqa: F401  (spawned workers re-import this module: register the package alias)
from lerobot_mujoco_sim2real_amd import shard, workloads as W


def test_shard_ranges_partition():
    for total in (1, 7, 4096, 65536, 65537):
        for world in (1, 2, 3, 8):
            ids = np.concatenate([shard.shard_ids(total, world, r) for r in range(world)])
            np.testing.assert_array_equal(ids, np.arange(total))


def test_draws_independent_of_world_size():
    """Initial states / chirp tables / DR params are keyed by global env id."""
    cm = W.model("contact")
    total = 1000
    full_q = W.initial_qpos(cm, np.arange(total))
    full_t = W.chirp_tables(np.arange(total))
    full_d = W.dr_params(np.arange(total))
    for world in (2, 8):
        for r in range(world):
            ids = shard.shard_ids(total, world, r)
            np.testing.assert_array_equal(W.initial_qpos(cm, ids), full_q[ids])
            np.testing.assert_array_equal(W.chirp_tables(ids)["amp"], full_t["amp"][ids])
            np.testing.assert_array_equal(W.dr_params(ids)["friction"], full_d["friction"][ids])


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = shard.shard_ids(total, world, rank)
    T = 3
    # stand-in rollout: row t of env id i = [t, i, ...] so order is checkable
    local = torch.zeros((T + 1, len(ids), 13), dtype=torch.float32)
    local[:, :, 0] = torch.arange(T + 1, dtype=torch.float32)[:, None]
    local[:, :, 1] = torch.as_tensor(ids, dtype=torch.float32)[None, :]
    g = shard.gather_rollouts(local, dst=0)
    if rank == 0:
        torch.save(g, out)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_world2(tmp_path):
    out = str(tmp_path / "g.pt")
    total = 9  # uneven shards (5 + 4)
    mp.spawn(_worker, args=(2, _port(), total, out), nprocs=2, join=True)
    g = torch.load(out, weights_only=True)
    assert tuple(g.shape) == (4, total, 13)
    np.testing.assert_array_equal(g[0, :, 1].numpy(), np.arange(total))
    np.testing.assert_array_equal(g[:, 3, 0].numpy(), np.arange(4))


import pytest  # noqa: E402


@pytest.mark.gpu
def test_rccl_gather_one_rank_device_rollout(gpu_lib):
    """The RCCL path of the rollout gather on one GPU (BASELINE.json configs[4]):
    a one-rank ``nccl`` process group gathers a device rollout [T+1, N, 13] produced by the
    simulator (DLS-IK actions on the arm scene) through shard.gather_rollouts -- the collective
    config 5 ends with -- and rank 0 gets the local tensor back bit for bit.  (N > 1 ranks need an
    8-GPU node; that path stays unmeasured on hardware.)"""
    from lerobot_mujoco_sim2real_amd.sim import BatchSim
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cm = W.model("rollout")
    n, T = 256, 8
    ids = np.arange(n)
    sim = BatchSim(cm, n)
    q0 = W.initial_qpos(cm, ids, 0)
    sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
    phase = torch.as_tensor(W.ik_phase(ids, 0), dtype=torch.float32, device=sim.device)
    rows = torch.zeros((T + 1, n, 13), dtype=torch.float32, device=sim.device)  # (row T: no action)
    rows[0, :, 5:] = sim.obs
    qstar = sim.qpos.clone()
    act = sim.action_buffer()
    for t in range(T):
        qstar, _, _ = sim.ik(W.fig8_targets(float(t), phase, lib=torch), q=qstar)
        act.copy_(W.ik_action(qstar[:5].T, sim.obs[:, 3:8], lib=torch))
        rows[t, :, :5] = act
        rows[t + 1, :, 5:] = sim.step(act)
    torch.cuda.synchronize()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=sim.device)
    try:
        assert dist.get_backend() == "nccl"
        g = shard.gather_rollouts(rows, dst=0)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    assert g.device == rows.device and g.shape == rows.shape
    assert torch.equal(g, rows)
    assert torch.isfinite(rows).all()
