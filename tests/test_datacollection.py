"""SOARM101_DataCollection host logic without a GPU: the input generators pinned against the
reference's formula, the keyed draws, per-split stream seeds, and the multi-GPU dataset build
(world-size-2 gloo, rollouts mocked by a deterministic function of (seed, global trajectory id,
step) so that only the sharding / gather / shard-file logic is under test)."""
import json
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import soarm_pkg  # noqa: F401  (spawned workers re-import this module)
from lerobot_mujoco_sim2real_amd import workloads as W
from lerobot_mujoco_sim2real_amd.args import Args
from lerobot_mujoco_sim2real_amd.SOARM101 import SOARM101_DataCollection as DC


# ------------------------------------------------ the reference's SineInputGenerator, restated
def _reference_tables(traj_num, udim, freq_range, amp_range):
    """SOARM101_DataCollection.py:48-50: three np.random.uniform draws, in this order."""
    f = np.random.uniform(freq_range[0], freq_range[1], size=(traj_num, udim))
    a = np.random.uniform(amp_range[0], amp_range[1], size=(traj_num, udim))
    p = np.random.uniform(0, 2 * np.pi, size=(traj_num, udim))
    return f, a, p


def _reference_call(tables, mode, freq_range, t, traj_i, T_total=200):
    """SOARM101_DataCollection.py:57-74."""
    f, a, p = tables
    if mode == "sin":
        freq = f[traj_i]
    else:  # chirp
        ratio = t / T_total
        freq = f[traj_i] + (freq_range[1] - freq_range[0]) * ratio
    u = np.zeros(f.shape[1])
    u[:] = a[traj_i] * np.sin(2 * np.pi * freq * t + p[traj_i])
    return u


def test_sine_chirp_match_reference_formula():
    """The generators of generate_physics_based_data (:97-103, freq (0.0025, 0.05), amp (-0.5,
    0.5)) against the reference's formula, t = 0..200, every trajectory, both modes; tables
    drawn from the same np.random state, so the values are bit-identical."""
    fr, ar = (0.0025, 0.05), (-0.5, 0.5)
    for mode in ("sin", "chirp"):
        np.random.seed(1234)
        ref = _reference_tables(37, 5, fr, ar)
        np.random.seed(1234)
        g = DC.SineInputGenerator(37, 5, fr, ar, mode=mode)  # rng None -> the global np.random
        np.testing.assert_array_equal(g.freq_table, ref[0])
        for t in range(201):
            b = g.batch(t)
            for i in (0, 17, 36):
                want = _reference_call(ref, mode, fr, t, i)
                np.testing.assert_array_equal(g(t, i), want)
                np.testing.assert_allclose(b[i], want, rtol=0, atol=1e-15)
        # the bench's chirp (workloads.chirp_action) is the same formula over its tables
        tab = dict(freq=g.freq_table, amp=g.amp_table, phase=g.phase_table, freq_start=fr[0], freq_end=fr[1])
        for t in (0, 7, 120, 200):
            if mode == "chirp":
                np.testing.assert_allclose(W.chirp_action(tab, t), g.batch(t), rtol=0, atol=1e-15)


def test_keyed_uniform_chunk_invariant():
    full = W.keyed_uniform(99, np.arange(1000), 7, 5, -0.5, 0.5)
    assert full.dtype == np.float32 and full.min() >= -0.5 and full.max() < 0.5
    np.testing.assert_array_equal(W.keyed_uniform(99, np.arange(300, 700), 7, 5, -0.5, 0.5), full[300:700])
    assert not np.array_equal(W.keyed_uniform(99, np.arange(1000), 8, 5, -0.5, 0.5), full)
    # distinct from the reset draw's stream (4th counter word 0)
    assert not np.array_equal(W.philox_uniform(99, np.arange(1000), 5), (full + 0.5))


def test_split_seeds_keyed_by_identity():
    a = DC.SOARM101DataGenerator(Args(["--seed", "5"]))
    b = DC.SOARM101DataGenerator(Args(["--seed", "5"]))
    b.next_seed(), b.next_seed()  # ad-hoc calls do not move the named splits' streams
    assert [a.split_seed(k) for k in DC.SPLIT_STREAM] == [b.split_seed(k) for k in DC.SPLIT_STREAM]
    assert len({a.split_seed(k) for k in DC.SPLIT_STREAM} | {a.next_seed()}) == 6


# ------------------------------------------------------------------- mocked rollouts
def _mock_rollout(self, n, steps, input_type="random", init_qpos=None, actions=None, seed=None, sine=None,
                  env_offset=0):
    """Stand-in for the device rollout: rows of global trajectory id g are a function of
    (seed, g, step) only, with the real input streams (keyed random draws / sine rows)."""
    ids = np.arange(env_offset, env_offset + n)
    rows = torch.zeros((steps + 1, n, 13), dtype=torch.float32)
    for i in range(steps + 1):
        if input_type == "random":
            u = W.keyed_uniform(seed, ids, i, 5, -0.5, 0.5)
        else:
            u = sine.batch(i)
        rows[i, :, :5] = torch.as_tensor(u, dtype=torch.float32)
        rows[i, :, 5:] = torch.as_tensor(W.keyed_uniform(seed ^ 0x5A5A, ids, i, 8, -1.0, 1.0))
    return rows


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dataset_worker(rank, world, port, root, shard_files, out=None, runs=1, hide=False):
    """One rank of a world-`world` dataset build; with `out`, each rank saves what its generator
    holds after every run (run 0 builds the files, run 1 finds them cached).  `hide`: rank 1
    sees no dataset file (a node-local filesystem)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    DC.SOARM101DataGenerator.rollout_device = _mock_rollout
    if hide and rank == 1:
        real = os.path.exists
        os.path.exists = lambda p: False if str(p).endswith(".npy") else real(p)
    a = Args(["--data_root", root, "--train_samples", "37", "--train_steps", "3", "--test_samples", "11",
              "--test_steps", "4"])
    for run in range(runs):
        g = DC.SOARM101DataGenerator(a, max_envs=8, shard_files=shard_files)
        g.generate_and_save_data()
        if out is not None:
            np.savez(os.path.join(out, f"rank{rank}_run{run}.npz"), train=g.train_data, val=g.val_data,
                     **{f"test_{k}": v for k, v in g.test_data_dict.items()})
    dist.barrier()
    dist.destroy_process_group()


def _single(root):
    DC.SOARM101DataGenerator.rollout_device = _mock_rollout
    a = Args(["--data_root", root, "--train_samples", "37", "--train_steps", "3", "--test_samples", "11",
              "--test_steps", "4"])
    g = DC.SOARM101DataGenerator(a, max_envs=64)
    g.generate_and_save_data()
    return g


def test_sharded_dataset_equals_single_rank(tmp_path, monkeypatch):
    """world 2 (gloo): gathered to rank 0, and per-rank shard files + manifest — both equal the
    single-process dataset (other chunking too: max_envs 8 vs 64)."""
    monkeypatch.setattr(DC.SOARM101DataGenerator, "rollout_device", _mock_rollout)
    ref = _single(str(tmp_path / "one"))
    names = {"train": "train_data_37_3", "val": "val_data_11_4", "test_random": "test_data_random_11_4",
             "test_sin": "test_data_sin_11_4", "test_chirp": "test_data_chirp_11_4"}
    want = {"train": ref.train_data, "val": ref.val_data, **{f"test_{k}": v for k, v in ref.test_data_dict.items()}}
    # splits are distinct streams
    assert not np.array_equal(want["val"][:, 0], want["train"][:11, 0])
    out = tmp_path / "held"
    out.mkdir()
    mp.spawn(_dataset_worker, args=(2, _port(), str(tmp_path / "gather"), False, str(out), 2), nprocs=2, join=True)
    d = tmp_path / "gather" / "SOARM101" / "data"
    for k, nm in names.items():
        np.testing.assert_array_equal(np.load(d / f"{nm}.npy"), want[k])
    # in gather mode every rank holds the whole dataset, on the first run (built and
    # gathered) and on the rerun (cached) alike -- never None on rank 1
    for r in range(2):
        for run in range(2):
            held = np.load(out / f"rank{r}_run{run}.npz")
            for k in names:
                np.testing.assert_array_equal(held[k], want[k])
    # a rank that cannot see the file (node-local storage) receives the arrays from rank 0
    out2 = tmp_path / "held2"
    out2.mkdir()
    mp.spawn(_dataset_worker, args=(2, _port(), str(tmp_path / "hidden"), False, str(out2), 2, True), nprocs=2,
             join=True)
    for r in range(2):
        for run in range(2):
            held = np.load(out2 / f"rank{r}_run{run}.npz")
            for k in names:
                np.testing.assert_array_equal(held[k], want[k])
    mp.spawn(_dataset_worker, args=(2, _port(), str(tmp_path / "files"), True), nprocs=2, join=True)
    d = tmp_path / "files" / "SOARM101" / "data"
    for k, nm in names.items():
        man = json.load(open(d / f"{nm}.manifest.json"))
        parts = [np.load(d / s["file"]) for s in man["shards"]]
        assert [s["traj"] for s in man["shards"]][0][0] == 0 and man["shape"][0] == want[k].shape[0]
        np.testing.assert_array_equal(np.concatenate(parts), want[k])


def test_regenerating_one_split_reproduces_it(tmp_path, monkeypatch):
    """with train cached and val deleted, val regenerates to the same rows (its own
    stream), and no val trajectory starts where a train one does."""
    monkeypatch.setattr(DC.SOARM101DataGenerator, "rollout_device", _mock_rollout)
    g = _single(str(tmp_path))
    val = g.val_data.copy()
    os.remove(g.args.data_dir_load_val)
    g2 = _single(str(tmp_path))
    np.testing.assert_array_equal(g2.val_data, val)
    np.testing.assert_array_equal(g2.train_data, g.train_data)
    assert (np.abs(g2.val_data[:, 0, 5:] - g2.train_data[:11, 0, 5:]).max(1) > 1e-3).all()
