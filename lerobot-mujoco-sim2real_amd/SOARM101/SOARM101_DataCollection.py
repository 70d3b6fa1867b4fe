"""Batched SOARM101_DataCollection: the reference's rollout loop, on device.

Reference: ``SOARM101/SOARM101_DataCollection.py``.  The reference steps one
env per trajectory serially (``:108-134``); here all ``traj_num``
trajectories are envs of one :class:`SOARM101VecEnv` stepped in lockstep on the
GPU, with the action generators evaluated on device, so a whole dataset build
is ``steps`` kernel launches.  The output layout is unchanged:
``ndarray[traj, steps+1, 13]`` float64 with columns ``[u(5) | ee_xyz(3) | q(5)]``,
row 0 = ``[u0, s0]`` and row i = ``[u_i, s_i]`` where ``s_i`` is the state
after applying ``u_{i-1}`` (``:118-134``).

Action sources (``input_type``):
* ``random``: u ~ U[-0.5, 0.5)^5 each step (``:115,132``);
* ``sin`` / ``chirp``: :class:`SineInputGenerator` (``:31-74``), tables
  freq ~ U(0.0025, 0.05), amp ~ U(-0.5, 0.5), phase ~ U(0, 2pi) per
  trajectory/dim (``:97-103``), chirp f += (f_end - f_start) t / 200;
* ``ik_fig8`` / ``ik_circle`` (build-defined extension, SURVEY.md §8a note ii):
  per env a Fig8/Circle Cartesian target stream (random phase), batched DLS-IK
  gives q*, action = clip((q* - q) / dt, +-max_speed).
"""
import json
import os

import numpy as np

from ..args import Args
from .SOARM101_Env import SOARM101VecEnv


class Collater:
    """Splits a batch [B, T, 13] into x = [:, :, u:u+x] and u = [:, :, :u] (``:13-29``)."""

    def __init__(self, x_dim: int, u_dim: int, device: str = "cuda"):
        self.x_dim, self.u_dim, self.device = x_dim, u_dim, device

    def __call__(self, batch_list):
        import torch

        batch = torch.stack(list(zip(*batch_list))[0], dim=0)
        return dict(x=batch[:, :, self.u_dim:self.u_dim + self.x_dim].to(self.device),
                    u=batch[:, :, :self.u_dim].to(self.device))

    def split_device(self, rollout):
        """Zero-copy views of a device rollout [T+1, N, 13] -> x [N, T+1, x], u [N, T+1, u]."""
        r = rollout.transpose(0, 1)
        return dict(x=r[:, :, self.u_dim:self.u_dim + self.x_dim], u=r[:, :, :self.u_dim])


class SineInputGenerator:
    """Per-trajectory sine / chirp inputs (reference ``:31-74``), vectorised over trajectories."""

    def __init__(self, traj_num, udim=5, freq_range=(0.01, 0.05), amp_range=(0.05, 0.15),
                 sine_mask=None, mode="sin", rng=None):
        rng = rng if rng is not None else np.random
        self.traj_num, self.udim, self.mode = traj_num, udim, mode
        self.freq_start, self.freq_end = freq_range
        self.freq_table = rng.uniform(freq_range[0], freq_range[1], size=(traj_num, udim))
        self.amp_table = rng.uniform(amp_range[0], amp_range[1], size=(traj_num, udim))
        self.phase_table = rng.uniform(0, 2 * np.pi, size=(traj_num, udim))
        self.sine_mask = np.ones((traj_num, udim), bool) if sine_mask is None else sine_mask.astype(bool)

    def freq(self, t, T_total=200):
        if self.mode == "chirp":
            return self.freq_table + (self.freq_end - self.freq_start) * (t / T_total)
        return self.freq_table

    def __call__(self, t, traj_i, T_total=200):
        f = self.freq(t, T_total)[traj_i]
        u = np.zeros(self.udim)
        v = self.amp_table[traj_i] * np.sin(2 * np.pi * f * t + self.phase_table[traj_i])
        m = self.sine_mask[traj_i]
        u[m] = v[m]
        return u

    def rows(self, lo, hi):
        """The generator of trajectories [lo, hi) (their table rows; same draws as the full one)."""
        g = object.__new__(SineInputGenerator)
        g.traj_num, g.udim, g.mode = hi - lo, self.udim, self.mode
        g.freq_start, g.freq_end = self.freq_start, self.freq_end
        g.freq_table, g.amp_table = self.freq_table[lo:hi], self.amp_table[lo:hi]
        g.phase_table, g.sine_mask = self.phase_table[lo:hi], self.sine_mask[lo:hi]
        return g

    def batch(self, t, T_total=200):
        """All trajectories at step t: [traj_num, udim] float64."""
        v = self.amp_table * np.sin(2 * np.pi * self.freq(t, T_total) * t + self.phase_table)
        return np.where(self.sine_mask, v, 0.0)


class DeviceSine:
    """The same generator evaluated on the GPU (tables resident, one fused torch expression per step)."""

    def __init__(self, gen: SineInputGenerator, device):
        import torch

        self.g = gen
        t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=device)
        self.f, self.a, self.p = t(gen.freq_table), t(gen.amp_table), t(gen.phase_table)
        self.m = torch.as_tensor(gen.sine_mask, device=device)

    def __call__(self, t, T_total=200):
        import torch

        f = self.f + (self.g.freq_end - self.g.freq_start) * (t / T_total) if self.g.mode == "chirp" else self.f
        v = self.a * torch.sin(2 * np.pi * f * t + self.p)
        return torch.where(self.m, v, torch.zeros_like(v)).float()


def cartesian_targets(kind, t_param, idx=1, scale=0.5):
    """Fig8 / Circle Cartesian paths of ``control/TrajectoryGenerator.py:138-166`` (numpy or torch)."""
    lib = np if isinstance(t_param, np.ndarray) else __import__("torch")
    one = lib.ones_like(t_param)
    s, c = lib.sin(t_param), lib.cos(t_param)
    if kind == "Fig8":
        a = b = 0.2 * scale
        if idx == 1:
            x, y, z = 0.4 * one, b * c / (1 + s ** 2), 0.2 + 2 * a * s * c / (1 + s ** 2)
        else:
            x, y, z = 0.3 + 2 * a * s * c / (1 + s ** 2), b * c / (1 + s ** 2), 0.2 * one
    elif kind == "Circle":
        r = 0.1
        if idx == 1:
            x, y, z = 0.4 * one, r * c, 0.2 + r * s
        else:
            x, y, z = 0.3 + r * c, r * s, 0.2 * one
    else:
        raise ValueError(f"unknown trajectory {kind}")
    return lib.stack([x, y, z], -1)


def stream_seed(seed, stream):
    """32-bit seed of rollout stream `stream` under the user seed (splitmix64 finaliser).

    The reference draws every dataset from ONE advancing ``np.random`` stream
    (``SOARM101_DataCollection.py:97-132``), so train / val / test splits are independent
    draws.  Here every split has a stream of its own, keyed by the split's identity
    (:data:`SPLIT_STREAM`), never by call order: regenerating one missing file of a
    partially cached dataset reproduces exactly that split, and no two splits share initial
    states or inputs."""
    m = (1 << 64) - 1
    z = (int(seed) * 0x9E3779B97F4A7C15 + (int(stream) + 1) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return int((z ^ (z >> 31)) & 0xFFFFFFFF)


# stream index of each dataset split of generate_and_save_data (SOARM101_DataCollection.py:138-181)
SPLIT_STREAM = {"train": 0, "val": 1, "test_random": 2, "test_sin": 3, "test_chirp": 4}
# counter words of the keyed draws (sim_rand_uniform): step i of the random input stream uses
# counter i; the IK phase uses PHASE_COUNTER
PHASE_COUNTER = 0xFFFFFFFF


def _dist():
    """(rank, world) of an initialised torch.distributed job, else (0, 1)."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except ImportError:
        pass
    return 0, 1


class SOARM101DataGenerator:
    """Reference ``SOARM101DataGenerator`` (``:77-205``) with a batched GPU rollout.

    Multi-GPU: under ``torchrun`` (one process per GPU, torch.distributed
    initialised) every dataset shards by global trajectory id — rank r rolls out
    ``shard.shard_range(traj_num, world, r)`` on its own GPU — and either gathers the rows to
    rank 0 (RCCL over xGMI) or writes per-rank ``.npy`` shards plus a manifest
    (``shard_files=True``).  Every draw (reset state, random inputs, sine tables, IK phase)
    is keyed by (split seed, global trajectory id), so the concatenated shards equal the
    single-GPU dataset bit for bit."""

    def __init__(self, args: Args = None, device: int = None, max_envs: int = 65536, model=None,
                 shard_files: bool = False):
        self.args = args if args is not None else Args()
        self.udim, self.xdim = self.args.u_dim, self.args.x_dim
        rank, world = _dist()
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", rank)) if world > 1 else 0
        self.device_index = device
        self.max_envs = max_envs
        self.model = model
        self.shard_files = shard_files
        self.collate_fn = Collater(self.args.x_dim, self.args.u_dim, self.args.device)
        self._envs = {}
        self._stream = 100  # ad-hoc rollout calls: streams after the named splits

    def next_seed(self):
        """Seed of the next ad-hoc rollout stream (see :func:`stream_seed`)."""
        s = stream_seed(self.args.seed, self._stream)
        self._stream += 1
        return s

    def split_seed(self, split):
        """Seed of a named dataset split (:data:`SPLIT_STREAM`)."""
        return stream_seed(self.args.seed, SPLIT_STREAM[split])

    def _env(self, n):
        if n not in self._envs:
            self._envs[n] = SOARM101VecEnv(num_envs=n, device=self.device_index, model=self.model,
                                           seed=self.args.seed)
            self.model = self._envs[n].model
        return self._envs[n]

    # ------------------------------------------------------------ device rollout
    def rollout_device(self, n, steps, input_type="random", init_qpos=None, actions=None, seed=None,
                       sine=None, env_offset=0):
        """Rollout of `n` envs for `steps` env-steps; returns a device tensor [steps+1, n, 13] fp32.

        Env i is global trajectory ``env_offset + i``: its reset state, random inputs and IK
        phase are keyed by (seed, that id), and ``sine`` (a :class:`SineInputGenerator` over
        these n trajectories) holds its table rows.
        actions: optional [steps+1, n, 5] (row i = u_i) to replay a fixed input sequence.
        seed: None takes the generator's next ad-hoc stream (:meth:`next_seed`)."""
        import torch

        env = self._env(n)
        env._env_offset = env_offset
        sim = env.sim
        dev = sim.device
        if seed is None:
            seed = self.next_seed()
        if input_type in ("sin", "chirp") and actions is None:
            sine = sine or SineInputGenerator(n, self.udim, (0.0025, 0.05), (-0.5, 0.5), mode=input_type,
                                              rng=np.random.default_rng(seed))
            dsine = DeviceSine(sine, dev)
        ik = input_type.startswith("ik_") and actions is None
        if ik:
            kind = "Fig8" if input_type == "ik_fig8" else "Circle"
            phase = sim.rand_uniform(seed, PHASE_COUNTER, 1, 0.0, 2 * np.pi, env_offset)[:, 0].double()
            qstar = None

        def u_at(i, obs):
            nonlocal qstar
            if actions is not None:
                return torch.as_tensor(actions[i], dtype=torch.float32, device=dev)
            if input_type == "random":  # (rand(5) - 0.5) * 2 * 0.5, keyed by (seed, traj id, step)
                return sim.rand_uniform(seed, i, self.udim, -0.5, 0.5, env_offset)
            if input_type in ("sin", "chirp"):
                return dsine(i)
            if ik:
                t = 1.6 + 0.02 * (i + 1) + phase
                tgt = cartesian_targets(kind, t).float()
                qstar, ok, _ = sim.ik(tgt, q=qstar if qstar is not None else sim.qpos.clone())
                q = obs[:, 3:8]
                return torch.clamp((qstar[:5].T - q) / env.dt, -env.max_speed, env.max_speed)
            raise ValueError(input_type)

        out = torch.empty((steps + 1, n, self.udim + self.xdim), dtype=torch.float32, device=dev)
        opts = None if init_qpos is None else {"initial_state": np.concatenate(
            [np.asarray(init_qpos), np.zeros_like(init_qpos)], axis=1)}
        # reset draw keyed by (seed, global id): SOARM101VecEnv keys it by (seed, call index 0)
        s, _ = env.reset(seed=seed, options=opts)
        u = u_at(0, s)
        out[0, :, :self.udim] = u
        out[0, :, self.udim:] = s
        for i in range(1, steps + 1):
            s, *_ = env.step(out[i - 1, :, :self.udim])
            u = u_at(i, s)
            out[i, :, :self.udim] = u
            out[i, :, self.udim:] = s
        return out

    def _rollout_ids(self, traj_num, steps, input_type, seed, lo, hi, **kw):
        """Rows of global trajectories [lo, hi) as a device tensor [steps+1, hi-lo, 13], in chunks of
        at most max_envs envs; the sine tables are the full dataset's rows lo..hi."""
        import torch

        sine_all = None
        if input_type in ("sin", "chirp") and "actions" not in kw:
            sine_all = SineInputGenerator(traj_num, self.udim, (0.0025, 0.05), (-0.5, 0.5), mode=input_type,
                                          rng=np.random.default_rng(seed))
        parts = []
        for s0 in range(lo, hi, self.max_envs):
            n = min(self.max_envs, hi - s0)
            sine = sine_all.rows(s0, s0 + n) if sine_all is not None else None
            parts.append(self.rollout_device(n, steps, input_type, seed=seed, sine=sine, env_offset=s0, **kw))
        if not parts:
            return torch.empty((steps + 1, 0, self.udim + self.xdim), dtype=torch.float32,
                               device=torch.device("cuda", self.device_index))
        return parts[0] if len(parts) == 1 else torch.cat(parts, dim=1)

    def generate_physics_based_data(self, traj_num, steps, input_type, seed=None, rank=None, world=None,
                                    gather=True, **kw):
        """Same contract as the reference (``:90-136``): ndarray[traj, steps+1, 13] float64.

        Multi-GPU (torch.distributed initialised, or explicit rank/world): this rank rolls
        out its shard of trajectory ids; with ``gather`` rank 0 receives the whole dataset
        (other ranks return None), otherwise every rank returns its own shard's rows."""
        from .. import shard

        if seed is None:
            seed = self.next_seed()
        drank, dworld = _dist()
        rank = drank if rank is None else rank
        world = dworld if world is None else world
        lo, hi = shard.shard_range(traj_num, world, rank)
        local = self._rollout_ids(traj_num, steps, input_type, seed, lo, hi, **kw)
        if world > 1 and gather and dworld > 1:
            full = shard.gather_rollouts(local, dst=0)
            return None if full is None else full.transpose(0, 1).double().cpu().numpy()
        return local.transpose(0, 1).double().cpu().numpy()

    def _split(self, path, split, samples, steps, input_type):
        """One dataset file: load it if cached, else generate (sharded under torch.distributed).

        Under torch.distributed rank 0 alone decides whether the cache exists and broadcasts the
        decision, so every rank takes the same branch into (or past) the gather collective.
        Gather mode: rank 0 writes the file, then every rank holds the full dataset (it loads
        the file after a barrier, or -- when the file is not visible on some rank, e.g. a
        node-local filesystem -- receives the array from rank 0).  Shard-file mode: every rank
        holds its own shard's rows."""
        from .. import shard

        rank, world = _dist()
        if world > 1:
            import torch.distributed as dist
            flag = [os.path.exists(path) if rank == 0 else None]
            dist.broadcast_object_list(flag, src=0)
            cached = bool(flag[0])
        else:
            cached = os.path.exists(path)
        if cached and (world == 1 or not self.shard_files):
            return np.load(path) if world == 1 else self._everyone_loads(path, None)
        seed = self.split_seed(split)
        if world > 1 and self.shard_files:
            base = path[:-4] if path.endswith(".npy") else path
            mine = f"{base}.rank{rank}-of-{world}.npy"
            if os.path.exists(mine):  # resume from this rank's shard
                return np.load(mine)
            part = self.generate_physics_based_data(samples, steps, input_type, seed=seed, gather=False)
            np.save(mine, part)
            if rank == 0:
                man = {"file": os.path.basename(path), "shape": [samples, steps + 1, self.udim + self.xdim],
                       "dtype": "float64", "seed": seed, "input_type": input_type,
                       "shards": [{"file": os.path.basename(f"{base}.rank{r}-of-{world}.npy"),
                                   "traj": list(shard.shard_range(samples, world, r))} for r in range(world)]}
                with open(f"{base}.manifest.json", "w") as f:
                    json.dump(man, f, indent=1)
            return part
        data = self.generate_physics_based_data(samples, steps, input_type, seed=seed)
        if rank == 0:
            np.save(path, data)
        return data if world == 1 else self._everyone_loads(path, data)

    @staticmethod
    def _everyone_loads(path, data):
        """Collective: every rank returns rank 0's dataset `path` (rank 0 passes `data`, or None to
        load it).  Ranks that see the file load it after the barrier that follows rank 0's save;
        if any rank cannot see it, rank 0 broadcasts the array instead."""
        import torch.distributed as dist

        dist.barrier()
        seen = [None] * dist.get_world_size()
        dist.all_gather_object(seen, os.path.exists(path))
        rank = dist.get_rank()
        if all(seen):
            return data if (rank == 0 and data is not None) else np.load(path)
        box = [(data if data is not None else np.load(path)) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def generate_and_save_data(self):
        """File cache / resume as the reference (``:138-181``); each split keyed by its name."""
        a = self.args
        os.makedirs(a.data_dir_save, exist_ok=True)
        self.train_data = self._split(a.data_dir_load_train, "train", a.train_samples, a.train_steps, "random")
        self.val_data = self._split(a.data_dir_load_val, "val", a.test_samples, a.test_steps, "random")
        self.test_data_dict = {}
        for t in ["random", "sin", "chirp"]:
            p = os.path.join(a.data_dir_save, f"test_data_{t}_{a.test_samples}_{a.test_steps}.npy")
            self.test_data_dict[t] = self._split(p, f"test_{t}", a.test_samples, a.test_steps, t)

    def get_train_loader(self):
        import torch
        from torch.utils.data import DataLoader, TensorDataset

        tr = DataLoader(TensorDataset(torch.tensor(self.train_data, dtype=torch.float32)),
                        batch_size=self.args.batch_size, collate_fn=self.collate_fn, shuffle=True)
        va = DataLoader(TensorDataset(torch.tensor(self.val_data, dtype=torch.float32)),
                        batch_size=self.args.eval_batch_size, collate_fn=self.collate_fn, shuffle=False)
        return tr, va

    def get_test_loader(self, test_type):
        import torch
        from torch.utils.data import DataLoader, TensorDataset

        d = torch.tensor(self.test_data_dict[test_type], dtype=torch.float32)
        return DataLoader(TensorDataset(d), batch_size=self.args.eval_batch_size,
                          collate_fn=self.collate_fn, shuffle=False)
