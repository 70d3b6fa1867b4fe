#!/usr/bin/env python3
"""Diagnostic: where a contact substep spends its cycles.

Needs the profiling build (tools/phase_prof.py --build compiles
csrc/soarm_sim.hip with -DSOARM_PHASE_PROF into tools/_prof/); on the GPU it
runs the bench's contact workload and prints the per-phase share of wave
cycles and the mean PGS sweep count."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("PROF_LIB") or os.path.join(ROOT, "tools", "_prof", "libsoarm_sim_prof.so")
SRC = os.path.join(ROOT, "lerobot-mujoco-sim2real_amd", "csrc", "soarm_sim.hip")

if "--build" in sys.argv:
    sys.path.insert(0, ROOT)
    import soarm_pkg  # noqa: F401
    from lerobot_mujoco_sim2real_amd.build import compile_lib

    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    compile_lib(LIB, ["-DSOARM_PHASE_PROF"] + [a for a in sys.argv[1:] if a.startswith("-D")])
    sys.exit(0)

sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import soarm_pkg  # noqa: E402,F401
from lerobot_mujoco_sim2real_amd import abi, workloads as W  # noqa: E402

lib = abi.load_lib(LIB)
abi._lib = lib
from lerobot_mujoco_sim2real_amd.sim import BatchSim  # noqa: E402

n = int(os.environ.get("ENVS", 4096))
T = int(sys.argv[1]) if len(sys.argv) > 1 else 120
cm = W.model(os.environ.get("CONFIG", "contact"), solver=os.environ.get("SOLVER", "PGS"))
ids = np.arange(n)
sim = BatchSim(cm, n, 0)
q0 = W.initial_qpos(cm, ids, 0)
sim.reset(init_qpos=q0[:, :5], extra_qpos=q0, seed=0)
tab = {k: (torch.as_tensor(v, dtype=torch.float32, device="cuda") if isinstance(v, np.ndarray) else v)
       for k, v in W.chirp_tables(ids, 0).items()}
out = (ctypes.c_double * 108)()
res = {}
every = int(os.environ.get("EVERY", 0))
starts = set(range(0, T, every)) if every else {0, T // 2, T - 10}
for t in range(T):
    if t in starts:
        torch.cuda.synchronize()
        lib.sim_phase_profile(ctypes.cast(out, ctypes.c_void_p), 1)
    sim.step(W.chirp_action(tab, float(t), lib=torch))
    if t - 9 in starts:
        torch.cuda.synchronize()
        lib.sim_phase_profile(ctypes.cast(out, ctypes.c_void_p), 1)
        v = list(out)
        tot = sum(v[:5])
        names = ["load", "smooth", "rows", "pgs", "integrate+out"]
        r = {nm: v[i] / tot for i, nm in enumerate(names)}
        r["cycles_per_wave"] = tot / max(v[5], 1)
        r["max_wave_cycles"] = v[8]
        r["fast_wave_frac"] = v[9] / max(v[5], 1)
        r["max_wave_pgs_cycles"] = v[10]
        r["mean_sweeps"] = v[6] / max(v[7], 1)
        r["mean_wave_max_sweeps"] = v[11] / max(v[5], 1)
        r["waves_with_limit"] = v[12] / max(v[5], 1)
        r["waves_with_nonblock_contact"] = v[13] / max(v[5], 1)
        r["waves_with_lds_overflow"] = v[14] / max(v[5], 1)
        r["max_ncon"] = v[15]
        r["rows_split"] = {"contact_rows": v[16] / tot, "warm_cost": v[17] / tot, "block_setup": v[18] / tot}
        r["variant_waves"] = {k: v[19 + i] / max(v[5], 1) for i, k in enumerate(["ypure", "yarm", "general", "other"])}
        r["variant_max_cycles"] = {k: v[23 + i] for i, k in enumerate(["ypure", "yarm", "general", "other"])}
        r["waves_with_free_nonblock"] = v[27] / max(v[5], 1)
        stamps = ["kinematics", "com_crb", "factor", "smooth_forces", "(gap)", "solve_m+Minv", "fric+limit rows",
                  "contact rows", "warm+cost", "pgs+qacc/fcon", "reload", "integrate", "store+obs",
                  "kinematics2", "geom poses"]
        r["stamps_per_wave"] = {nm: round(v[28 + i] / max(v[5], 1)) for i, nm in enumerate(stamps)}
        r["nony_lanes"] = {"npost": v[43:47], "free_extras": v[47:50], "nl>5": v[50], "limit": v[51], "overflow": v[52]}
        r["row_split_per_wave"] = {nm: round(v[53 + i] / max(v[5], 1)) for i, nm in
                                   enumerate(["loads+frame", "jacobian", "gram", "edges+writes"])}
        r["armstop_waves"] = v[57] / max(v[5], 1)
        r["mean_armstop_sweep"] = v[58] / max(v[57], 1)
        r["max_wave_cycles_kept_retired"] = [v[59], v[60]]
        r["yarm_subvariants"] = {k: {"waves": v[61 + i], "max_cycles": v[65 + i],
                                     "mean_pgs_cycles": v[69 + i] / max(v[61 + i], 1),
                                     "mean_retire_sweep": v[73 + i] / max(v[61 + i], 1)}
                                 for i, k in enumerate(["E", "E_coupled", "EF", "EF_coupled"])}
        if v[77 + 11] > 0:  # RS kernel split (soarm_pgs.h rs_solve, Newton profiler slots)
            w = v[77 + 11]
            r["rs"] = {"setup_cycles_per_wave": v[77 + 8] / w, "sweep_cycles_per_wave": v[77 + 9] / w,
                       "final_cycles_per_wave": v[77 + 10] / w, "sweeps_per_wave": v[77 + 16] / w,
                       "cycles_per_sweep": v[77 + 9] / max(v[77 + 16], 1),
                       "fallback_waves_per_launch": v[77 + 17] / max(v[5] / (n // 4), 1),
                       "fallback_max_cycles": v[77 + 18], "fallback_mean_cycles": v[77 + 19] / max(v[77 + 17], 1),
                       "fallback_lanes_by_cause": dict(zip(["limit", "overflow", "order", "ct>4", "at>1", "ac>1", "at+ac"],
                                                           [v[101 + k] for k in range(7)]))}
        if v[77] > 0:
            r["newton"] = {"solves": v[77], "mean_iters": v[78] / v[77], "mean_ls_evals": v[79] / v[77],
                           "coupled_frac": v[80] / v[77], "mean_cycles": v[81] / v[77], "max_cycles": v[82],
                           "max_iters": v[83], "max_ls_evals": v[84],
                           "split": {"arm_iters": v[85] / v[77], "arm_ls": v[86] / v[77],
                                     "free_iters": v[87] / v[77], "free_ls": v[88] / v[77]},
                           "wave_mean_max_ls": v[90] / max(v[89], 1), "wave_mean_max_iters": v[91] / max(v[89], 1),
                           "wave_mean_cycles": v[92] / max(v[89], 1),
                           "split_cycles_per_env": {k: v[93 + i] / v[77] for i, k in enumerate(["warm", "hessian+factor", "line_search", "new_point_pass"])},
                           "split_cycles_wave_max": {k: v[97 + i] / max(v[89], 1) for i, k in enumerate(["warm", "hessian+factor", "line_search", "new_point_pass"])}}
        res[t] = r
        print(t, json.dumps(r), flush=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", f"phase_prof_{os.environ.get('CONFIG', 'contact')}_{os.environ.get('SOLVER', 'PGS').lower()}.json"), "w"), indent=1)
