#!/bin/bash
# phase profile of the RS substep over the bench's steady window (per-wave rows)
mkdir -p gpurun_out
SOARM_RS=1 PROF_LIB=tools/_rsprof/libsoarm_sim_prof.so EVERY=20 timeout -k 10 300 python tools/phase_prof.py 130 > gpurun_out/phase_rs1.log 2>&1 || exit $?
python3 - <<'PY'
import json
for l in open("gpurun_out/phase_rs1.log"):
    if not l[0].isdigit(): continue
    t, js = l.split(" ", 1); r = json.loads(js)
    print(t, "mean", round(r["cycles_per_wave"]), "max", r["max_wave_cycles"], "maxpgs", r["max_wave_pgs_cycles"],
          "variants", {k: round(v, 4) for k, v in r["variant_waves"].items()}, "vmax", r["variant_max_cycles"],
          "nonblock", r["waves_with_nonblock_contact"], "maxncon", r["max_ncon"], "lim", r["waves_with_limit"])
    print("   rs", {k: (round(v, 2) if not isinstance(v, dict) else v) for k, v in r.get("rs", {}).items()})
PY
