#!/bin/bash
# phase profile of the contact substep, wide kernel on and off (driver window and steady window)
mkdir -p gpurun_out
for w in 1 0; do
  SOARM_WIDE=$w EVERY=20 timeout -k 10 300 python tools/phase_prof.py 120 > gpurun_out/phase_w$w.log 2>&1 || exit $?
  cp gpurun_out/phase_prof_contact_pgs.json gpurun_out/phase_w$w.json
done
python - <<'PY'
import json
for w in (1, 0):
    d = json.load(open(f"gpurun_out/phase_w{w}.json"))
    for t, r in d.items():
        print("wide", w, "t", t, "cyc/wave", round(r["cycles_per_wave"]), "max", r["max_wave_cycles"], "pgs share", round(r["pgs"], 3),
              "maxpgs", r["max_wave_pgs_cycles"], "variants", {k: round(v, 4) for k, v in r["variant_waves"].items()},
              "varmax", r["variant_max_cycles"], "yarm", {k: (v["waves"], v["max_cycles"]) for k, v in r["yarm_subvariants"].items()})
PY
