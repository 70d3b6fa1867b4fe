#!/usr/bin/env python3
"""Summarise gpurun_out/phase_rs{1,0}.log (tools/phase_prof.py output)."""
import json
import os
import sys
for w in sys.argv[1:] or ["1"]:
    p = f"gpurun_out/phase_rs{w}.log"
    if not os.path.exists(p):
        continue
    print("RS" if w == "1" else "QUAD")
    for l in open(p):
        if not l[0].isdigit():
            continue
        t, js = l.split(" ", 1)
        r = json.loads(js)
        print(t, "cyc/wave", round(r["cycles_per_wave"]), "max", r["max_wave_cycles"], "pgs", round(r["pgs"], 3),
              "rows", round(r["rows"], 3), "smooth", round(r["smooth"], 3), "int", round(r["integrate+out"], 3),
              "sweeps", round(r["mean_sweeps"], 1), "wmax", round(r["mean_wave_max_sweeps"], 1), "maxpgs", r["max_wave_pgs_cycles"])
        if "rs" in r:
            print("   rs", {k: round(v, 1) for k, v in r["rs"].items()})
        print("   ", r["stamps_per_wave"])
