#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of tools/gpu_profile.sh into
profiles/<tag>_pmc_summary.json and profiles/pmc_traffic.json.

HBM traffic per launch follows MI355X_MICROARCH.md "HBM [CDNA4]":
FETCH_SIZE and WRITE_SIZE (kilobytes, memory-side L2 requests) come from
separate passes; on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so it is
doubled; WRITE_SIZE is taken as is.  SQ_* cycle counters are quad-cycles.

    python tools/pmc_summary.py gpurun_out/prof_r02_contact r02 [config]
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {"k_substep": "substep", "k_collide": "collide", "k_step": "step_fused", "k_geom": "geom",
         "k_mpc_step": "mpc_step", "k_bias": "bias", "k_bilinear": "bilinear", "k_encode": "encode"}


def short(name):
    for k, v in SHORT.items():
        if k + "(" in name or k + "<" in name:
            return v
    return None


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    res = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        res[k] = {"grid": int(r["Grid_Size"]), "block": int(r["Workgroup_Size"]),
                  "lds_bytes": int(r["LDS_Block_Size"]), "scratch_bytes": int(r["Scratch_Size"]),
                  "vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]), "sgpr": int(r["SGPR_Count"])}
    return agg, res


def main():
    d, tag = sys.argv[1], sys.argv[2]
    cfg = sys.argv[3] if len(sys.argv) > 3 else "contact"
    out = {"source": f"rocprofv3 --pmc passes of tools/gpu_profile.sh ({d})", "config": cfg, "kernels": {}}
    traffic = {}
    agg_all, res_all = {}, {}
    for name in ("pmc_fetch", "pmc_write", "pmc_sq"):
        p = os.path.join(d, f"{name}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg, res = load(p)
        res_all.update(res)
        for k, cs in agg.items():
            agg_all.setdefault(k, {}).update({c: sum(v) / len(v) for c, v in cs.items()})
            agg_all[k]["_launches_" + name] = len(next(iter(cs.values())))
    for k, c in agg_all.items():
        e = dict(res_all.get(k, {}))
        e.update({kk: vv for kk, vv in c.items()})
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            fetch = 2.0 * c["FETCH_SIZE"] * 1024
            write = c["WRITE_SIZE"] * 1024
            e["hbm_bytes_per_launch"] = fetch + write
            e["hbm_fetch_bytes_per_launch_corrected"] = fetch
            e["hbm_write_bytes_per_launch"] = write
            traffic[k] = fetch + write
        if "SQ_WAVE_CYCLES" in c and c.get("SQ_WAVES"):
            w = c["SQ_WAVES"]
            e["per_wave"] = {"cycles": 4 * c["SQ_WAVE_CYCLES"] / w,
                             "valu_insts": c.get("SQ_INSTS_VALU", 0) / w,
                             "lds_insts": c.get("SQ_INSTS_LDS", 0) / w,
                             "salu_insts": c.get("SQ_INSTS_SALU", 0) / w,
                             "wait_frac": c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"],
                             "active_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]}
        out["kernels"][k] = e
    pdir = os.path.join(ROOT, "profiles")
    json.dump(out, open(os.path.join(pdir, f"{tag}_pmc_summary_{cfg}.json"), "w"), indent=1)
    tp = os.path.join(pdir, "pmc_traffic.json")
    allt = json.load(open(tp)) if os.path.exists(tp) else {}
    allt[cfg] = traffic
    allt["_note"] = ("HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KB->B), separate rocprofv3 --pmc passes, "
                     "MI355X_MICROARCH.md HBM section; source " + tag)
    json.dump(allt, open(tp, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
