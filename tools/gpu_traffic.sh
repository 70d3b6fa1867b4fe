#!/bin/bash
# HBM bytes per launch of the contact workload's kernels (FETCH / WRITE passes, as gpu_final_r05.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
KRE="k_substep|k_collide|k_geom"
NP="--steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-steady --no-other-solver"
P=$O/prof_traffic
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $P -o pmc_fetch -- python3 $R/bench.py $NP > /dev/null || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $P -o pmc_write -- python3 $R/bench.py $NP > /dev/null || exit $?
python3 - <<'PY'
import csv, glob, collections, os
P = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/prof_traffic"
for name in ("pmc_fetch", "pmc_write"):
    f = glob.glob(f"{P}/**/{name}_counter_collection.csv", recursive=True)[0]
    acc, cnt = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
        acc[k] += float(r["Counter_Value"]); cnt[k] += 1
    print(name, {k: round(v / cnt[k]) for k, v in acc.items()}, "KB per launch (FETCH x2 for HBM bytes)")
PY
