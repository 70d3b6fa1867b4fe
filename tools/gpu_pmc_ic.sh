#!/bin/bash
# instruction/scalar-cache counters of the contact substep: RS kernel vs quad kernel
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for w in 1 0; do
  SOARM_RS=$w timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_HITS \
    -d $R/gpurun_out/pmc_ic$w -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-other-solver --no-steady --steps 3 --warmup 2 > $R/gpurun_out/pmc_ic$w.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ["GRAFT_REPO_ROOT"]
for w in ("1", "0"):
    f = glob.glob(f"{R}/gpurun_out/pmc_ic{w}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVES": cnt[k] += 1
    for k, d in acc.items():
        if "substep" in k or "collide" in k:
            n = cnt[k]
            print("RS" if w == "1" else "QUAD", k, {c: round(v / n) for c, v in sorted(d.items())})
PY
