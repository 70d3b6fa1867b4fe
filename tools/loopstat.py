#!/usr/bin/env python3
"""Diagnostic: VALU / AGPR-read / DPP counts of the PGS sweep loops (loops holding
quad-broadcast DPP movs) of k_substep<6,1> in a gfx950 .s dump.
usage: loopstat.py k.s"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
st = [i for i, l in enumerate(lines) if re.match(r"^_Z9k_substepILi6ELi1", l)][0]
en = [i for i, l in enumerate(lines) if i > st and l.startswith(".Lfunc_end")][0]
body = lines[st:en]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
res = []
for i, l in enumerate(body):
    m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        a = labels[m.group(1)]
        seg = [x.strip() for x in body[a:i + 1]]
        if any("quad_perm" in x for x in seg) and i - a < 900:
            res.append((sum(x.startswith("v_") for x in seg), sum(x.startswith("v_pk_") for x in seg),
                         sum("accvgpr_read" in x for x in seg), sum("scratch_" in x for x in seg), sum(x.startswith("ds_") for x in seg), a))
for r in sorted(set(res)):
    print("valu %4d  pk %3d  agpr %3d  scratch %2d  lds %3d  @%d" % r)
