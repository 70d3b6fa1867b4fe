#!/usr/bin/env python3
"""Diagnostic: per-loop instruction mix of one kernel in a gfx950 .s dump.

usage: isa_loops.py k.s <kernel-substring> [top]
Splits the kernel into basic blocks, finds back edges (branch to an earlier
label) and prints, per loop (label range), the VALU / LDS / SALU / VMEM
instruction counts of its body — the per-iteration issue cost of a sweep."""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
lines = open(path).read().split("\n")
start = end = None
for i, l in enumerate(lines):
    if start is None:
        if re.match(r"^_Z\w*:", l) and pat in l.split(":")[0]:
            start = i
    elif re.match(r"^\.Lfunc_end", l):
        end = i
        break
body = lines[start:end]
labels = {}
order = []
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
loops = []
for i, l in enumerate(body):
    m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        loops.append((labels[m.group(2)], i, m.group(2)))


def mix(a, b):
    c = {"valu": 0, "lds": 0, "salu": 0, "vmem": 0, "smem": 0, "pk": 0, "trans": 0, "other": 0}
    for l in body[a:b + 1]:
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        if op.startswith("v_"):
            c["valu"] += 1
            if op.startswith("v_pk_"):
                c["pk"] += 1
            if any(x in op for x in ("rcp", "rsq", "sqrt", "exp", "log", "sin", "cos")):
                c["trans"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer"):
            c["smem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        else:
            c["other"] += 1
    return c


loops.sort(key=lambda x: -(x[1] - x[0]))
print(f"kernel lines {len(body)}, loops {len(loops)}")
for a, b, name in loops[:top]:
    print(name, f"lines {a}-{b}", mix(a, b))

if len(sys.argv) > 4 and sys.argv[4][:1].isdigit():  # mix of [a, b] minus nested loops: python isa_loops.py k.s pat top a-b
    a, b = map(int, sys.argv[4].split("-"))
    inner = [(x, y) for x, y, _ in loops if a <= x and y <= b and (x, y) != (a, b)]
    # keep outermost inner loops
    inner = [(x, y) for x, y in inner if not any(p <= x and y <= q and (p, q) != (x, y) for p, q in inner)]
    tot = mix(a, b)
    for x, y in sorted(set(inner)):
        c = mix(x, y)
        print(f"  inner {x}-{y}", c)
        for k in tot:
            tot[k] -= c[k]
    print("straight-line part", tot)

if "--innermost" in sys.argv:
    uniq = sorted({(a, b) for a, b, _ in loops})
    inner = [(a, b) for a, b in uniq if not any(x >= a and y <= b and (x, y) != (a, b) for x, y in uniq)]
    print("innermost loops (body instructions):")
    for a, b in sorted(inner, key=lambda t: -(t[1] - t[0]))[:top]:
        c = mix(a, b)
        print(f"  {a}-{b}", c, "total", sum(c[k] for k in ("valu", "lds", "salu", "vmem", "smem")))
