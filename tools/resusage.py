#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS usage of the HIP library (compiler remarks).

    python tools/resusage.py [out.txt]

Compiles csrc/soarm_sim.hip with -Rpass-analysis=kernel-resource-usage into a
throwaway .so and prints one line per kernel; used to check that an edit did
not change the hot kernels' register allocation (A/B before measuring).
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import soarm_pkg  # noqa: F401,E402
from lerobot_mujoco_sim2real_amd import build  # noqa: E402


def main():
    cmd = [build.HIPCC] + build.FLAGS + ["-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/_resusage.so"]
    cmd += [os.path.join(build.SRC_DIR, s) for s in build.SOURCES]
    out = subprocess.run(cmd, cwd=build.SRC_DIR, capture_output=True, text=True).stderr
    rows, cur = [], None
    for ln in out.splitlines():
        m = re.search(r"remark:\s+(\w[\w /\[\]]*?): (.*?) \[-Rpass", ln)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    lines = [f"{r['name'][:70]:70s} V{r.get('VGPRs', '?'):>4} A{r.get('AGPRs', '?'):>4} S{r.get('TotalSGPRs', '?'):>4} spill{r.get('VGPRs Spill', '?')} "
             f"scr{r.get('ScratchSize [bytes/lane]', '?'):>5} lds{r.get('LDS Size [bytes/block]', '?'):>7}" for r in rows]
    txt = "\n".join(lines)
    print(txt)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(txt + "\n")


if __name__ == "__main__":
    main()
