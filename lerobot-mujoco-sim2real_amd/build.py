"""Compile the HIP C-ABI library in-tree for gfx950 (no JIT caches)."""
import os
import subprocess

from .abi import LIB_PATH, PKG_DIR

SRC_DIR = os.path.join(PKG_DIR, "csrc")
SOURCES = ["soarm_sim.hip"]
HEADERS = ["dmodel.h", "soarm_kernels.h", "soarm_step.h", "soarm_collide.h", "soarm_pgs.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -fno-slp-vectorize: the per-lane algebra gains nothing from v_pk_* packing; the
# packing's operand shuffles (v_mov) and the extra register pressure (AGPR
# round trips) cost ~13% of the PGS sweep's VALU issue (ISA count, k_substep).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize"]


def _stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(SRC_DIR, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(PKG_DIR, "..", "include", "soarm_sim.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    """Build csrc/libsoarm_sim.so if missing or older than its sources."""
    if not force and not _stale():
        return LIB_PATH
    cmd = [HIPCC] + FLAGS + ["-o", LIB_PATH] + [os.path.join(SRC_DIR, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd, cwd=SRC_DIR)
    return LIB_PATH
