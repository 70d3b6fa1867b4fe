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
    tmp = f"{LIB_PATH}.{os.getpid()}.tmp"
    cmd = [HIPCC] + FLAGS + ["-o", tmp] + [os.path.join(SRC_DIR, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd, cwd=SRC_DIR)
    os.replace(tmp, LIB_PATH)  # atomic: concurrent loaders never see a partial file
    return LIB_PATH


def ensure_built(local_rank=0, timeout_s=600):
    """Multi-process entry (bench under torch.distributed.run): never rebuild a library
    that exists (file times may not survive a copy to another box); if it is missing,
    local rank 0 builds it and the other ranks wait for it."""
    import time

    if os.path.exists(LIB_PATH):
        return LIB_PATH
    if local_rank == 0:
        return build(force=True)
    t0 = time.time()
    while not os.path.exists(LIB_PATH):
        if time.time() - t0 > timeout_s:
            raise RuntimeError(f"{LIB_PATH} did not appear (built by local rank 0)")
        time.sleep(1.0)
    return LIB_PATH
