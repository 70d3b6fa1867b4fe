"""Compile the HIP C-ABI library in-tree for gfx950 (no JIT caches).

Staleness is decided by content, not file times: the build writes
``libsoarm_sim.so.srchash`` (sha256 of the sources, headers and flags it was
built from) beside the library, so a tree copied to another box (where file
times may not survive) still knows whether its library matches its sources,
and a header edit is never benchmarked against a stale library.
"""
import hashlib
import os
import subprocess
import time

from .abi import LIB_PATH, PKG_DIR

SRC_DIR = os.path.join(PKG_DIR, "csrc")
SOURCES = ["soarm_sim.hip", "koopman_mpc.hip", "soarm_cpu.hip"]
# translation units compiled for the host only (the CPU backend: no kernels)
HOST_ONLY = {"soarm_cpu.hip"}
HEADERS = ["dmodel.h", "soarm_kernels.h", "soarm_step.h", "soarm_collide.h", "soarm_pgs.h", "soarm_newton.h",
           "soarm_substep.h",
           "soarm_env.h", "sim_internal.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -fno-slp-vectorize: the per-lane algebra gains nothing from v_pk_* packing; the
# packing's operand shuffles (v_mov) and the extra register pressure (AGPR
# round trips) cost ~13% of the PGS sweep's VALU issue (ISA count, k_substep).
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize"]
STAMP = LIB_PATH + ".srchash"


def source_hash():
    """sha256 over the flags and every source/header the library is built from."""
    h = hashlib.sha256(" ".join(FLAGS).encode())
    deps = [os.path.join(SRC_DIR, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(PKG_DIR, "..", "include", h) for h in ("soarm_sim.h", "koopman_mpc.h")]
    for d in deps:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def built_hash():
    try:
        with open(STAMP) as f:
            return f.read().strip()
    except OSError:
        return None


def _stale():
    return not os.path.exists(LIB_PATH) or built_hash() != source_hash()


def compile_lib(out, defines=(), verbose=False):
    """Compile every translation unit (concurrently) and link `out`; defines: extra -D flags
    (the diagnostic builds of tools/phase_prof.py and tools/bl_prof.py)."""
    out = os.path.abspath(out)  # (hipcc runs in csrc/)
    tmp = f"{out}.{os.getpid()}.tmp"
    cflags = [f for f in FLAGS if f != "-shared"] + list(defines)
    objs, procs = [], []
    for src in SOURCES:
        obj = f"{tmp}.{os.path.splitext(src)[0]}.o"
        extra = ["-x", "hip", "--offload-host-only"] if src in HOST_ONLY else []
        cmd = [HIPCC] + cflags + extra + ["-c", os.path.join(SRC_DIR, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        objs.append(obj)
        procs.append(subprocess.Popen(cmd, cwd=SRC_DIR))
    try:
        rcs = [p.wait() for p in procs]
        if any(rcs):
            raise subprocess.CalledProcessError(max(rcs, key=abs), "hipcc")
        cmd = [HIPCC] + FLAGS + ["-o", tmp] + objs + ["-lpthread"]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd, cwd=SRC_DIR)
    finally:
        for o in objs:
            if os.path.exists(o):
                os.remove(o)
    os.replace(tmp, out)  # atomic: concurrent loaders never see a partial file
    return out


def build(force=False, verbose=False):
    """Build csrc/libsoarm_sim.so if missing or built from other sources."""
    if not force and not _stale():
        return LIB_PATH
    want = source_hash()
    compile_lib(LIB_PATH, verbose=verbose)
    with open(STAMP + f".{os.getpid()}.tmp", "w") as f:
        f.write(want + "\n")
    os.replace(STAMP + f".{os.getpid()}.tmp", STAMP)
    return LIB_PATH


def ensure_built(local_rank=0, timeout_s=900):
    """Multi-process entry (bench under torch.distributed.run): local rank 0 (re)builds the
    library if it is missing or stale; the other ranks wait until the library on disk
    matches the sources."""
    if local_rank == 0:
        return build()
    want, t0 = source_hash(), time.time()
    while not (os.path.exists(LIB_PATH) and built_hash() == want):
        if time.time() - t0 > timeout_s:
            raise RuntimeError(f"{LIB_PATH} was not (re)built by local rank 0 within {timeout_s} s")
        time.sleep(1.0)
    return LIB_PATH


def library_info():
    """What the bench line records about the library it measured."""
    st = os.stat(LIB_PATH)
    return {"path": os.path.relpath(LIB_PATH, os.path.join(PKG_DIR, "..")), "mtime": st.st_mtime,
            "srchash": (built_hash() or "")[:16], "fresh": built_hash() == source_hash()}
