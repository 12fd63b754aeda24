"""Build libgibbs_hip.so in-tree for gfx950 (hipcc, no JIT cache)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", "gs_kernels.hip"), os.path.join(HERE, "csrc", "gs_sht.hip"),
           os.path.join(HERE, "csrc", "gs_masked.hip")]
HEADERS = [os.path.join(HERE, "csrc", h) for h in ("gs_rng.h", "gs_common.h", "gs_bm_tables.h", "gs_block.h")] + \
    [os.path.join(ROOT, "include", "gibbs_capi.h")]
LIB = os.path.join(HERE, "libgibbs_hip.so")
ARCH = os.environ.get("GIBBS_OFFLOAD_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True):
    deps = SOURCES + HEADERS
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-I", os.path.join(ROOT, "include"), "-o", LIB + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force=True)
