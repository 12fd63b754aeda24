"""Build libgibbs_hip.so in-tree for gfx950 (hipcc, no JIT cache).

Variants (debug builds):
  * ``variant="debug"``: -DGS_DEBUG -- device-side bounds assertions (GS_ASSERT)
    at the kernels' index computations; -> libgibbs_hip_debug.so
  * ``variant="asan"``: host code under AddressSanitizer (-Xarch_host
    -fsanitize=address; device code unchanged) for the plan-building and
    argument-validation paths; -> libgibbs_hip_asan.so, loaded with the clang
    ASan runtime preloaded (tests/test_capi_asan.py)
  * ``variant="timeline"``: -DGS_MH_TIMELINE -- s_memrealtime stamps at the
    MH kernel's stage boundaries (gs_debug_mh_timeline; tools/mh_timeline.py)
Select a variant at run time with GIBBS_HIP_LIB=<path>.
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", "gs_kernels.hip"), os.path.join(HERE, "csrc", "gs_sht.hip"),
           os.path.join(HERE, "csrc", "gs_masked.hip")]
HEADERS = [os.path.join(HERE, "csrc", h) for h in ("gs_rng.h", "gs_common.h", "gs_bm_tables.h", "gs_block.h")] + \
    [os.path.join(ROOT, "include", "gibbs_capi.h")]
LIB = os.path.join(HERE, "libgibbs_hip.so")
ARCH = os.environ.get("GIBBS_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=on: a*b+c is fused only within one expression (decided by the
# source), never across statements (hipcc's default "fast-honor-pragmas" lets
# the backend fuse depending on the inlining context), so the same device
# function gives the same bits in every kernel that inlines it -- e.g. the
# sweep's latency and throughput forms, the in-sweep and tabulated CR operator
# (tests/test_gpu_graph.py::test_sweep_latency_form_bit_identical)
COMMON = ["-ffp-contract=on"]
VARIANTS = {
    None: (LIB, ["-O3"] + COMMON),
    "debug": (os.path.join(HERE, "libgibbs_hip_debug.so"), ["-O3", "-DGS_DEBUG"] + COMMON),
    "timeline": (os.path.join(HERE, "libgibbs_hip_timeline.so"), ["-O3", "-DGS_MH_TIMELINE"] + COMMON),
    "asan": (os.path.join(HERE, "libgibbs_hip_asan.so"),
             ["-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host", "-fsanitize=address", "-shared-libasan"] + COMMON),
}


def asan_runtime():
    """clang's shared ASan runtime that an ASan build needs preloaded."""
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, variant=None):
    lib, flags = VARIANTS[variant]
    deps = SOURCES + HEADERS + [os.path.abspath(__file__)]
    if not force and not _stale(lib, deps):
        return lib
    # one object per source, compiled in parallel (no device code crosses a
    # translation unit, so no -fgpu-rdc), then one link
    base = ["hipcc", f"--offload-arch={ARCH}"] + flags + ["-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include")]
    objs, procs = [], []
    for src in SOURCES:
        obj = lib + "." + os.path.splitext(os.path.basename(src))[0] + ".o"
        cmd = base + ["-c", "-o", obj, src]
        if verbose:   # stderr: a rebuild must never precede bench.py's JSON line on stdout
            print(" ".join(cmd), file=sys.stderr)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    bad = [p.wait() for p in procs]
    if any(bad):
        raise subprocess.CalledProcessError(max(bad), "hipcc -c")
    link = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp"] + objs
    if "-shared-libasan" in flags:
        link += ["-fsanitize=address", "-shared-libasan"]
    subprocess.run(link, check=True)
    for o in objs:
        os.remove(o)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    import sys
    build(force=True, variant=sys.argv[1] if len(sys.argv) > 1 else None)
