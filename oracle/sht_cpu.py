"""ctypes wrapper of oracle/sht_cpu.cpp, the C++/OpenMP HEALPix SHT (TEST /
MEASUREMENT INFRASTRUCTURE: tests/, __graft_entry__ and bench.py's CPU
baseline only -- the product path never imports it).

Same interface and conventions as oracle/sht.py (healpy complex m-major
a_lm; 1-D map / alm = spin 0, [3, ...] = T,E,B <-> T,Q,U) plus ``comps=2``
(E,B <-> Q,U only), so callers can swap the dense oracle for it at sizes the
dense sums cannot reach.  Built by ``build()`` (below; __graft_entry__.build
calls it) into oracle/libsht_cpu.so with g++ -fopenmp.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "sht_cpu.cpp")
LIB = os.path.join(HERE, "libsht_cpu.so")
_lib = None


def build(force=False):
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        cmd = ["g++", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c++17", "-o", LIB + ".tmp", SRC]
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


def _load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(LIB)
        vp, ci = ctypes.c_void_p, ctypes.c_int
        lib.shtc_alm2map.argtypes = [ci, ci, ci, vp, vp, ci]
        lib.shtc_map2alm.argtypes = [ci, ci, ci, vp, vp, ci, ci]
        lib.shtc_alm2map.restype = lib.shtc_map2alm.restype = ci
        _lib = lib
    return _lib


def threads():
    """the worker count: min(CPU affinity, 32) -- 32 = one GPU's fair share of the
    8-GPU node's 256 cores"""
    return max(1, min(len(os.sched_getaffinity(0)), 32))


def nlm(lmax):
    return (lmax + 1) * (lmax + 2) // 2


def alm2map(alms, nside, lmax, comps=None, nthreads=None):
    """alms: complex [nlm] (T) or [ncomp, nlm] (comps 3: T,E,B; 2: E,B) -> maps."""
    a = np.ascontiguousarray(alms, dtype=np.complex128)
    one = a.ndim == 1
    a2 = a[None] if one else a
    comps = comps or (1 if one else (3 if a2.shape[0] == 3 else 2))
    nc = {1: 1, 2: 2, 3: 3}[comps]
    if a2.shape != (nc, nlm(lmax)):
        raise ValueError("alm shape does not match comps / lmax")
    out = np.empty((nc, 12 * nside * nside))
    rc = _load().shtc_alm2map(nside, lmax, comps, a2.ctypes.data, out.ctypes.data, nthreads or threads())
    if rc:
        raise RuntimeError("shtc_alm2map failed")
    return out[0] if one else out


def map2alm(maps, nside, lmax, iter=0, comps=None, nthreads=None):
    """healpy map2alm(iter) (use_weights=False): maps [Npix] (T) or [ncomp, Npix]."""
    m = np.ascontiguousarray(maps, dtype=np.float64)
    one = m.ndim == 1
    m2 = m[None] if one else m
    comps = comps or (1 if one else (3 if m2.shape[0] == 3 else 2))
    out = np.empty((m2.shape[0], nlm(lmax)), dtype=np.complex128)
    rc = _load().shtc_map2alm(nside, lmax, comps, m2.ctypes.data, out.ctypes.data, int(iter), nthreads or threads())
    if rc:
        raise RuntimeError("shtc_map2alm failed")
    return out[0] if one else out


class Auto:
    """oracle.sht's interface over this library, skipping the transform of an
    all-zero T row of a [3, ...] input (the EB problems carry a zero T row)."""

    @staticmethod
    def alm2map(alms, nside, lmax):
        a = np.asarray(alms)
        if a.ndim == 2 and a.shape[0] == 3 and not np.any(a[0]):
            out = np.zeros((3, 12 * nside * nside))
            out[1:] = alm2map(a[1:], nside, lmax, comps=2)
            return out
        return alm2map(a, nside, lmax)

    @staticmethod
    def map2alm(maps, nside, lmax, iter=0):
        m = np.asarray(maps)
        if m.ndim == 2 and m.shape[0] == 3 and not np.any(m[0]):
            out = np.zeros((3, nlm(lmax)), dtype=np.complex128)
            out[1:] = map2alm(m[1:], nside, lmax, iter=iter, comps=2)
            return out
        return map2alm(m, nside, lmax, iter=iter)
