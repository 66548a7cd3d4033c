"""ORACLE (test infrastructure only) -- ctypes wrapper of oracle/build/liboracle.so,
the C restatement of the ExpGP model and Stan's recursive NUTS (fitoct_oracle.c).

Parity status vs rstan: **parity unpinned** (see fitoct_oracle.c header).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# FITOCT_SANITIZE=1: the ASan/UBSan build (make -C oracle sanitize) in oracle/build_san/
SANITIZE = os.environ.get("FITOCT_SANITIZE", "0") not in ("", "0")
BUILD_DIR = os.path.join(HERE, "build_san" if SANITIZE else "build")
LIB = os.path.join(BUILD_DIR, "liboracle.so")
_L = None


_BUILT = False


def build(force: bool = False) -> str:
    """make -C oracle (once per process; make tracks the sources)."""
    global _BUILT
    if force or not _BUILT:
        subprocess.run(["make", "-s", "-C", HERE] + (["sanitize"] if SANITIZE else [])
                       + (["-B"] if force else []), check=True)
        _BUILT = True
    return LIB


def lib():
    global _L
    if _L is None:
        build()
        from fitoct_amd import _lib as abi   # ABI struct layouts (include/fitoct.h)
        L = C.CDLL(LIB)
        dp = C.POINTER(C.c_double)
        L.oracle_basis.argtypes = [C.POINTER(abi.Problem), dp]
        L.oracle_logp_grad.argtypes = [C.POINTER(abi.Problem), C.c_int, dp, dp, dp, dp]
        L.oracle_sample.argtypes = [C.POINTER(abi.Problem), C.POINTER(abi.Config), dp, dp, dp,
                                    C.POINTER(C.c_longlong), C.c_int]
        L.oracle_philox.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                    C.POINTER(C.c_uint32)]
        L.oracle_normals.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_int, dp]
        L.oracle_sample_init.argtypes = [C.POINTER(abi.Problem), C.POINTER(abi.Config), dp, dp,
                                         dp, C.POINTER(C.c_longlong), C.c_int, dp, dp, dp]
        _L = L
    return _L


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox(c, k, o)
    return list(o)


def normals(seed, stream, tag, it, s, D):
    out = np.empty(D)
    lib().oracle_normals(seed, stream, tag, it, s, D, _dp(out))
    return out


def basis(prob):
    """prob: fitoct_amd.ExpGPProblem"""
    B = np.zeros((prob.N, prob.Nn))
    p = prob.to_c()
    assert lib().oracle_basis(C.byref(p), _dp(B)) == 0
    return B


def logp_grad(prob, q):
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
    P, D = q.shape
    lp, g, s2 = np.zeros(P), np.zeros((P, D)), np.zeros(P)
    p = prob.to_c()
    assert lib().oracle_logp_grad(C.byref(p), P, _dp(q), _dp(lp), _dp(g), _dp(s2)) == 0
    return lp, g, s2


def sample(prob, cfg, nthreads: int = 0, q_init=None, init_stepsize=None, init_inv_metric=None):
    """prob: ExpGPProblem, cfg: SamplerConfig -> dict(draws, stepsize, inv_metric, leapfrogs).
    q_init [chains, D] / init_stepsize [chains] / init_inv_metric [chains, D]: the warm
    restart of fitoct_plan_set_init (None = the default start)."""
    D = prob.D
    arrs = [None if a is None else np.ascontiguousarray(a, dtype=np.float64)
            for a in (q_init, init_stepsize, init_inv_metric)]
    iters = cfg.warmup + cfg.samples if cfg.save_warmup else cfg.samples
    draws = np.full((cfg.chains, iters, D + 8), np.nan)
    eps = np.zeros(cfg.chains)
    minv = np.zeros((cfg.chains, D))
    lf = np.zeros(cfg.chains, dtype=np.int64)
    p, c = prob.to_c(), cfg.to_c()
    rc = lib().oracle_sample_init(C.byref(p), C.byref(c), _dp(draws), _dp(eps), _dp(minv),
                                  lf.ctypes.data_as(C.POINTER(C.c_longlong)), int(nthreads),
                                  *[None if a is None else _dp(a) for a in arrs])
    if rc != 0:
        raise RuntimeError(f"oracle_sample failed with status {rc}")
    return {"draws": draws, "stepsize": eps, "inv_metric": minv, "leapfrogs": lf}
