"""ORACLE (test infrastructure only) -- libfitoct's host drivers (L-BFGS and
ADVI, fitoct_amd/csrc/optimize.cpp) linked against a CPU evaluator of the C
oracle density (oracle/evaluator_shim.c) -> oracle/build/libdrivers_cpu.so.

:func:`patched` makes :mod:`fitoct_amd.optim_vb` call these drivers, so the CPU
suite covers the drivers' logic; the GPU tests run the same drivers over the
HIP evaluator.  Only tests/ may import this module.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

from . import nuts_c

LIB = os.path.join(nuts_c.BUILD_DIR, "libdrivers_cpu.so")
_L = None
NAMES = ("fitoct_optimize", "fitoct_vb", "fitoct_default_optim_config",
         "fitoct_default_vb_config", "fitoct_evaluator_create", "fitoct_evaluator_run",
         "fitoct_evaluator_destroy", "fitoct_constrain", "fitoct_last_error")


def lib():
    global _L
    if _L is None:
        nuts_c.build()
        from fitoct_amd import _lib
        L = C.CDLL(LIB)
        for name, res, args in _lib.SIGNATURES:
            if name in NAMES:
                f = getattr(L, name)
                f.restype, f.argtypes = res, args
        _L = L
    return _L


class _Composite:
    """The drivers from the CPU library, everything else from libfitoct."""

    def __init__(self, real):
        self._real = real

    def __getattr__(self, name):
        return getattr(lib() if name in NAMES else self._real, name)


@contextlib.contextmanager
def patched():
    from fitoct_amd import _lib, optim_vb
    comp = _Composite(_lib.lib())
    saved = (optim_vb.lib, _lib.lib)
    optim_vb.lib = lambda: comp
    _lib.lib = lambda: comp          # check() reads fitoct_last_error through it
    try:
        yield
    finally:
        optim_vb.lib, _lib.lib = saved
