"""The R-free half of the R `.Call` shim (rshim/src/fitoct_drive.c), called through
ctypes as fitoct_R.c calls it from R: plan -> launch -> poll loop (progress lines,
user-interrupt checks) -> wait -> download -> destroy (errors,
threading, ownership; server.R:457-484 progress).

CPU: the driver builds against include/fitoct.h and the in-tree libfitoct, exports
its entry point, and passes argument / no-device errors through with nothing called
back.  GPU: a driven run's draws equal a plain Plan.run bit for bit with monotone
progress ending at the total, and an interrupt cancels the run (FITOCT_E_CANCELLED)
after the kernel drained.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np
import pytest

from fitoct_amd import _lib
from fitoct_amd.api import ExpGPProblem, Plan, SamplerConfig
from fitoct_amd.synth import default_prior, synth_decay
from rshim import build as rbuild

PROGRESS = C.CFUNCTYPE(None, C.c_void_p, C.c_int64, C.c_int64)
INTERRUPT = C.CFUNCTYPE(C.c_int32, C.c_void_p)


def _drive_lib():
    _lib.lib()   # libfitoct first (the driver's NEEDED entry resolves to the same object)
    L = C.CDLL(rbuild.build())
    L.fitoct_drive_sample.restype = C.c_int32
    L.fitoct_drive_sample.argtypes = [C.POINTER(_lib.Problem), C.POINTER(_lib.Config),
                                      C.POINTER(_lib.Result), C.c_int32, PROGRESS, INTERRUPT,
                                      C.c_void_p]
    return L


def _drive(prob, cfg, interrupt_after=None, poll_ms=5):
    """Run the driver; returns (status, draws, progress calls, interrupt polls)."""
    p, c = prob.to_c(), cfg.to_c()
    iters = cfg.warmup + cfg.samples
    draws = np.full((cfg.chains, iters, len(prob.column_names())), np.nan)
    eps = np.empty(cfg.chains)
    r = _lib.Result()
    r.draws = draws.ctypes.data_as(C.POINTER(C.c_double))
    r.draws_capacity = draws.size
    r.stepsize = eps.ctypes.data_as(C.POINTER(C.c_double))
    seen, polls = [], [0]

    def on_progress(_ctx, done, total):
        seen.append((done, total))

    def on_interrupt(_ctx):
        polls[0] += 1
        return int(interrupt_after is not None and seen and seen[-1][0] >= interrupt_after)

    cb_p, cb_i = PROGRESS(on_progress), INTERRUPT(on_interrupt)
    rc = _drive_lib().fitoct_drive_sample(C.byref(p), C.byref(c), C.byref(r), poll_ms, cb_p,
                                          cb_i, None)
    return rc, draws, seen, polls[0]


def _prob(N=512, Nn=10):
    t0, S0 = default_prior()
    d = synth_decay(N, "sincExp", 3)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="normal")


def test_driver_builds_and_exports():
    L = _drive_lib()
    assert hasattr(L, "fitoct_drive_sample")


def test_driver_passes_argument_errors_through():
    """chains = 0: FITOCT_E_ARG from plan creation, nothing launched or called back."""
    rc, _, seen, polls = _drive(_prob(N=64), SamplerConfig(chains=0, warmup=5, samples=5))
    assert rc == -1 and seen == [] and polls == 0
    assert b"chains" in _lib.lib().fitoct_last_error()


@pytest.mark.skipif(_lib.lib().fitoct_device_count() > 0, reason="a GPU is visible")
def test_driver_no_device():
    rc, _, seen, polls = _drive(_prob(N=64), SamplerConfig(chains=2, warmup=5, samples=5))
    assert rc == -3 and seen == [] and polls == 0


@pytest.mark.gpu
def test_driver_matches_plan_and_reports_progress():
    prob = _prob()
    cfg = SamplerConfig(chains=64, warmup=100, samples=100, seed=11, max_treedepth=8)
    rc, draws, seen, polls = _drive(prob, cfg)
    assert rc == 0, _lib.lib().fitoct_last_error()
    total = 64 * 200
    assert seen and seen[-1] == (total, total)
    dones = [d for d, _ in seen]
    assert all(b >= a for a, b in zip(dones, dones[1:])), "progress went backwards"
    assert polls >= 1
    with Plan(prob, cfg) as pl:
        pl.run()
        ref = pl.download()
    assert np.array_equal(draws, ref.draws, equal_nan=True)


@pytest.mark.gpu
def test_driver_interrupt_cancels_and_drains():
    """Sized so that a failed cancellation would still end within ~30 s."""
    prob = _prob()
    cfg = SamplerConfig(chains=32, warmup=100, samples=20000, seed=12, max_treedepth=8)
    t0 = time.time()
    rc, _, seen, polls = _drive(prob, cfg, interrupt_after=32 * 16)
    dt = time.time() - t0
    assert rc == -8
    assert seen and seen[-1][0] < seen[-1][1]
    assert dt < 20.0, f"interrupted run took {dt:.1f} s"
    # the library is usable afterwards (no leaked plan state)
    rc2, _, seen2, _ = _drive(prob, SamplerConfig(chains=4, warmup=20, samples=20, seed=13,
                                                  max_treedepth=6))
    assert rc2 == 0 and seen2[-1] == (160, 160)
