"""Warm restart (fitoct_plan_set_init, SURVEY.md §5 "Checkpoint / resume"): a run starts
from given per-chain positions, step sizes and inverse metrics, e.g. a previous run's
last_q / stepsize / inv_metric.  The oracle restates the same start (oracle_set_init),
so the HIP chains and the oracle's are the same Markov chain from that start: the
leading-horizon statistic of test_gpu_sampler.py holds with and without adaptation.
"""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import Plan, SamplerConfig, sample
from fitoct_amd._lib import FitOCTError
from oracle import nuts_c
from test_gpu_sampler import NTHREADS, _prob, first_mismatch, horizon_ok

pytestmark = pytest.mark.gpu

C = 32


@pytest.fixture(scope="module")
def first_run():
    prob = _prob("normal", 256, 10)
    out = sample(prob, SamplerConfig(chains=C, warmup=150, samples=20, seed=5, max_treedepth=8))
    return prob, out


@pytest.mark.parametrize("adapt", [False, True], ids=["resume", "readapt"])
def test_warm_restart_matches_oracle(first_run, adapt):
    prob, prev = first_run
    cfg = SamplerConfig(chains=C, warmup=100 if adapt else 0, samples=60, seed=6,
                        max_treedepth=8, adapt_engaged=adapt)
    with Plan(prob, cfg) as pl:
        pl.set_init(prev.last_q, prev.stepsize, prev.inv_metric)
        pl.run()
        g = pl.download()
    o = nuts_c.sample(prob, cfg, nthreads=NTHREADS, q_init=prev.last_q,
                      init_stepsize=prev.stepsize, init_inv_metric=prev.inv_metric)
    fm = first_mismatch(g.draws, o["draws"])
    assert horizon_ok(fm), fm.tolist()
    if not adapt:   # the given step size and metric are used unchanged
        assert np.array_equal(g.stepsize, prev.stepsize)
        assert np.array_equal(g.inv_metric, prev.inv_metric)
        assert np.array_equal(g.draws[:, :, 2], np.repeat(prev.stepsize[:, None], 60, axis=1))
        # the chains start in the posterior's typical set: no burn-in transient in lp__
        lp_prev = prev.draws[:, -20:, 0].mean()
        assert abs(g.draws[:, :5, 0].mean() - lp_prev) < 5.0 * prev.draws[:, -20:, 0].std()


def test_resume_via_sample_and_clear(first_run):
    """sample(resume=...) equals the explicit set_init; set_init() with no arguments
    restores the default start (the same draws as a plan that never had one)."""
    prob, prev = first_run
    cfg = SamplerConfig(chains=C, warmup=0, samples=10, seed=8, max_treedepth=8,
                        adapt_engaged=False)
    a = sample(prob, cfg, resume=prev)
    with Plan(prob, cfg) as pl:
        pl.set_init(prev.last_q, prev.stepsize, prev.inv_metric)
        pl.run()
        b = pl.download()
        pl.set_init()
        pl.run()
        c = pl.download()
    assert np.array_equal(a.draws, b.draws)
    assert np.array_equal(c.draws, sample(prob, cfg).draws)


def test_warm_restart_argument_errors(first_run):
    prob, prev = first_run
    cfg = SamplerConfig(chains=C, warmup=0, samples=5, adapt_engaged=False)
    with Plan(prob, cfg) as pl:
        for kw in [dict(stepsize=np.zeros(C)), dict(inv_metric=-prev.inv_metric),
                   dict(q_init=np.full_like(prev.last_q, np.nan))]:
            with pytest.raises(FitOCTError) as ei:
                pl.set_init(**kw)
            assert ei.value.code == -1


def test_non_finite_start_fails_with_init_status(first_run):
    """A given start whose density is not finite is not retried: the chain reports
    FITOCT_E_INIT (-4), the others run."""
    prob, prev = first_run
    q = prev.last_q.copy()
    q[3, 0] = 800.0   # theta1 = exp(800) overflows: lp = -inf
    cfg = SamplerConfig(chains=C, warmup=0, samples=5, adapt_engaged=False)
    with Plan(prob, cfg) as pl:
        pl.set_init(q, prev.stepsize, prev.inv_metric)
        pl.run()
        with pytest.raises(FitOCTError) as ei:
            pl.download()
    assert ei.value.code == -4


def test_warm_restart_chain_addressing_across_kernels():
    """Resumed chains keep the chain-addressing invariance: a 600-chain horseshoe plan
    (several chains per tile, migrating kernel) resumed from a previous run's end state gives
    chains 0..7 the same draws, bit for bit, as an 8-chain plan (one chain per tile,
    speculative kernel) resumed from those chains' rows -- the start is read per chain
    of the launch in every kernel variant."""
    prob = _prob("horseshoe", 300, 8)
    prev = sample(prob, SamplerConfig(chains=600, warmup=80, samples=10, seed=31,
                                      max_treedepth=6))
    cfg = SamplerConfig(chains=600, warmup=0, samples=15, seed=32, max_treedepth=6,
                        adapt_engaged=False)
    with Plan(prob, cfg) as pl:
        assert pl.info["chains_per_tile"] >= 2 and pl.info["sampler"] == 3   # MIGRATE_SPEC
        pl.set_init(prev.last_q, prev.stepsize, prev.inv_metric)
        pl.run()
        big = pl.download()
    small_cfg = SamplerConfig(chains=8, warmup=0, samples=15, seed=32, max_treedepth=6,
                              adapt_engaged=False)
    with Plan(prob, small_cfg) as pl:
        assert pl.info["chains_per_tile"] == 1 and pl.info["sampler"] == 2   # SPECULATIVE
        pl.set_init(prev.last_q[:8], prev.stepsize[:8], prev.inv_metric[:8])
        pl.run()
        small = pl.download()
    assert np.array_equal(big.draws[:8], small.draws)
    assert np.array_equal(big.stepsize, prev.stepsize)
