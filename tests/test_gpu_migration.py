"""Chain migration between tiles (work balance, nuts_device.hip try_donate /
receive_chain): a chain handed to another tile at a transition boundary must
produce exactly the draws it produces without migration (same arithmetic in
every tile, Philox addressed by global chain id and iteration), and the
hand-over must actually happen when tiles finish unevenly."""
from __future__ import annotations

import os

import numpy as np
import pytest

from fitoct_amd import Plan, SamplerConfig
from test_gpu_sampler import _prob

pytestmark = pytest.mark.gpu


def _run(prob, cfg, migrate):
    old = os.environ.pop("FITOCT_NO_MIGRATE", None)
    if not migrate:
        os.environ["FITOCT_NO_MIGRATE"] = "1"
    try:
        with Plan(prob, cfg) as pl:
            pl.run()
            return pl.info, pl.download()
    finally:
        os.environ.pop("FITOCT_NO_MIGRATE", None)
        if old is not None:
            os.environ["FITOCT_NO_MIGRATE"] = old


@pytest.mark.parametrize("family,N", [("horseshoe", 512), ("normal", 2048), ("lasso", 1024)])
def test_migration_preserves_draws_bitwise(family, N):
    prob = _prob(family, N, 15)
    cfg = SamplerConfig(chains=1024, warmup=100, samples=100, seed=21, max_treedepth=7)
    info, a = _run(prob, cfg, migrate=True)
    _, b = _run(prob, cfg, migrate=False)
    assert info["chains_per_tile"] == 4
    assert b.migrations == 0
    assert a.migrations > 0, "no chain was handed over"
    np.testing.assert_array_equal(a.draws, b.draws)
    np.testing.assert_array_equal(a.stepsize, b.stepsize)
    np.testing.assert_array_equal(a.inv_metric, b.inv_metric)
    np.testing.assert_array_equal(a.last_q, b.last_q)
    assert a.total_leapfrogs == b.total_leapfrogs


def _run_env(prob, cfg, **env):
    old = {k: os.environ.get(k) for k in env}
    try:
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        with Plan(prob, cfg) as pl:
            pl.run()
            return pl.info, pl.download()
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


@pytest.mark.parametrize("family,N,left", [("horseshoe", 2048, None),
                                           ("normal", 512, None),
                                           ("lasso", 1024, "256"),
                                           ("normal", 512, "512")])
def test_tail_two_ended_preserves_draws_bitwise(family, N, left):
    """The launch's tail (nuts_device.hip receive_chain, P.tail_bidi): once at most
    tail_left chains are unfinished (default: every chain of the launch; 256: one per
    tile), a chain alone in its migrating tile recruits two idle receivers of the tile as
    producers and grows both trajectory ends at once, booking the leaves itself.  Draws,
    step sizes, metrics, last positions and leapfrog counts equal those of the same launch
    without it (FITOCT_NO_TAIL_BIDI=1) and without migration at all, and the run reports
    two-ended transitions."""
    prob = _prob(family, N, 15)
    cfg = SamplerConfig(chains=1024, warmup=100, samples=100, seed=23, max_treedepth=8)
    info, a = _run_env(prob, cfg, FITOCT_NO_TAIL_BIDI=None, FITOCT_TAIL_LEFT=left,
                       FITOCT_NO_MIGRATE=None)
    _, b = _run_env(prob, cfg, FITOCT_NO_TAIL_BIDI="1", FITOCT_TAIL_LEFT=None,
                    FITOCT_NO_MIGRATE=None)
    _, c = _run_env(prob, cfg, FITOCT_NO_TAIL_BIDI=None, FITOCT_TAIL_LEFT=None,
                    FITOCT_NO_MIGRATE="1")
    assert info["chains_per_tile"] == 4 and info["sampler"] == 3
    assert a.two_ended_transitions > 0, "no tail transition was two-ended"
    assert b.two_ended_transitions == 0 and c.two_ended_transitions == 0
    for x in (b, c):
        np.testing.assert_array_equal(a.draws, x.draws)
        np.testing.assert_array_equal(a.stepsize, x.stepsize)
        np.testing.assert_array_equal(a.inv_metric, x.inv_metric)
        np.testing.assert_array_equal(a.last_q, x.last_q)
        assert a.total_leapfrogs == x.total_leapfrogs


def test_tail_producer_that_gives_up_leaves_no_lone_chain_waiting():
    """a tail producer idle past its bound (FITOCT_TEST_TAIL_IDLE_US=20: 20 us
    instead of minutes) leaves its role only while it holds the tile's TW_BUSY word, and
    withdraws it (TW_JOIN, its TW_CLAIM bit), so a lone chain never claims a pair with a
    producer missing and then waits for records that no wave will write (ERR_TIMEOUT on a
    healthy chain).  Producers come and go all through the tail here: every chain finishes,
    with the draws of the launch without two-ended tails."""
    prob = _prob("horseshoe", 512, 15)
    cfg = SamplerConfig(chains=1024, warmup=100, samples=100, seed=29, max_treedepth=8)
    info, a = _run_env(prob, cfg, FITOCT_NO_TAIL_BIDI=None, FITOCT_NO_MIGRATE=None,
                       FITOCT_TEST_TAIL_IDLE_US="20")
    _, b = _run_env(prob, cfg, FITOCT_NO_TAIL_BIDI="1", FITOCT_NO_MIGRATE=None,
                    FITOCT_TEST_TAIL_IDLE_US=None)
    assert info["two_ended"] == 2
    np.testing.assert_array_equal(a.draws, b.draws)
    np.testing.assert_array_equal(a.stepsize, b.stepsize)
    assert a.total_leapfrogs == b.total_leapfrogs
