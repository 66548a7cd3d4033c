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


@pytest.mark.parametrize("family,N", [("horseshoe", 512), ("normal", 2048)])
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
