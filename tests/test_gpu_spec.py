"""Speculative leaves (nuts_device.hip leaf_spec / act_spec_book and the helper wave):
with one chain per tile the next leapfrog position is swept while the current leaf's
merges and U-turn checks run, and a helper wave computes its prior part.  The draws
must equal the plain sampler's (FITOCT_NO_SPEC=1) bit for bit, trajectory ends
(discarded speculations) included, for every prior family."""
from __future__ import annotations

import os

import numpy as np
import pytest

from fitoct_amd import Plan, SamplerConfig
from test_gpu_sampler import _prob

pytestmark = pytest.mark.gpu


def _run(prob, cfg, spec):
    old = os.environ.pop("FITOCT_NO_SPEC", None)
    if not spec:
        os.environ["FITOCT_NO_SPEC"] = "1"
    try:
        with Plan(prob, cfg) as pl:
            pl.run()
            return pl.info, pl.download()
    finally:
        os.environ.pop("FITOCT_NO_SPEC", None)
        if old is not None:
            os.environ["FITOCT_NO_SPEC"] = old


@pytest.mark.parametrize("family,N,depth", [("normal", 512, 10), ("lasso", 300, 8),
                                            ("horseshoe", 2048, 8)])
def test_speculative_leaves_preserve_draws_bitwise(family, N, depth):
    prob = _prob(family, N, 15)
    cfg = SamplerConfig(chains=24, warmup=80, samples=60, seed=33, max_treedepth=depth)
    info, a = _run(prob, cfg, spec=True)
    info0, b = _run(prob, cfg, spec=False)
    assert info["chains_per_tile"] == 1
    assert info["sampler"] == 2 and info0["sampler"] == 0   # FITOCT_SAMPLER_SPECULATIVE / _PLAIN
    np.testing.assert_array_equal(a.draws, b.draws)
    np.testing.assert_array_equal(a.stepsize, b.stepsize)
    np.testing.assert_array_equal(a.inv_metric, b.inv_metric)
    assert a.total_leapfrogs == b.total_leapfrogs


def test_tiles_of_several_chains_do_not_speculate():
    prob = _prob("normal", 512, 15)
    cfg = SamplerConfig(chains=1024, warmup=10, samples=10, seed=3, max_treedepth=6)
    with Plan(prob, cfg) as pl:
        assert pl.info["chains_per_tile"] == 4 and pl.info["sampler"] != 2
