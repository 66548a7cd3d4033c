"""Speculative leaves (nuts_device.hip leaf_spec / act_spec_book and the helper wave):
with one chain per tile the next leapfrog position is swept while the current leaf's
merges and U-turn checks run, and a helper wave computes its prior part.  The draws
must equal the plain sampler's (FITOCT_NO_SPEC=1) bit for bit, trajectory ends
(discarded speculations) included, for every prior family; likewise in tiles of
several chains, migrating or not, where there is no helper wave and a chain speculates
only while its tile has thinned out (or at every leaf with FITOCT_SPEC=1)."""
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
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("live", [None, "4"])
def test_migrating_plans_speculate_in_the_tail_bitwise(live):
    """The headline sampler (MIGRATE_SPEC): tiles of four migrating chains speculate once
    they host <= 3 live chains (the launch's tail; FITOCT_SPEC_LIVE=4: at every leaf), a
    chain switching paths leaf by leaf and moving between tiles.  Same draws, step sizes,
    metrics and leapfrog counts as the plain migrating sampler."""
    prob = _prob("horseshoe", 2048, 15)
    cfg = SamplerConfig(chains=1024, warmup=60, samples=40, seed=3, max_treedepth=7)
    info, a = _run_env(prob, cfg, FITOCT_SPEC_LIVE=live, FITOCT_NO_SPEC=None)
    info0, b = _run_env(prob, cfg, FITOCT_SPEC_LIVE=None, FITOCT_NO_SPEC="1")
    assert info["chains_per_tile"] == 4 and info["sampler"] == 3   # MIGRATE_SPEC
    assert info0["sampler"] == 1                                   # MIGRATE
    np.testing.assert_array_equal(a.draws, b.draws)
    np.testing.assert_array_equal(a.stepsize, b.stepsize)
    np.testing.assert_array_equal(a.inv_metric, b.inv_metric)
    assert a.total_leapfrogs == b.total_leapfrogs
    assert a.migrations > 0 and b.migrations > 0


def test_tiles_of_several_chains_speculate_without_helper_bitwise():
    """With FITOCT_SPEC=1 and no migration, tiles of four chains take the speculative
    path with no helper wave: each chain's wave computes the weight and the next prior
    part itself (not the default: it is slower there).  Same draws as the plain sampler."""
    prob = _prob("horseshoe", 512, 15)
    cfg = SamplerConfig(chains=1024, warmup=40, samples=30, seed=5, max_treedepth=7)
    old = {k: os.environ.get(k) for k in ("FITOCT_NO_MIGRATE", "FITOCT_SPEC")}
    os.environ["FITOCT_NO_MIGRATE"] = "1"
    os.environ["FITOCT_SPEC"] = "1"
    try:
        info, a = _run(prob, cfg, spec=True)
        info0, b = _run(prob, cfg, spec=False)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert info["chains_per_tile"] == 4
    assert info["sampler"] == 2 and info0["sampler"] == 0
    np.testing.assert_array_equal(a.draws, b.draws)
    assert a.total_leapfrogs == b.total_leapfrogs


def test_batch_speculates_bitwise():
    """Batch tiles of four chains do not speculate by default (they lose 7 % with it,
    profiles/r03_ab_spec_live.txt); with FITOCT_SPEC=1 they do, bit for bit."""
    from fitoct_amd import sample_batch
    probs = [_prob("normal", 481, 15, seed=40 + f) for f in range(6)]
    cfg = SamplerConfig(chains=4, warmup=40, samples=30, seed=9)
    old = {k: os.environ.pop(k, None) for k in ("FITOCT_NO_SPEC", "FITOCT_SPEC")}
    try:
        os.environ["FITOCT_SPEC"] = "1"
        a = sample_batch(probs, cfg)
        os.environ.pop("FITOCT_SPEC")
        os.environ["FITOCT_NO_SPEC"] = "1"
        b = sample_batch(probs, cfg)
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.draws, y.draws)


def test_headline_tiles_fit_four_chains_at_depth_12():
    """The LDS carve of a tile decides how many chains it hosts: the headline shape must
    keep four chains per tile (1024 chains on 256 CUs, migration on) under the
    hard-geometry profile's max_treedepth 12 too (bench.py hard_geometry)."""
    prob = _prob("horseshoe", 2048, 15)
    for depth in (10, 12):
        cfg = SamplerConfig(chains=1024, warmup=10, samples=10, seed=3, max_treedepth=depth)
        with Plan(prob, cfg) as pl:
            assert pl.info["chains_per_tile"] == 4, (depth, pl.info)
            assert pl.info["sampler"] == 3 and pl.info["lds_bytes"] <= 160 * 1024


@pytest.mark.parametrize("family,N,Nn,depth", [
    ("normal", 512, 15, 10), ("normal", 512, 15, 4), ("horseshoe", 2048, 15, 8),
    ("lasso", 300, 15, 12), ("horseshoe", 2048, 15, 10),
    # Nn = 20: two parameters per lane (the ppl = 2 chain areas), shallow enough to fit
    ("normal", 512, 20, 6)])
def test_two_ended_trajectories_preserve_draws_bitwise(family, N, Nn, depth):
    """Tiles of one chain grow both ends of each trajectory at once: two producer waves build
    the subtrees of each direction whole (weights, merges, U-turn checks, proposal) in chain
    areas of their own and hand the chain's wave one record per subtree, which it books at the
    trajectory level in Stan's tree order (nuts_device.hip "two-ended trajectories").  Same
    draws, step sizes, metrics and leapfrog counts as the one-ended deep-speculation path
    (FITOCT_NO_BIDI=1), with trees cut at max_treedepth 4 and the ppl = 2 carve (Nn = 20).
    The plan reports the mode and its records in flight per end (ABI 7: one).  With up to
    128 such tiles on the chip the tiles are also paired (test_gpu_pair.py); here both."""
    prob = _prob(family, N, Nn)
    cfg = SamplerConfig(chains=24, warmup=80, samples=60, seed=35, max_treedepth=depth)
    for pair in (None, "1"):
        info, a = _run_env(prob, cfg, FITOCT_NO_BIDI=None, FITOCT_NO_PAIR=pair, FITOCT_NO_SPEC=None)
        info0, b = _run_env(prob, cfg, FITOCT_NO_BIDI="1", FITOCT_NO_PAIR=None, FITOCT_NO_SPEC=None)
        assert info["chains_per_tile"] == 1 and info["sampler"] == 2
        assert info["two_ended"] == 1 and info0["two_ended"] == 0 and info0["ring_records"] == 0
        assert info["ring_records"] == 1 and info["ring_records_in_levels"] == 0
        assert info["lds_bytes"] <= 160 * 1024 - 1024
        assert info["lds_bytes"] > info0["lds_bytes"]   # the producers' two chain areas
        assert a.two_ended_transitions > 0
        np.testing.assert_array_equal(a.draws, b.draws)
        np.testing.assert_array_equal(a.stepsize, b.stepsize)
        np.testing.assert_array_equal(a.inv_metric, b.inv_metric)
        assert a.total_leapfrogs == b.total_leapfrogs


def test_two_ended_off_where_three_chain_areas_do_not_fit():
    """Nn = 20 (two parameters per lane) at max_treedepth 10: three chain areas would take
    ~181 KB of the 160 KB of LDS, so the one-chain tiles stay on the one-ended path (round
    4 planned the two-ended carve anyway and the launch failed: ADVICE r4).  The reference's
    usual 4 chains run and match the plain sampler bit for bit."""
    prob = _prob("normal", 512, 20)
    cfg = SamplerConfig(chains=4, warmup=60, samples=40, seed=21, max_treedepth=10)
    info, a = _run_env(prob, cfg, FITOCT_NO_BIDI=None, FITOCT_NO_SPEC=None)
    assert info["chains_per_tile"] == 1 and info["two_ended"] == 0
    assert info["lds_bytes"] <= 160 * 1024
    _, b = _run_env(prob, cfg, FITOCT_NO_BIDI=None, FITOCT_NO_SPEC="1")
    np.testing.assert_array_equal(a.draws, b.draws)
    assert np.all(np.isfinite(a.draws[:, :, 0]))


def test_batch_of_one_chain_tiles_two_ended_bitwise():
    """A batch whose tiles host one chain each (few files: config 5 spread over 8 GPUs)
    takes the two-ended path per problem: same draws as without it."""
    from fitoct_amd import sample_batch
    probs = [_prob("normal", 481, 15, seed=60 + f) for f in range(5)]
    cfg = SamplerConfig(chains=4, warmup=40, samples=30, seed=11)
    old = {k: os.environ.pop(k, None) for k in ("FITOCT_NO_SPEC", "FITOCT_SPEC", "FITOCT_NO_BIDI")}
    try:
        a = sample_batch(probs, cfg)
        os.environ["FITOCT_NO_BIDI"] = "1"
        b = sample_batch(probs, cfg)
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.draws, y.draws)


@pytest.mark.parametrize("files,chains,env", [(80, 4, {}), (75, 4, {}),
                                              (1, 301, {"FITOCT_NO_MIGRATE": "1"})])
def test_two_chain_tiles_deep_speculation_bitwise(files, chains, env):
    """Tiles of two chains without migration (257..512 chains: config 5's per-GPU share at 2
    GPUs, 128 files x 4 chains) give each chain a spare NUTS wave as its helper (wave 2 + c
    books chain c's leaves while chain c's wave completes the next gradient and stages the
    one after): same draws, step sizes and leapfrog counts as the plain sampler, including
    a last tile that hosts one chain (301 chains)."""
    from fitoct_amd import Batch
    probs = [_prob("normal", 481, 15, seed=200 + f) for f in range(files)]
    cfg = SamplerConfig(chains=chains, warmup=40, samples=30, seed=13)
    outs = {}
    for spec in (True, False):
        old = {k: os.environ.get(k) for k in ("FITOCT_NO_SPEC", "FITOCT_SPEC", *env)}
        try:
            for k in old:
                os.environ.pop(k, None)
            os.environ.update(env)
            if not spec:
                os.environ["FITOCT_NO_SPEC"] = "1"
            with Batch(probs, cfg) as b:
                b.run()
                outs[spec] = (b.info, [b.download(p) for p in range(files)])
        finally:
            for k, v in old.items():
                os.environ.pop(k, None)
                if v is not None:
                    os.environ[k] = v
    (ia, a), (ib, b) = outs[True], outs[False]
    assert ia["chains_per_tile"] == 2 and ia["sampler"] == 2 and ib["sampler"] == 0
    assert ia["lds_bytes"] <= 160 * 1024
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x.draws, y.draws)
        np.testing.assert_array_equal(x.stepsize, y.stepsize)
        assert x.total_leapfrogs == y.total_leapfrogs
