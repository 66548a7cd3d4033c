"""Paired tiles (nuts_device.hip "paired tiles", KParams::pair): when a launch's one-chain
tiles fit on the chip twice (2 x tiles <= CUs: config 2's 128 chains on 256 CUs, config 5's
8-GPU share, the reference's own 4-chain call, server.R:469), each tile's trajectory grows
its forward end in a partner workgroup with its own four gradient waves; bridge waves in
the two tiles carry the transition's start, the booking's progress and the subtree records
through write-through (sc1) global memory.

The partner runs the same producer on the same values, so draws, step sizes, metrics, last
positions and leapfrog counts must equal the unpaired two-ended path (FITOCT_NO_PAIR=1) and
the one-ended path (FITOCT_NO_BIDI=1) bit for bit -- for every prior family, deep trees
(one count guards the three slots of a subtree record's path), tile counts that are not a
multiple of 8 (padding blocks), batches, and when partners never join
(FITOCT_TEST_PAIR_ABSENT=1: every primary grows both ends itself after the hand-shake)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from fitoct_amd import Batch, Plan, SamplerConfig
from test_gpu_sampler import _prob

pytestmark = pytest.mark.gpu

ENV = ("FITOCT_PAIR", "FITOCT_NO_PAIR", "FITOCT_NO_BIDI", "FITOCT_TEST_PAIR_ABSENT", "FITOCT_NO_SPEC")


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in ENV}
    try:
        for k in ENV:
            os.environ.pop(k, None)
        os.environ.update({k: v for k, v in env.items() if v is not None})
        return fn()
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


def _plan_run(prob, cfg, **env):
    def go():
        with Plan(prob, cfg) as pl:
            pl.run()
            return pl.info, pl.download()
    return _with_env(env, go)


def _same(a, b):
    np.testing.assert_array_equal(a.draws, b.draws)
    np.testing.assert_array_equal(a.stepsize, b.stepsize)
    np.testing.assert_array_equal(a.inv_metric, b.inv_metric)
    np.testing.assert_array_equal(a.last_q, b.last_q)
    assert a.total_leapfrogs == b.total_leapfrogs


@pytest.mark.parametrize("family,N,chains,depth", [
    ("normal", 512, 128, 10),     # config 2's shape: 128 tiles -> 256 workgroups
    ("lasso", 300, 24, 8),        # 24 tiles: the last group of 8 is whole
    ("horseshoe", 2048, 37, 8),   # 37 tiles: padding blocks in the last group of 16
    ("normal", 481, 4, 10),       # the reference's 4-chain call (server.R:469)
    ("horseshoe", 512, 16, 12),   # deep trees: the record slot throttles the producers
])
def test_paired_tiles_preserve_draws_bitwise(family, N, chains, depth):
    prob = _prob(family, N, 15)
    cfg = SamplerConfig(chains=chains, warmup=80, samples=60, seed=41, max_treedepth=depth)
    info, a = _plan_run(prob, cfg, FITOCT_PAIR="1")   # (row mode pairs only on request)
    i1, b = _plan_run(prob, cfg, FITOCT_NO_PAIR="1")
    i2, c = _plan_run(prob, cfg, FITOCT_NO_BIDI="1")
    assert info["chains_per_tile"] == 1 and info["two_ended"] == 1 and info["paired"] == 1
    assert info["workgroups"] == 16 * ((info["tiles"] + 7) // 8)
    assert i1["paired"] == 0 and i1["workgroups"] == i1["tiles"] and i2["paired"] == 0
    # every two-ended transition of a resident pair grows its forward end in the partner
    assert a.two_ended_transitions > 0
    assert a.paired_transitions == a.two_ended_transitions, (a.paired_transitions,
                                                             a.two_ended_transitions)
    assert b.paired_transitions == 0 and c.paired_transitions == 0
    assert b.two_ended_transitions == a.two_ended_transitions
    _same(a, b)
    _same(a, c)


def test_absent_partners_leave_the_primary_to_grow_both_ends():
    """FITOCT_TEST_PAIR_ABSENT=1: every partner tile leaves at once without joining, as one
    that gets no CU at launch would.  Each primary's hand-shake at its first transition then
    finds no partner and grows both ends itself: no wait, no timeout, the same draws and no
    paired transition."""
    prob = _prob("normal", 512, 15)
    cfg = SamplerConfig(chains=64, warmup=60, samples=40, seed=43, max_treedepth=8)
    info, a = _plan_run(prob, cfg, FITOCT_TEST_PAIR_ABSENT="1", FITOCT_PAIR="1")
    _, b = _plan_run(prob, cfg, FITOCT_NO_PAIR="1")
    assert info["paired"] == 1
    assert a.paired_transitions == 0 and a.two_ended_transitions > 0
    _same(a, b)


def test_batch_of_one_chain_tiles_pairs_bitwise():
    """A batch whose tiles host one chain each (config 5's 8-GPU share: 32 files x 4 chains)
    pairs its tiles across problems: same draws per problem as without pairing."""
    probs = [_prob("normal", 481, 15, seed=300 + f) for f in range(32)]
    cfg = SamplerConfig(chains=4, warmup=40, samples=30, seed=17)

    def go():
        with Batch(probs, cfg) as b:
            b.run()
            return b.info, [b.download(p) for p in range(len(probs))]
    ia, a = _with_env({"FITOCT_PAIR": "1"}, go)
    ib, b = _with_env({"FITOCT_NO_PAIR": "1"}, go)
    assert ia["chains_per_tile"] == 1 and ia["paired"] == 1 and ib["paired"] == 0
    assert ia["workgroups"] == 256 and ib["workgroups"] == 128
    assert sum(x.paired_transitions for x in a) > 0
    for x, y in zip(a, b):
        _same(x, y)


def test_pairs_off_where_twice_the_tiles_do_not_fit():
    """256 one-chain tiles fill the 256 CUs: no partner would get a CU, so the plan does not
    pair (and 129..256 chains keep their one-tile two-ended path)."""
    prob = _prob("normal", 512, 15)
    cfg = SamplerConfig(chains=200, warmup=10, samples=10, seed=1, max_treedepth=6)
    info, a = _plan_run(prob, cfg)
    assert info["chains_per_tile"] == 1 and info["two_ended"] == 1
    assert info["paired"] == 0 and a.paired_transitions == 0


def test_pairing_default_follows_the_basis_mode():
    """By default one-chain tiles pair only with the factorised basis (N > 512): with the basis
    rows (N <= 512) an unpaired tile, whose chain's wave books the forward end, is faster
    (config 2: 253 k vs 245 k draws/s, profiles/r06_ab_unpaired.txt); FITOCT_PAIR=1 pairs it."""
    cfg = SamplerConfig(chains=16, warmup=10, samples=10, seed=3, max_treedepth=6)
    info, _ = _plan_run(_prob("normal", 512, 15), cfg)
    assert info["basis_mode"] == 1 and info["two_ended"] == 1 and info["paired"] == 0
    info, _ = _plan_run(_prob("normal", 512, 15), cfg, FITOCT_PAIR="1")
    assert info["paired"] == 1
    info, _ = _plan_run(_prob("horseshoe", 2048, 15), cfg)
    assert info["basis_mode"] == 0 and info["paired"] == 1
