"""Batch mode (fitoct_batch_*): FitOCT.R's per-file loop (FitOCT.R:70-124) as
one launch.  Parity criteria:

1. Addressing: problem p of a batch is the same Markov chain as a single plan of
   that problem with chain_offset = p * chains.  With a common bin layout the
   draws are bit-identical; when a problem is restaged to the batch's wider bin
   layout (a different bin-to-lane order, so different rounding in the sums) the
   leading-horizon criterion of test_gpu_sampler applies.
2. Each problem of a batch against the C oracle (leading horizon, same
   tolerances as test_gpu_sampler.py).
3. Problems that cannot share one kernel (different Nn / prior family) are
   rejected with FITOCT_E_ARG and a message.
"""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import Batch, ExpGPProblem, FitOCTError, Plan, SamplerConfig
from fitoct_amd.synth import MODULATIONS, default_prior, synth_decay
from oracle import nuts_c
from test_gpu_sampler import H_ALL, H_MED, first_mismatch

pytestmark = pytest.mark.gpu

MODS = MODULATIONS   # synthData.R:21,35,49,63


def _prob(N, mod, seed, family="normal", Nn=15):
    t0, S0 = default_prior()
    d = synth_decay(N, mod, seed)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=family)


def _single(prob, cfg, offset):
    c = SamplerConfig(**{**cfg.__dict__, "chain_offset": offset})
    with Plan(prob, c) as pl:
        pl.run()
        return pl.download()


def test_batch_equals_single_plans_bitwise():
    probs = [_prob(481, MODS[p % 4], 100 + p) for p in range(6)]
    cfg = SamplerConfig(chains=4, warmup=60, samples=40, seed=5, max_treedepth=6)
    with Batch(probs, cfg) as b:
        assert b.info["tiles"] * b.info["chains_per_tile"] >= 24
        b.run()
        outs = [b.download(p) for p in range(len(b))]
    for p, prob in enumerate(probs):
        ref = _single(prob, cfg, p * cfg.chains)
        np.testing.assert_array_equal(outs[p].draws, ref.draws)
        np.testing.assert_array_equal(outs[p].stepsize, ref.stepsize)
        assert outs[p].total_leapfrogs == ref.total_leapfrogs
        assert outs[p].chain_offset == p * cfg.chains


def test_batch_ragged_sizes_against_oracle():
    # N = 481 / 300 / 700: the batch runs every problem in the widest bin layout
    probs = [_prob(481, "sincExp", 1), _prob(300, "sincExp1", 2), _prob(700, "sincExp2", 3)]
    cfg = SamplerConfig(chains=4, warmup=80, samples=60, seed=9, max_treedepth=7)
    with Batch(probs, cfg) as b:
        assert b.info["bins_per_thread"] == 4
        b.run()
        outs = [b.download(p) for p in range(len(b))]
    for p, prob in enumerate(probs):
        c = SamplerConfig(**{**cfg.__dict__, "chain_offset": p * cfg.chains})
        o = nuts_c.sample(prob, c, nthreads=4)
        fm = first_mismatch(outs[p].draws, o["draws"])
        assert fm.min() >= H_ALL and np.median(fm) >= H_MED, (p, fm.tolist())


def test_batch_headline_tiling():
    # config 5 shape on one GPU, shortened: 256 files x 4 chains -> one tile per file
    probs = [_prob(481, MODS[p % 4], 1234 + p) for p in range(256)]
    cfg = SamplerConfig(chains=4, warmup=30, samples=20, seed=3, max_treedepth=5)
    with Batch(probs, cfg) as b:
        assert b.info["chains_per_tile"] == 4 and b.info["tiles"] == 256
        b.run()
        for p in (0, 131, 255):
            o = b.download(p)
            assert np.all(np.isfinite(o.draws[:, :, 0]))
            assert np.all(o.stepsize > 0)


def test_batch_rejects_mixed_models():
    probs = [_prob(300, "sincExp", 1), _prob(300, "sincExp", 2, Nn=10)]
    with pytest.raises(FitOCTError, match="share prior_type and Nn"):
        Batch(probs, SamplerConfig(chains=2, warmup=10, samples=10))
    probs = [_prob(300, "sincExp", 1), _prob(300, "sincExp", 2, family="lasso")]
    with pytest.raises(FitOCTError, match="share prior_type and Nn"):
        Batch(probs, SamplerConfig(chains=2, warmup=10, samples=10))


def test_basis_mode_rows_resident_up_to_512_bins():
    """N <= 512 (configs 2 and 5): the sweep reads the basis rows from registers (basis_mode
    1, 1-2 bins of 15 doubles per lane) and the sampler's leaf has no K^-1 products; wider
    problems use the factorised basis (basis_mode 0).  A batch takes one mode for all its
    problems: rows only if every problem has N <= 512 (`fitoct_plan_info::basis_mode`)."""
    cfg = SamplerConfig(chains=4, warmup=10, samples=10, seed=2, max_treedepth=5)
    for N, mode, bpt in ((481, 1, 2), (200, 1, 1), (512, 1, 2), (700, 0, 4), (2048, 0, 8)):
        with Plan(_prob(N, "sincExp", 7), cfg) as pl:
            assert (pl.info["basis_mode"], pl.info["bins_per_thread"]) == (mode, bpt), N
    with Batch([_prob(481, "sincExp", 1), _prob(200, "sincExp1", 2)], cfg) as b:
        assert (b.info["basis_mode"], b.info["bins_per_thread"]) == (1, 2)
    with Batch([_prob(481, "sincExp", 1), _prob(700, "sincExp1", 2)], cfg) as b:
        assert (b.info["basis_mode"], b.info["bins_per_thread"]) == (0, 4)
