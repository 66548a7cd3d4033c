"""HIP NUTS sampler (nuts_kernel) vs the C oracle and known answers.

Parity criteria (the oracle replays Stan's algorithm with the same Philox
addressing, so the two are the same Markov chain up to floating-point
rounding; HMC trajectories amplify a last-ulp difference chaotically, so
draw-by-draw equality only holds over a leading horizon):

1. Leading-horizon identity, as a statistic over chains: at least ``FRAC_ALL``
   of the chains agree with the oracle to 1e-6 relative in every column (lp__,
   the sampler diagnostics, parameters, br) for the first ``H_ALL`` stored
   iterations, the median chain for ``H_MED``, and every chain for its first stored
   iteration (init and chain addressing are exact).  A fixed per-chain horizon
   guarded bit patterns rather than correctness: one borderline chain's first
   mismatch moves whenever the sweep's last bits change (e.g. a 1-ulp more
   accurate exp), while the statistic stays put.
2. Distributional parity: per-parameter posterior means within 4.5 combined
   Monte-Carlo standard errors (n_eff from split chains); theta and sigma means
   within 1% (north-star tolerance) at the headline shape.
3. Known answers (prior-only, tests/kat_cases.py) on the GPU path.
4. Chain addressing: results per global chain id are bit-identical whatever
   the chain count per launch or the chain offset (sharding / tile packing).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import kat_cases as K
from conftest import golden_files, load_golden
from fitoct_amd import ExpGPProblem, Plan, SamplerConfig, sample
from fitoct_amd.stanfit import split_rhat_ess
from fitoct_amd.synth import default_prior, synth_decay
from oracle import nuts_c

pytestmark = pytest.mark.gpu

H_ALL, H_MED, FRAC_ALL = 4, 10, 0.9
NTHREADS = 16


def horizon_ok(fm):
    """The leading-horizon statistic of the module docstring (criterion 1), plus every
    chain's first stored iteration: an init or addressing error (a partial last tile,
    chain_offset, warm-restart indexing) then fails deterministically, however few chains
    it hits."""
    return np.mean(fm >= H_ALL) >= FRAC_ALL and np.median(fm) >= H_MED and fm.min() >= 1


def first_mismatch(a, b, rtol=1e-6):
    rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-12)
    rel = np.where(np.isnan(a) & np.isnan(b), 0.0, rel)
    bad = (rel > rtol).any(axis=2)
    return np.array([int(np.argmax(r)) if r.any() else a.shape[1] for r in bad])


def _prob(family, N, Nn, seed=11, mod="sincExp", **kw):
    t0, S0 = default_prior()
    d = synth_decay(N, mod, seed)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=family, **kw)


@pytest.mark.parametrize("path", golden_files("draws"), ids=lambda p: os.path.basename(p))
def test_reproduces_oracle_draw_fixture(path):
    fx = load_golden(path)
    m = fx["meta"]
    prob = ExpGPProblem(fx["x"], fx["y"], fx["uy"], Nn=m["Nn"], gridType=m["grid_type"],
                        theta0=fx["theta0"], Sigma0=fx["Sigma0"], prior_type=m["family"])
    cfg = SamplerConfig(chains=m["chains"], warmup=m["warmup"], samples=m["samples"],
                        seed=m["seed"], max_treedepth=m["max_treedepth"])
    out = sample(prob, cfg)
    fm = first_mismatch(out.draws, fx["draws"])
    assert horizon_ok(fm), fm.tolist()


CASES = [("normal", 256, 10, 150, 100, 64), ("horseshoe", 300, 8, 150, 100, 64),
         ("lasso", 200, 12, 100, 100, 64), ("normal", 1000, 15, 150, 60, 32),
         ("horseshoe", 2048, 15, 100, 40, 32),
         ("lasso", 3001, 15, 100, 40, 32)]   # 16 bins per lane (compact layout) with padding


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-N{c[1]}")
def test_leading_horizon_and_distribution(case):
    fam, N, Nn, W, S, C = case
    prob = _prob(fam, N, Nn)
    cfg = SamplerConfig(chains=C, warmup=W, samples=S, seed=77, max_treedepth=8)
    g = sample(prob, cfg)
    o = nuts_c.sample(prob, cfg, nthreads=NTHREADS)
    fm = first_mismatch(g.draws, o["draws"])
    assert horizon_ok(fm), fm.tolist()
    # leapfrog budget: same algorithm -> same work to within a few percent
    lf_o = int(o["leapfrogs"].sum())
    assert abs(g.total_leapfrogs - lf_o) <= 0.1 * lf_o
    assert np.all(g.stepsize > 0) and np.all(np.isfinite(g.inv_metric))


def _bench_problem(prior, N):
    """bench.py's synthetic input at a BASELINE config shape (restated synthData.R
    'sincExp' decay, data seed 1234, Nn = 15 extremal)."""
    return _prob(prior, N, 15, seed=1234, lambda_scale=10.0, nu=1.0)


@pytest.mark.parametrize("config", [2, 4])
def test_config_shapes_match_oracle(config):
    """The exact BASELINE config shapes the bench measures, against the oracle:
    config 2 (normal, N = 512, Nn = 15, 128 chains: one chain per tile, G = 1) and
    config 4 (lasso, N = 4096, Nn = 15: 16 bins per lane, the compact BPT = 16
    instantiation).  Leading horizon, leapfrog budget, median adapted step size."""
    prior, N, C = {2: ("normal", 512, 128), 4: ("lasso", 4096, 32)}[config]
    prob = _bench_problem(prior, N)
    cfg = SamplerConfig(chains=C, warmup=150, samples=60, seed=1000, max_treedepth=10)
    with Plan(prob, cfg) as pl:
        assert pl.info["bins_per_thread"] == (16 if config == 4 else 2)
        assert pl.info["chains_per_tile"] == 1
        pl.run()
        g = pl.download()
    o = nuts_c.sample(prob, cfg, nthreads=NTHREADS)
    fm = first_mismatch(g.draws, o["draws"])
    assert horizon_ok(fm), fm.tolist()
    lf_o = int(o["leapfrogs"].sum())
    assert abs(g.total_leapfrogs - lf_o) <= 0.1 * lf_o
    # adapted step sizes: the chains part ways after the horizon, so compare the spread
    ms_g, ms_o = np.median(g.stepsize), np.median(o["stepsize"])
    assert abs(ms_g - ms_o) <= 0.1 * ms_o, (ms_g, ms_o)


def _mean_parity(gd, od, W, cols, skip=()):
    fails = []
    for j, name in enumerate(cols):
        if j < 7 or name in skip:
            continue
        a, b = gd[:, W:, j], od[:, W:, j]
        if np.isnan(a).all():
            continue
        _, ea = split_rhat_ess(a)
        _, eb = split_rhat_ess(b)
        se = np.sqrt(a.var() / ea + b.var() / eb)
        if abs(a.mean() - b.mean()) > 4.5 * se + 1e-12 * abs(b.mean()):
            fails.append(f"{name}: gpu {a.mean():.6g} oracle {b.mean():.6g} se {se:.3g}")
    return fails


@pytest.mark.parametrize("fam", ["normal", "lasso", "horseshoe"])
def test_posterior_means_match_oracle(fam):
    prob = _prob(fam, 384, 10, seed=3, mod="sincExp1")
    cfg = SamplerConfig(chains=32, warmup=300, samples=400, seed=1234)
    g = sample(prob, cfg)
    cfg_o = SamplerConfig(chains=32, chain_offset=10_000, warmup=300, samples=400, seed=1234)
    o = nuts_c.sample(prob, cfg_o, nthreads=NTHREADS)   # independent chains (other ids)
    # heavy-tailed inverse-gamma auxiliaries have no finite mean: compare r1/z/theta/sigma/br
    cols = prob.column_names()
    skip = {c for c in cols if c.startswith("r2_")}
    fails = _mean_parity(g.draws, o["draws"], cfg.warmup, cols, skip)
    assert not fails, fails


@pytest.mark.parametrize("family", ["normal", "lasso", "horseshoe"])
def test_prior_known_answers_on_gpu(family):
    prob = K.problem(family)
    cfg = K.config(chains=32)
    out = sample(prob, cfg)
    fails = K.check(family, out.draws, prob.column_names(), cfg.warmup,
                    lambda x: split_rhat_ess(x)[1])
    assert not fails, fails


def test_testgamma_known_answer_on_gpu():
    """Tests/testGamma.R:19-47 on the HIP sampler at the reference's own settings and
    precision: 4 chains x (500 + 49,500) iterations, adapt_delta 0.99, max_treedepth 12,
    lambda ~ exponential(1/10) on each theta_k (mono-exponential model, theta_prior = 1,
    prior_PD = 1): mean = sd = 10 and median 10 ln 2 within 3 %, no divergences, split
    R-hat < 1.01 -- and the leading iterations are the C oracle's chain."""
    prob = K.gamma_problem()
    cfg = K.gamma_config()
    out = sample(prob, cfg)
    cols = prob.column_names()
    fails = K.gamma_check(out.draws, cols, cfg.warmup)
    assert not fails, fails
    post = out.draws[:, cfg.warmup:, :]
    assert post[:, :, 5].sum() == 0
    assert max(split_rhat_ess(post[:, :, cols.index(f"theta.{k}")])[0] for k in (1, 2, 3)) < 1.01
    short = SamplerConfig(chains=4, warmup=40, samples=20, seed=cfg.seed, adapt_delta=0.99,
                          max_treedepth=12)
    g, o = sample(prob, short).draws, nuts_c.sample(prob, short, nthreads=4)["draws"]
    np.testing.assert_allclose(g[:, :4, :], o[:, :4, :], rtol=1e-9, atol=1e-12)


def test_chain_addressing_is_schedule_independent():
    """1024 chains in one launch (4 chains per tile) vs 8-chain launches at
    offsets 0 and 517 (1 chain per tile): bit-identical per global chain id."""
    prob = _prob("horseshoe", 512, 8)
    base = dict(warmup=20, samples=10, seed=5, max_treedepth=6)
    big = sample(prob, SamplerConfig(chains=1024, **base))
    a = sample(prob, SamplerConfig(chains=8, **base))
    b = sample(prob, SamplerConfig(chains=8, chain_offset=517, **base))
    np.testing.assert_array_equal(big.draws[:8], a.draws)
    np.testing.assert_array_equal(big.draws[517:525], b.draws)
    np.testing.assert_array_equal(big.stepsize[517:525], b.stepsize)
    again = sample(prob, SamplerConfig(chains=8, **base))
    np.testing.assert_array_equal(a.draws, again.draws)


def test_plan_external_buffer_and_stream():
    """fitoct_plan_run into a caller-owned HBM buffer on a caller stream."""
    import torch
    prob = _prob("lasso", 700, 10)
    cfg = SamplerConfig(chains=64, warmup=60, samples=40, seed=9)
    ref = sample(prob, cfg)
    with Plan(prob, cfg) as pl:
        buf = torch.full((pl.info["draws_bytes"] // 8,), float("nan"), dtype=torch.float64,
                         device="cuda")
        s = torch.cuda.Stream()
        pl.run(d_draws=buf.data_ptr(), stream=s.cuda_stream)
        torch.cuda.synchronize()
        dev = buf.view(64, pl.info["iters_saved"], pl.info["n_cols"]).cpu().numpy()
        out = pl.download()
    np.testing.assert_array_equal(dev, ref.draws)
    np.testing.assert_array_equal(out.draws, ref.draws)


def test_mixed_precision_sampler_close_to_f64():
    prob = _prob("normal", 1024, 12, seed=4)
    c64 = SamplerConfig(chains=64, warmup=300, samples=300, seed=2)
    cmx = SamplerConfig(chains=64, warmup=300, samples=300, seed=2, precision="mixed")
    a, b = sample(prob, c64), sample(prob, cmx)
    cols = prob.column_names()
    fails = _mean_parity(a.draws, b.draws, 300, cols)
    assert not fails, fails


@pytest.mark.parametrize("seed", [1000, 1019])
def test_headline_shape_converges_and_matches_oracle(seed):
    """Config 3 (horseshoe, N=2048, Nn=15, 1024 chains, warmup 500 / 1000 draws) at
    rstan's default controls, on bench.py's own input and step seeds (1000: the first
    timed step and the rocprof profile; 1019: the last step of the driver's 20-step run,
    whose line is BENCH_r02's).

    The horseshoe's global/local-scale funnel traps ~1-2 % of chains at
    adapt_delta 0.8 (divergence rate > 50 %, acceptance < 0.3).  The C oracle
    reproduces the same rate on the same chain ids (e.g. chain 346 is stuck in
    both; 2/96 oracle vs 4/96 GPU chains over ids 300..395), so it
    is the algorithm's behaviour, not the port's.  Beyond the fully trapped chains,
    chains that visit the funnel's neck for part of the run inflate split R-hat of the
    funnel coordinates (z, r1_*): BENCH_r02 (seed 1019) measured split 1.037 / rank
    1.012 without the trapped chains.  Rank-normalised R-hat (Vehtari et al. 2021) is
    robust to those heavy tails and is what is asserted: < 1.015 over the bench's
    columns (theta, z, r1_*, sigma, br) without the trapped chains, at most 2.5 % trapped
    (the C oracle traps 8 of 512 = 1.6 % on the same problem and seed,
    tests/golden/trapped_headline.npz; tests/test_gpu_funnel.py compares the rates),
    and theta / sigma posterior means within 1 % of a 16-chain oracle run.  The
    north-star R-hat < 1.01 holds under the reference's hard-geometry profile (next
    test; bench.py's hard_geometry sub-line)."""
    from fitoct_amd.stanfit import rank_rhat
    prob = _bench_problem("horseshoe", 2048)
    cfg = SamplerConfig(chains=1024, warmup=500, samples=1000, seed=seed)
    g = sample(prob, cfg)
    cols = prob.column_names()
    W = cfg.warmup
    stuck = g.draws[:, W:, 5].mean(1) > 0.5
    assert stuck.mean() < 0.025, int(stuck.sum())
    keep = g.draws[~stuck, W:, :]
    rr = {n: rank_rhat(keep[:, :, j]) for j, n in enumerate(cols)
          if j >= 7 and not n.startswith("r2_")}
    assert max(rr.values()) < 1.015, sorted(rr.items(), key=lambda t: -t[1])[:5]
    if seed != 1000:
        return
    o = nuts_c.sample(prob, SamplerConfig(chains=NTHREADS, chain_offset=5000, warmup=500,
                                          samples=1000, seed=42), nthreads=NTHREADS)
    for name in ["theta.1", "theta.2", "theta.3", "sigma"]:
        j = cols.index(name)
        mg, mo = g.draws[:, W:, j].mean(), o["draws"][:, W:, j].mean()
        assert abs(mg - mo) <= 0.01 * abs(mo), (name, mg, mo)


@pytest.mark.parametrize("seed", [1000, 1001, 1019])
def test_headline_shape_hard_geometry_rhat_below_1_01(seed):
    """The north-star convergence target (max split R-hat < 1.01) at the headline shape,
    under the reference's own hard-geometry profile (Tests/testGamma.R:45: adapt_delta
    0.99, max_treedepth 12), 1024 chains, 500 warmup + 1000 draws.  bench.py's
    hard_geometry sub-line runs seed 1000 (fixed, bench.HARD_SEED); 1001 is the next step's
    seed and 1019 the last step of a 20-step run, where one chain fell into the horseshoe's
    funnel in the second half of sampling (round 4).

    Properties (no chain id, no bit pattern: a last-bit change to the sweep moves which
    chain traps, not whether the statements hold):
    - at most 0.3 % of the chains (3 of 1024) are trapped by the fixed rule
      (fitoct_amd.stanfit.trapped_chains: > 50 % divergent over the run or either half);
    - (rounds 4-5 also asserted that a trapped chain stays trapped; round 6's per-subtree
      acceptance sums moved the last bits, and at seed 1000 a chain 84 % divergent in the
      first half of its draws escaped the funnel's neck in the second (0.2 %): the neck is
      not absorbing, so that is no property of the sampler);
    - split and rank-normalised R-hat < 1.01 over the other chains, every parameter column
      but the inverse-gamma auxiliaries r2_*;
    - at the bench's seed, R-hat < 1.01 over ALL chains (the bench line's claim), and
      divergences stay ~1 %."""
    from fitoct_amd.stanfit import rank_rhat, trapped_chains
    prob = _bench_problem("horseshoe", 2048)
    cfg = SamplerConfig(chains=1024, warmup=500, samples=1000, seed=seed, adapt_delta=0.99,
                        max_treedepth=12)
    g = sample(prob, cfg)
    post = g.draws[:, cfg.warmup:, :]
    div = post[:, :, 5]
    trapped = trapped_chains(div)
    assert trapped.sum() <= 3, np.where(trapped)[0]
    assert div[~trapped].mean() < 0.03
    cols = prob.column_names()
    par = [j for j, n in enumerate(cols) if j >= 7 and not n.startswith("r2_")]
    for keep in ([post[~trapped]] + ([post] if seed == 1000 else [])):
        rh = {cols[j]: split_rhat_ess(keep[:, :, j])[0] for j in par}
        rr = {cols[j]: rank_rhat(keep[:, :, j]) for j in par}
        assert max(rh.values()) < 1.01, sorted(rh.items(), key=lambda t: -t[1])[:5]
        assert max(rr.values()) < 1.01, sorted(rr.items(), key=lambda t: -t[1])[:5]
