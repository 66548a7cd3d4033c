"""C-oracle NUTS (oracle/fitoct_oracle.c): prior-only known answers, chain
addressing (sharding invariance), determinism, and the committed draw fixtures.
(CPU only -- these pin the checker that the GPU tests compare against.)
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import kat_cases as K
from conftest import golden_files, load_golden
from fitoct_amd import ExpGPProblem, SamplerConfig
from oracle import diag_np, nuts_c


@pytest.mark.parametrize("family", ["normal", "lasso", "horseshoe"])
def test_prior_known_answers(family):
    prob = K.problem(family)
    cfg = K.config()
    o = nuts_c.sample(prob, cfg, nthreads=8)
    fails = K.check(family, o["draws"], prob.column_names(), cfg.warmup, diag_np.split_ess)
    assert not fails, fails
    # well-mixed: split R-hat on every parameter column (the normal family's
    # funnel lets a chain linger in the neck now and then: looser bound)
    post = o["draws"][:, cfg.warmup:, 7:-1]
    rh = [diag_np.split_rhat(post[:, :, j]) for j in range(post.shape[2])]
    assert max(rh) < (1.05 if family == "normal" else 1.01)


def test_testgamma_known_answer_at_reference_precision():
    """Tests/testGamma.R:19-47 at its own settings (4 chains x 49,500 draws, adapt_delta
    0.99, max_treedepth 12): lambda ~ exponential(1/10) on each theta_k of the
    mono-exponential model with theta_prior = 1 -- mean = sd = 10, median 10 ln 2
    within 3 %, no divergences (no funnel), every chain mixing."""
    prob = K.gamma_problem()
    cfg = K.gamma_config()
    o = nuts_c.sample(prob, cfg, nthreads=4)
    cols = prob.column_names()
    fails = K.gamma_check(o["draws"], cols, cfg.warmup)
    assert not fails, fails
    post = o["draws"][:, cfg.warmup:, :]
    assert post[:, :, 5].sum() == 0
    assert max(diag_np.split_rhat(post[:, :, cols.index(f"theta.{k}")]) for k in (1, 2, 3)) < 1.01


def _small(family="normal", N=48, Nn=5):
    from fitoct_amd.synth import default_prior, synth_decay
    t0, S0 = default_prior()
    d = synth_decay(N, "sincExp", 3)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=family)


def test_chain_addressing_is_shard_invariant():
    """Chains are keyed by (seed, chain_offset + local id): running [0,6) in one
    call equals [0,2) + [2,6) in two calls (what distributed sharding relies on)."""
    prob = _small()
    base = dict(warmup=40, samples=30, seed=11, max_treedepth=6)
    full = nuts_c.sample(prob, SamplerConfig(chains=6, **base), nthreads=3)["draws"]
    a = nuts_c.sample(prob, SamplerConfig(chains=2, **base), nthreads=2)["draws"]
    b = nuts_c.sample(prob, SamplerConfig(chains=4, chain_offset=2, **base), nthreads=2)["draws"]
    np.testing.assert_array_equal(np.concatenate([a, b]), full)


def test_deterministic_and_seed_sensitive():
    prob = _small("lasso")
    cfg = SamplerConfig(chains=3, warmup=30, samples=20, seed=5, max_treedepth=6)
    d1 = nuts_c.sample(prob, cfg, nthreads=3)["draws"]
    d2 = nuts_c.sample(prob, cfg, nthreads=1)["draws"]
    np.testing.assert_array_equal(d1, d2)
    cfg.seed = 6
    assert not np.array_equal(d1, nuts_c.sample(prob, cfg, nthreads=3)["draws"])


@pytest.mark.parametrize("path", golden_files("draws"), ids=lambda p: os.path.basename(p))
@pytest.mark.skipif(nuts_c.SANITIZE, reason="the fixture pins the gcc -O3 -march=x86-64-v3 "
                    "build's arithmetic; the sanitized oracle is clang -O1")
def test_oracle_reproduces_draw_fixture(path):
    fx = load_golden(path)
    m = fx["meta"]
    prob = ExpGPProblem(fx["x"], fx["y"], fx["uy"], Nn=m["Nn"], gridType=m["grid_type"],
                        theta0=fx["theta0"], Sigma0=fx["Sigma0"], prior_type=m["family"])
    cfg = SamplerConfig(chains=m["chains"], warmup=m["warmup"], samples=m["samples"],
                        seed=m["seed"], max_treedepth=m["max_treedepth"])
    o = nuts_c.sample(prob, cfg, nthreads=4)
    np.testing.assert_allclose(o["draws"], fx["draws"], rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(o["leapfrogs"], fx["leapfrogs"])


def test_sampler_columns_consistent():
    """Stan sampler diagnostics columns: treedepth/n_leapfrog relation, accept in
    [0,1], stepsize constant after warmup, sigma/theta positive, br >= 0."""
    prob = _small("horseshoe", Nn=4)
    cfg = SamplerConfig(chains=2, warmup=60, samples=40, seed=3, max_treedepth=6)
    d = nuts_c.sample(prob, cfg, nthreads=2)["draws"]
    cols = prob.column_names()
    c = {n: i for i, n in enumerate(cols)}
    td, nl = d[..., c["treedepth__"]], d[..., c["n_leapfrog__"]]
    # base_nuts: depth_ is not incremented when the subtree just built is invalid
    assert np.all(nl >= 2 ** td - 1) and np.all(nl <= 2 ** (td + 1) - 1)
    acc = d[..., c["accept_stat__"]]
    assert np.all((acc >= 0) & (acc <= 1))
    eps = d[:, cfg.warmup:, c["stepsize__"]]
    assert np.all(eps == eps[:, :1])
    assert np.all(d[..., c["sigma"]] > 0) and np.all(d[..., c["theta.3"]] > 0)
    assert np.all(d[..., c["br"]] >= 0)
    assert np.all(td <= cfg.max_treedepth)


def test_warm_restart_restatement():
    """oracle_set_init (the restatement of fitoct_plan_set_init): with adaptation off the
    given step size and metric are used unchanged, the chains start at the given point
    (no jittered init: the run does not depend on init_radius), a start whose density is
    not finite fails with FITOCT_E_INIT instead of being retried, and clearing the start
    restores the default run."""
    prob = _small()
    first = nuts_c.sample(prob, SamplerConfig(chains=4, warmup=150, samples=20, seed=3),
                          nthreads=4)
    last = first["draws"][:, -1, 7:7 + prob.D]
    logc = np.array([k < 3 or k >= 3 + prob.Nn for k in range(prob.D)])
    q0 = last.copy()
    q0[:, logc] = np.log(last[:, logc])
    cfg = SamplerConfig(chains=4, warmup=0, samples=30, seed=4, adapt_engaged=False)
    kw = dict(q_init=q0, init_stepsize=first["stepsize"], init_inv_metric=first["inv_metric"])
    a = nuts_c.sample(prob, cfg, nthreads=4, **kw)
    cfg_r = SamplerConfig(chains=4, warmup=0, samples=30, seed=4, adapt_engaged=False,
                          init_radius=0.5)
    b = nuts_c.sample(prob, cfg_r, nthreads=4, **kw)
    assert np.array_equal(a["draws"], b["draws"], equal_nan=True)
    assert np.array_equal(a["stepsize"], first["stepsize"])
    assert np.array_equal(a["inv_metric"], first["inv_metric"])
    assert np.all(a["draws"][:, :, 2] == first["stepsize"][:, None])
    # started in the typical set: lp__ of the first draws matches the first run's tail
    tail = first["draws"][:, -20:, 0]
    assert abs(a["draws"][:, :5, 0].mean() - tail.mean()) < 5.0 * tail.std()
    bad = q0.copy()
    bad[1, 0] = 800.0   # theta1 = exp(800): lp = -inf
    with pytest.raises(RuntimeError, match="status -4"):
        nuts_c.sample(prob, cfg, nthreads=4, q_init=bad)
    d0 = nuts_c.sample(prob, cfg, nthreads=4)
    d1 = nuts_c.sample(prob, cfg, nthreads=4)
    assert np.array_equal(d0["draws"], d1["draws"], equal_nan=True)
    assert not np.array_equal(d0["draws"], a["draws"], equal_nan=True)


def test_batch_fixture_reproduces_from_the_committed_script():
    """tests/golden/batch_files.npz (config 5's per-file oracle behaviour, compared with the
    GPU in test_gpu_funnel.py) is what tests/golden/make_trapped.py computes: the first
    files re-run here give the stored per-file R-hat, step size, depth and divergences."""
    import sys as _s
    _s.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_trapped as T
    fx = T.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             "batch_files.npz"))
    B = fx["meta"]
    assert (B["files"], B["chains"], B["warmup"], B["samples"]) == (256, 4, 100, 100)
    for f in (0, 1, 2):
        prob = T.batch_problem(f)
        cfg = SamplerConfig(chains=B["chains"], chain_offset=f * B["chains"], warmup=B["warmup"],
                            samples=B["samples"], seed=B["seed"], adapt_delta=B["adapt_delta"],
                            max_treedepth=B["max_treedepth"])
        o = nuts_c.sample(prob, cfg, nthreads=4)
        st = T.file_stats(o["draws"], B["warmup"], prob.column_names())
        np.testing.assert_allclose(st, [fx["rhat_max"][f], fx["stepsize"][f], fx["treedepth"][f],
                                        fx["div_rate"][f]], rtol=1e-12)
