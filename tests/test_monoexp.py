"""fitMonoExp: the mono-exponential model of
FitOCTLib::fitMonoExp (FitOCT.R:95, server.R:341) on the same engine.

CPU: the oracle's restatement of the model (numpy / C), the data-driven
initialisation and the Birge-ratio gate (printBr, plotMonoExp.R:10,
FitOCT.R:100).  GPU (marked): the MAP + Hessian path against an independent
host least-squares fit, and the device sampler against the oracle.
"""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import ExpGPProblem, SamplerConfig
from fitoct_amd.monoexp import OptimFit, decay, fitMonoExp, initial_theta, mono_problem, printBr
from fitoct_amd.synth import synth_decay
from oracle import diag_np, nuts_c
from oracle import model_np as M

TRUE = np.array([1000.0, 2000.0, 300.0])   # synthData.R:3-7, dataType 2: theta3 = 2 l0


def _data(N=256, seed=3):
    return synth_decay(N, "monoExp", seed)


def _ls_reference(d, dataType=2):
    """Independent MAP: weighted least squares in log theta (scipy, numpy model)."""
    from scipy.optimize import least_squares
    x, y, uy = d["x"], d["y"], d["uy"]

    def res(q):
        return (y - decay(x, np.exp(q), dataType)) / uy
    r = least_squares(res, np.log(initial_theta(x, y, dataType)), xtol=1e-15, ftol=1e-15,
                      gtol=1e-15, method="lm")
    return np.exp(r.x)


def test_initial_theta_is_close_enough():
    d = _data()
    t = initial_theta(d["x"], d["y"], 2)
    assert np.all(np.abs(np.log(t / TRUE)) < 0.5)


def test_numpy_model_is_weighted_least_squares():
    d = _data()
    P = M.Problem(d["x"], d["y"], d["uy"], family=M.MONOEXP, theta0=TRUE)
    q = np.log(TRUE * np.array([1.01, 0.99, 1.02]))
    lp, g, s2 = M.logp_grad(q, P)
    r = (d["y"] - decay(d["x"], np.exp(q))) / d["uy"]
    assert lp == pytest.approx(-0.5 * r @ r + q.sum(), rel=1e-13)
    assert s2 == pytest.approx(r @ r, rel=1e-13)
    np.testing.assert_allclose(g, M.fd_grad(q, P), rtol=1e-5, atol=1e-4)


def test_oracle_sampler_recovers_truth():
    d = _data()
    prob = mono_problem(d["x"], d["y"], d["uy"], 2)
    cfg = SamplerConfig(chains=4, warmup=300, samples=500, seed=4)
    o = nuts_c.sample(prob, cfg, nthreads=4)
    th = o["draws"][:, 300:, 7:10]
    for k in range(3):
        x = th[:, :, k]
        assert abs(x.mean() - TRUE[k]) < 5 * x.std() + 1e-9
        assert diag_np.split_rhat(x) < 1.02
    br = o["draws"][:, 300:, 10]
    assert 0.7 < br.mean() < 1.4     # noise sd is the true uy: br ~ chi2_N / N


def test_printbr_gate():
    d = _data(N=400)
    r = (d["y"] - d["y_true"]) / d["uy"]
    fit = OptimFit({"theta": TRUE, "m": d["y_true"], "resid": r, "br": float(r @ r) / r.size},
                   0.0, np.eye(3), ["theta.1", "theta.2", "theta.3"])
    ok = printBr(fit, silent=True)
    assert ok["alert"] is None and ok["interval"][0] < ok["br"] < ok["interval"][1]
    fit.par["br"] = 3.0
    assert printBr(fit, silent=True)["alert"] is not None


def test_argument_contract():
    d = _data(N=64)
    with pytest.raises(ValueError):
        fitMonoExp(d["x"], d["y"], d["uy"], method="mcmc")
    prob = mono_problem(d["x"], d["y"], d["uy"])
    assert prob.D == 3 and prob.column_names()[7:] == ["theta.1", "theta.2", "theta.3", "br"]


# ------------------------------------------------------------------ GPU --
@pytest.mark.gpu
def test_gpu_map_matches_least_squares():
    d = _data()
    out = fitMonoExp(d["x"], d["y"], d["uy"], dataType=2, method="optim")
    ref = _ls_reference(d)
    np.testing.assert_allclose(out["best.theta"], ref, rtol=1e-6)
    fit = out["fit"]
    np.testing.assert_allclose(fit.par["m"], decay(d["x"], ref), rtol=1e-6)
    # Hessian (unconstrained, no Jacobian) vs numpy finite differences
    P = M.Problem(d["x"], d["y"], d["uy"], family=M.MONOEXP, theta0=ref)
    q = np.log(out["best.theta"])
    h = 1e-4

    def g(qq):
        return M.logp_grad(qq, P)[1] - 1.0
    Hn = np.stack([(g(q + h * e) - g(q - h * e)) / (2 * h) for e in np.eye(3)], axis=1)
    np.testing.assert_allclose(fit.hessian, 0.5 * (Hn + Hn.T), rtol=1e-3)
    c = out["cor.theta"]
    assert np.allclose(np.diag(c), 1.0) and np.all(np.abs(c) <= 1.0 + 1e-12)
    assert printBr(fit, silent=True)["alert"] is None


@pytest.mark.gpu
def test_gpu_sampler_matches_oracle():
    d = _data()
    prob = mono_problem(d["x"], d["y"], d["uy"], 2)
    cfg = SamplerConfig(chains=16, warmup=300, samples=400, seed=8)
    from fitoct_amd import sample
    g = sample(prob, cfg)
    o = nuts_c.sample(prob, SamplerConfig(chains=16, chain_offset=100, warmup=300, samples=400,
                                          seed=8), nthreads=16)
    for j in range(7, 11):
        a, b = g.draws[:, 300:, j], o["draws"][:, 300:, j]
        _, ea = diag_np.split_rhat(a), diag_np.split_ess(a)
        eb = diag_np.split_ess(b)
        se = np.sqrt(a.var() / ea + b.var() / eb)
        assert abs(a.mean() - b.mean()) < 4.5 * se, (j, a.mean(), b.mean(), se)
    res = fitMonoExp(d["x"], d["y"], d["uy"], method="sample", nb_warmup=300, nb_iter=700,
                     nb_chains=8, seed=3)
    assert np.all(np.abs(res["best.theta"] / TRUE - 1) < 0.05)


def _initial_theta_np(x, y, dataType=2):
    """numpy restatement of fitoct_mono_initial_theta (include/fitoct.h)."""
    x, y = np.asarray(x, float), np.asarray(y, float)
    n = x.size
    tail = max(3, n // 10)
    order = np.argsort(x, kind="stable")
    xs, ys = x[order], y[order]
    t1 = float(np.median(ys[-tail:]))
    amp = ys - t1
    ok = amp > 0.05 * max(float(amp.max()), 1e-12)
    if ok.sum() >= 3:
        slope, icpt = np.polyfit(xs[ok], np.log(amp[ok]), 1)
    else:
        slope, icpt = -1.0 / max(xs.max() - xs.min(), 1e-12), np.log(max(amp.max(), 1e-12))
    slope = min(slope, -1e-12)
    return np.array([max(abs(t1), 1e-6), max(np.exp(icpt), 1e-6),
                     max(float(dataType) / -slope, 1e-6)])


@pytest.mark.parametrize("case", ["decay", "reversed", "flat", "two_bins", "amplitude"])
def test_initial_theta_matches_restatement(case):
    rng = np.random.default_rng(5)
    x = np.linspace(20, 500, 300)
    y = 1000 + 2000 * np.exp(-2 * x / 300) + rng.normal(0, 5, x.size)
    dt = 2
    if case == "reversed":
        x, y = x[::-1].copy(), y[::-1].copy()
    elif case == "flat":
        y = 1000 + 0 * x
    elif case == "two_bins":
        x, y = x[:2].copy(), y[:2].copy()
    elif case == "amplitude":
        y = 20 + 80 * np.exp(-x / 150)
        dt = 1
    np.testing.assert_allclose(initial_theta(x, y, dt), _initial_theta_np(x, y, dt), rtol=1e-9)
