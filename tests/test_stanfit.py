"""Host-side result object and the fitExpGP mirror (no GPU): StanFit access
paths the reference's consumers use (plotExpGP.R:7-50, server.R:88-237),
horseshoe transformed parameters (horseShoePrior.stan:25-33), Stan-CSV export,
and fitExpGP's argument contract (FitOCT.R:110-124)."""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import ExpGPProblem, SamplerConfig, fitExpGP
from fitoct_amd.api import SampleOutput
from fitoct_amd.stanfit import StanFit
from fitoct_amd.synth import default_prior, synth_decay
from oracle import diag_np, nuts_c


def _run(family, prior_PD=0, Nn=4, chains=3):
    t0, S0 = default_prior()
    d = synth_decay(48, "sincExp", 2)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=family, prior_PD=prior_PD)
    cfg = SamplerConfig(chains=chains, warmup=40, samples=60, seed=8, max_treedepth=6)
    o = nuts_c.sample(prob, cfg, nthreads=3)
    out = SampleOutput(o["draws"], prob.column_names(), cfg.warmup, o["stepsize"],
                       o["inv_metric"], o["inv_metric"] * 0, int(o["leapfrogs"].sum()), 0, 0,
                       cfg=cfg)
    return prob, cfg, StanFit.from_output(out, prob), o


def test_extract_as_matrix_summary():
    prob, cfg, fit, o = _run("normal")
    assert fit.chains == 3 and fit.iterations == 60 and fit.warmup == 40
    th = fit.extract("theta")
    assert list(th) == ["theta.1", "theta.2", "theta.3"]
    assert th["theta.1"].shape == (3, 60)
    assert fit.extract("br", inc_warmup=True)["br"].shape == (3, 100)
    m = fit.as_matrix(["theta", "sigma"])
    assert m.shape == (180, 4)
    np.testing.assert_array_equal(m[:60, 0], o["draws"][0, 40:, 7])
    s = fit.summary(["theta", "yGP", "lambda", "sigma", "br", "lp__"])
    assert set(s["theta.2"]) >= {"mean", "se_mean", "sd", "2.5%", "50%", "97.5%", "n_eff", "Rhat"}
    x = fit.extract("theta.2")["theta.2"]
    assert s["theta.2"]["Rhat"] == pytest.approx(diag_np.split_rhat(x), rel=1e-10)
    assert s["theta.2"]["n_eff"] == pytest.approx(diag_np.split_ess(x), rel=1e-8)
    assert s["theta.2"]["mean"] == pytest.approx(x.mean())
    txt = fit.print(["theta"])
    assert "theta.3" in txt and "Rhat" in txt
    with pytest.raises(KeyError):
        fit.extract("nope")


def test_horseshoe_transformed_parameters():
    prob, cfg, fit, o = _run("horseshoe", Nn=3)
    cols = fit.columns
    assert {"yGP.1", "yGP.3", "tau", "lambda.2"} <= set(cols)
    c = {n: i for i, n in enumerate(prob.column_names())}
    d = o["draws"]
    tau = d[..., c["r1_global"]] * np.sqrt(d[..., c["r2_global"]])
    lam2 = d[..., c["r1_local.2"]] * np.sqrt(d[..., c["r2_local.2"]])
    y2 = d[..., c["z.2"]] * lam2 * tau
    np.testing.assert_allclose(fit.extract("tau", inc_warmup=True)["tau"], tau)
    np.testing.assert_allclose(fit.extract("yGP.2", inc_warmup=True)["yGP.2"], y2)
    assert cols[-1] == "br"


def test_prior_pd_drops_br():
    _, _, fit, _ = _run("lasso", prior_PD=1)
    assert "br" not in fit.columns
    with pytest.raises(KeyError):
        fit.extract("br")


def test_stan_csv_roundtrip(tmp_path):
    _, cfg, fit, o = _run("lasso")
    paths = fit.write_stan_csv(str(tmp_path))
    assert len(paths) == 3
    lines = open(paths[1]).read().splitlines()
    header = [l for l in lines if not l.startswith("#")][0].split(",")
    assert header == fit.columns
    assert any(l.startswith("# Step size") for l in lines)
    assert any("algorithm = hmc" in l for l in lines) and any("Elapsed Time" in l for l in lines)
    rows = [l for l in lines if not l.startswith("#")][1:]
    data = np.array([[float(v) for v in r.split(",")] for r in rows])
    np.testing.assert_array_equal(data, fit._draws[1])   # lasso: + the constant lambda column


def test_fitexpgp_argument_contract():
    d = synth_decay(32, "sincExp", 1)
    t0, S0 = default_prior()
    with pytest.raises(ValueError):
        fitExpGP(d["x"], d["y"], d["uy"], method="mcmc", theta0=t0, Sigma0=S0)
    with pytest.raises(ValueError):
        fitExpGP(d["x"], d["y"], d["uy"], theta0=t0, Sigma0=S0, nb_warmup=100, nb_iter=100)
    with pytest.raises(ValueError):
        fitExpGP(d["x"], d["y"], d["uy"], theta0=None)
    with pytest.raises(ValueError):
        ExpGPProblem(d["x"], d["y"][:-1], d["uy"])
    with pytest.raises(ValueError):
        ExpGPProblem(d["x"], d["y"], d["uy"], gridType="bogus")
