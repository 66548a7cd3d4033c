"""Stan output of the library (include/fitoct.h "Stan output"), without a GPU:

* the output layout resolves every ``pars`` list the reference's consumers pass, for
  every prior family with and without ``prior_PD`` (plotExpGP.R:9,41-43;
  server.R:88-237);
* the CmdStan CSV written by ``fitoct_write_stan_csv`` (the one writer the R shim and
  the Python mirror share) carries what rstan::read_stan_csv reads -- argument header,
  adaptation block between warmup and sampling rows, elapsed-time trailer -- and its
  draws round-trip bit for bit;
* ``fitoct_write_vb_csv`` (rstan::vb's stanfit);
* the rstan-format progress lines decode, through a port of the Shiny server's parser
  (server.R:457-472), to a monotone 0..100.
The draws come from the C oracle (the GPU path writes through the same code; its
GPU tests are in test_rshim_driver.py).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import stancsv_reader
from fitoct_amd import _lib
from fitoct_amd.api import ExpGPProblem, SampleOutput, SamplerConfig
from fitoct_amd.stanfit import SAMPLER_COLS, StanFit, _base, materialise, output_columns
from fitoct_amd.synth import default_prior, synth_decay
from oracle import nuts_c
from shiny_progress import do_progress, replay

# every pars list of the reference's consumers
PARS = {
    "plotExpGP.R:9": ["theta", "yGP", "lambda", "sigma", "br"],
    "plotExpGP.R:41": ["theta", "yGP", "lambda", "sigma", "br", "lp__"],
    "plotExpGP.R:43": ["theta", "yGP", "lambda", "sigma", "lp__"],
    "server.R:203": ["theta", "yGP", "lambda", "sigma", "br"],
    "server.R:220": ["theta", "yGP", "lambda", "sigma"],
}


def _prob(family, prior_PD=0, Nn=4, N=48):
    t0, S0 = default_prior()
    d = synth_decay(N, "sincExp", 2)
    return ExpGPProblem(d["x"], d["y"], d["uy"], Nn=Nn, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type=family, prior_PD=prior_PD)


def _run(family, prior_PD=0, Nn=4, chains=3, save_warmup=True):
    prob = _prob(family, prior_PD, Nn)
    cfg = SamplerConfig(chains=chains, warmup=40, samples=60, seed=8, max_treedepth=6,
                        save_warmup=save_warmup)
    o = nuts_c.sample(prob, cfg, nthreads=chains)
    out = SampleOutput(o["draws"], prob.column_names(), cfg.warmup if save_warmup else 0,
                       o["stepsize"], o["inv_metric"], o["inv_metric"] * 0,
                       int(o["leapfrogs"].sum()), 1234.5, 0, cfg=cfg)
    return prob, cfg, StanFit.from_output(out, prob), o


@pytest.mark.parametrize("family", ["normal", "lasso", "horseshoe"])
@pytest.mark.parametrize("prior_PD", [0, 1])
def test_consumer_pars_resolve(family, prior_PD):
    cols = output_columns(_prob(family, prior_PD, Nn=5))
    bases = {_base(c) for c in cols}
    for where, pars in PARS.items():
        if prior_PD and "br" in pars:
            continue          # plotExpGP.R:42-43 drops br for the prior run
        missing = set(pars) - bases
        assert not missing, f"{where}: {missing} not in the {family} fit"
    assert ("br" in bases) == (not prior_PD)
    assert sum(_base(c) == "yGP" for c in cols) == 5
    assert cols[:7] == SAMPLER_COLS


def test_monoexp_layout():
    t0, _ = default_prior()
    d = synth_decay(40, "sincExp", 2)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=2, theta0=t0, Sigma0=np.eye(3),
                        prior_type="monoexp")
    assert output_columns(prob, lead=()) == ["theta.1", "theta.2", "theta.3", "br"]


def test_layout_values():
    """horseshoe: tau, lambda, yGP of horseShoePrior.stan:30-32; lasso: lambda = lambda_s
    (⚑, a constant); normal: the kernel's columns unchanged."""
    prob, _, fit, o = _run("horseshoe", Nn=3)
    c = {n: i for i, n in enumerate(prob.column_names())}
    d = o["draws"]
    tau = d[..., c["r1_global"]] * np.sqrt(d[..., c["r2_global"]])
    lam = d[..., [c[f"r1_local.{k}"] for k in (1, 2, 3)]] * \
        np.sqrt(d[..., [c[f"r2_local.{k}"] for k in (1, 2, 3)]])
    ygp = d[..., [c[f"z.{k}"] for k in (1, 2, 3)]] * lam * tau[..., None]
    j = {n: i for i, n in enumerate(fit.columns)}
    got = fit.extract(None, inc_warmup=True)
    np.testing.assert_array_equal(got["tau"], tau)
    for k in range(3):
        np.testing.assert_array_equal(got[f"lambda.{k+1}"], lam[..., k])
        np.testing.assert_array_equal(got[f"yGP.{k+1}"], ygp[..., k])
    assert fit.columns[-1] == "br" and j["tau"] == j["sigma"] + 1
    prob, _, fit, o = _run("lasso", Nn=3)
    assert np.all(fit.extract("lambda", inc_warmup=True)["lambda"] == prob.lambda_scale)
    assert fit.columns.index("lambda") == fit.columns.index("sigma") + 1
    prob, _, fit, o = _run("normal", Nn=3)
    np.testing.assert_array_equal(fit._draws, o["draws"])


@pytest.mark.parametrize("family,prior_PD", [("normal", 0), ("lasso", 1), ("horseshoe", 0)])
def test_stan_csv_what_read_stan_csv_reads(tmp_path, family, prior_PD):
    prob, cfg, fit, o = _run(family, prior_PD)
    paths = fit.write_stan_csv(str(tmp_path))
    assert len(paths) == 3
    for ch, path in enumerate(paths):
        r = stancsv_reader.read(path)
        v = r["values"]
        assert v["num_samples"] == "60" and v["num_warmup"] == "40" and v["save_warmup"] == "1"
        assert v["thin"] == "1" and v["algorithm"] == "hmc" and v["engine"] == "nuts"
        assert v["metric"] == "diag_e" and v["max_depth"] == "6" and v["delta"] == "0.8"
        assert v["id"] == str(ch + 1) and v["seed"] == "8" and v["method"] == "sample"
        assert r["header"] == fit.columns
        assert r["rows"].shape == (100, len(fit.columns))
        assert r["rows_before_adaptation"] == 40           # warmup rows first (traceplot)
        np.testing.assert_array_equal(r["rows"], fit._draws[ch])     # %.17g: exact
        assert r["stepsize"] == o["stepsize"][ch]
        np.testing.assert_array_equal(r["inv_metric"], o["inv_metric"][ch])
        t = r["times"]
        assert t["Total"] == pytest.approx(1.2345, abs=2e-6)
        assert t["Warm-up"] + t["Sampling"] == pytest.approx(t["Total"], abs=2e-6)
        lf = o["draws"][ch, :, 4]
        assert t["Warm-up"] == pytest.approx(1.2345 * lf[:40].sum() / lf.sum(), abs=2e-6)
        assert ("br" in r["header"]) == (not prior_PD)


def test_stan_csv_without_warmup_rows(tmp_path):
    _, cfg, fit, o = _run("normal", save_warmup=False)
    r = stancsv_reader.read(fit.write_stan_csv(str(tmp_path))[0])
    assert r["values"]["save_warmup"] == "0" and r["rows"].shape[0] == 60
    assert r["rows_before_adaptation"] == 0


def test_stan_csv_nonfinite_values(tmp_path):
    prob, cfg, fit, o = _run("normal", chains=1)
    raw = o["draws"].copy()
    raw[0, 3, 0] = np.nan
    raw[0, 4, 6] = np.inf
    raw[0, 5, 6] = -np.inf
    p, c = prob.to_c(), cfg.to_c()
    path = str(tmp_path / "x.csv")
    assert _lib.lib().fitoct_write_stan_csv(
        path.encode(), C.byref(p), C.byref(c), 0, _lib.dptr(np.ascontiguousarray(raw[0])), 0.1,
        None, 0.0, 0.0) == 0
    txt = open(path).read()
    assert ",Inf," in txt or ",Inf\n" in txt or txt.count("Inf") >= 2
    r = stancsv_reader.read(path)
    assert np.isnan(r["rows"][3, 0]) and r["rows"][4, 6] == np.inf and r["rows"][5, 6] == -np.inf
    assert np.all(r["inv_metric"] == 1.0)      # NULL metric: unit diagonal


def test_stan_csv_errors(tmp_path):
    prob, cfg, fit, o = _run("normal", chains=1)
    p, c = prob.to_c(), cfg.to_c()
    L = _lib.lib()
    raw = np.ascontiguousarray(o["draws"][0])
    assert L.fitoct_write_stan_csv(str(tmp_path / "no/such/dir.csv").encode(), C.byref(p),
                                   C.byref(c), 0, _lib.dptr(raw), 0.1, None, 0, 0) == -1
    assert b"cannot open" in L.fitoct_last_error()
    assert L.fitoct_write_stan_csv(str(tmp_path / "a.csv").encode(), C.byref(p), C.byref(c), 5,
                                   _lib.dptr(raw), 0.1, None, 0, 0) == -1


def test_vb_csv(tmp_path):
    """CmdStan variational layout: mean row first, then draws with log_p__ / log_g__."""
    prob = _prob("horseshoe", Nn=3)
    D, S = prob.D, 7
    rng = np.random.default_rng(3)
    mu = rng.normal(0, 0.1, D)
    mu[:3] = np.log(prob.theta0)
    q = mu + rng.normal(0, 0.05, (S, D))
    lp, lg, s2 = rng.normal(size=S), rng.normal(size=S), rng.uniform(40, 60, S)
    vc = _lib.VbConfig()
    _lib.lib().fitoct_default_vb_config(C.byref(vc))
    vc.output_samples = S
    p = prob.to_c()
    path = str(tmp_path / "vb.csv")
    assert _lib.lib().fitoct_write_vb_csv(path.encode(), C.byref(p), C.byref(vc), _lib.dptr(mu),
                                          50.0, S, _lib.dptr(q), _lib.dptr(lp), _lib.dptr(lg),
                                          _lib.dptr(s2), 0.1) == 0
    r = stancsv_reader.read(path)
    assert r["values"]["method"] == "variational" and r["values"]["output_samples"] == str(S)
    assert r["header"] == output_columns(prob, lead=["lp__", "log_p__", "log_g__"])
    assert r["rows"].shape == (S + 1, len(r["header"]))
    from fitoct_amd.optim_vb import constrain
    raw = np.concatenate([np.zeros((S, 1)), lp[:, None], lg[:, None], constrain(prob, q),
                          (s2 / prob.N)[:, None]], axis=1)
    np.testing.assert_array_equal(r["rows"][1:], materialise(raw, prob, n_lead=3))
    mean = materialise(np.concatenate([[0, 0, 0], constrain(prob, mu)[0], [50.0 / prob.N]]),
                       prob, n_lead=3)
    np.testing.assert_array_equal(r["rows"][0], mean)


def _line(done, total, W, S):
    buf = C.create_string_buffer(160)
    pct = _lib.lib().fitoct_progress_line(done, total, W, S, buf, 160)
    return pct, buf.value.decode()


@pytest.mark.parametrize("chains,W,S", [(4, 500, 1000), (1024, 500, 1000), (1, 3, 1), (7, 0, 13)])
def test_progress_lines_decode_monotone(chains, W, S):
    """Every overall percentage the driver would print, through the Shiny parser."""
    total = chains * (W + S)
    lines, printed = [], []
    for done in sorted(set(np.linspace(0, total, 997).astype(int).tolist() + [total])):
        pct, txt = _line(done, total, W, S)
        assert pct == 100 * done // total
        if not printed or pct != printed[-1]:
            lines.append(txt)
            printed.append(pct)
    shown = replay(lines)
    assert shown[0] == 0 and shown[-1] == 100
    assert all(b >= a for a, b in zip(shown, shown[1:]))
    assert shown == printed      # the Shiny display shows the run's true overall percentage


def test_progress_line_format():
    pct, txt = _line(0, 4 * 1500, 500, 1000)
    assert txt == "Chain 1: Iteration:    0 / 1500 [  0%]  (Warmup)" and pct == 0
    pct, txt = _line(3 * 1500, 4 * 1500, 500, 1000)       # 75 % overall
    assert txt == "Chain 4: Iteration:    0 / 1500 [  0%]  (Warmup)" and pct == 75
    assert do_progress([txt]) == 75
    pct, txt = _line(4 * 1500, 4 * 1500, 500, 1000)
    assert txt == "Chain 4: Iteration: 1500 / 1500 [100%]  (Sampling)" and pct == 100
    assert do_progress([txt]) == 100
    pct, txt = _line(int(4 * 1500 * 0.6), 4 * 1500, 500, 1000)   # 2.4 chains: chain 3 at 40 %
    assert txt.startswith("Chain 3: Iteration:  600 / 1500 [ 40%]  (Sampling)")
    assert do_progress([txt]) == 60
    assert _lib.lib().fitoct_progress_line(1, 0, 5, 5, C.create_string_buffer(160), 160) == -1
