"""Generated quantities against the sampler: the br column the kernel writes per
draw (sum of squared normalised residuals / N at the sampled point) equals the
host recomputation from the stored theta / yGP (fitoct_amd.genquant), and
fitExpGP(method='optim') exposes fit$par$m / resid / dL (server.R:351,636)."""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import SamplerConfig, fitExpGP, sample
from fitoct_amd.genquant import generated_quantities
from fitoct_amd.stanfit import StanFit
from fitoct_amd.synth import default_prior, synth_decay
from test_gpu_sampler import _prob

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("family,N", [("horseshoe", 512), ("normal", 2048), ("lasso", 3001)])
def test_br_column_equals_recomputed(family, N):
    prob = _prob(family, N, 15)
    out = sample(prob, SamplerConfig(chains=8, warmup=60, samples=40, seed=4, max_treedepth=6))
    fit = StanFit.from_output(out, prob)
    g = generated_quantities(fit, prob, n=64, seed=0)
    br = fit.as_matrix("br")[g["index"], 0]
    np.testing.assert_allclose(g["br"], br, rtol=1e-10)
    assert g["m"].shape == (64, N) and np.all(np.isfinite(g["m"]))


def test_optim_fit_has_curves():
    t0, S0 = default_prior()
    d = synth_decay(481, "sincExp", 2)
    res = fitExpGP(d["x"], d["y"], d["uy"], Nn=10, gridType="extremal", method="optim",
                   theta0=t0, Sigma0=S0)
    par = res["fit"].par
    assert par["m"].shape == (481,) and par["resid"].shape == (481,)
    np.testing.assert_allclose(np.mean(par["resid"] ** 2), par["br"], rtol=1e-9)
