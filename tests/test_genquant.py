"""Generated quantities (fitoct_amd.genquant): m, dL, resid, br from parameter
draws, against the numpy oracle's sum of squared normalised residuals."""
from __future__ import annotations

import numpy as np
import pytest

from fitoct_amd import ExpGPProblem
from fitoct_amd.genquant import expgp_curves
from fitoct_amd.synth import default_prior, synth_decay
from oracle import model_np as M


@pytest.mark.parametrize("grid,dt", [("extremal", 2), ("internal", 1)])
def test_curves_match_oracle_residuals(grid, dt):
    t0, S0 = default_prior()
    d = synth_decay(300, "sincExp1", 4)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], dataType=dt, Nn=12, gridType=grid, theta0=t0,
                        Sigma0=S0, prior_type="normal")
    npp = M.Problem(d["x"], d["y"], d["uy"], data_type=dt, Nn=12, grid_type=grid, theta0=t0,
                    Sigma0=S0, family=M.NORMAL)
    rng = np.random.default_rng(1)
    for _ in range(5):
        th = t0 * np.exp(rng.normal(0, 0.02, 3))
        ygp = rng.normal(0, 0.05, 12)
        q = np.concatenate([np.log(th), ygp, [np.log(0.1), 0.0]])
        _, _, s2 = M.logp_grad(q, npp)
        g = expgp_curves(prob, th, ygp)
        assert abs(g["br"][0] * prob.N - s2) <= 1e-10 * s2
        B, _ = prob.basis()
        np.testing.assert_allclose(g["dL"][0], B @ ygp, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(g["resid"][0], (d["y"] - g["m"][0]) / d["uy"], rtol=1e-12)
