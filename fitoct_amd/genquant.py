"""Generated quantities of the ExpGP model for selected draws:
the modulation ``dL = B yGP``, the model ``m = theta1 + theta2 exp(-c x / (theta3 (1+dL)))``
(ShinyInterface/ui.R:88, synthData.R:22), the normalised residuals
``resid = (y - m) / uy`` and the Birge ratio ``br = mean(resid^2)``, as FitOCTLib's
Stan model exposes them to ``plotExpGP`` (plotExpGP.R:46-57, nMC = 100 spaghetti
draws) and as ``fit$par$m`` / ``fit$par$resid`` of an optimisation
(server.R:351,636).  The sampler itself stores ``br`` per draw; these per-bin
vectors are recomputed on the host for the draws a caller asks for (a few
hundred for plots), since storing N of each per draw would multiply the draw
buffer by ~3N/D.
"""
from __future__ import annotations

import numpy as np


def expgp_curves(prob, theta, ygp, B=None):
    """dict(dL, m, resid, br) for parameter rows ``theta[S, 3]``, ``ygp[S, Nn]``."""
    theta = np.atleast_2d(np.asarray(theta, np.float64))
    ygp = np.atleast_2d(np.asarray(ygp, np.float64))
    if B is None:
        B, _ = prob.basis()
    x, y, uy = prob.x, prob.y, prob.uy
    c = float(prob.dataType)
    dL = ygp @ B.T
    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        m = theta[:, :1] + theta[:, 1:2] * np.exp(-c * x[None, :] / (theta[:, 2:3] * (1.0 + dL)))
    resid = (y[None, :] - m) / uy[None, :]
    return {"dL": dL, "m": m, "resid": resid, "br": np.mean(resid * resid, axis=1)}


def generated_quantities(fit, prob, n=100, seed=None, draws=None):
    """Generated quantities for ``n`` post-warmup draws of a StanFit chosen at
    random (``seed``), or for the explicit flat draw indices ``draws``.  Returns
    dict(index, theta, yGP, dL, m, resid, br) with rows per selected draw."""
    theta = fit.as_matrix("theta")
    ygp = fit.as_matrix("yGP")
    S = theta.shape[0]
    if draws is None:
        rng = np.random.default_rng(seed)
        draws = np.sort(rng.choice(S, size=min(n, S), replace=False))
    draws = np.asarray(draws, dtype=np.int64)
    out = expgp_curves(prob, theta[draws], ygp[draws])
    out.update({"index": draws, "theta": theta[draws], "yGP": ygp[draws]})
    return out
