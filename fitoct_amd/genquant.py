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

import ctypes as C

import numpy as np

from . import _lib


def expgp_curves(prob, theta, ygp=None, B=None):
    """dict(dL, m, resid, br) for parameter rows ``theta[S, 3]``, ``ygp[S, Nn]``
    (``ygp`` is ignored for the mono-exponential model), computed by the library
    (``fitoct_expgp_curves``, the code the R shim uses for ``fit$par$m``)."""
    theta = np.ascontiguousarray(np.atleast_2d(np.asarray(theta, np.float64)))
    n, N = theta.shape[0], prob.N
    p = prob.to_c()
    if B is not None:
        B = np.ascontiguousarray(B, dtype=np.float64)
        p.B = _lib.dptr(B)
    if prob.prior_type == "monoexp":
        ygp = None
    else:
        ygp = np.ascontiguousarray(np.atleast_2d(np.asarray(ygp, np.float64)))
        if ygp.shape != (n, prob.Nn):
            raise ValueError(f"yGP has shape {ygp.shape}, expected {(n, prob.Nn)}")
    dL, m, resid, br = np.empty((n, N)), np.empty((n, N)), np.empty((n, N)), np.empty(n)
    _lib.check(_lib.lib().fitoct_expgp_curves(C.byref(p), n, _lib.dptr(theta), _lib.dptr(ygp),
                                              _lib.dptr(dL), _lib.dptr(m), _lib.dptr(resid),
                                              _lib.dptr(br)))
    return {"dL": dL, "m": m, "resid": resid, "br": br}


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
