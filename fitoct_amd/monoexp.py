"""``FitOCTLib::fitMonoExp`` and ``printBr`` on the HIP engine.

The reference calls ``fitMonoExp(x, y, uy, dataType)`` (FitOCT.R:95,
server.R:341-343) and reads ``best.theta`` / ``cor.theta`` (FitOCT.R:96-97),
``fit$par$m`` / ``fit$par$resid`` (plotMonoExp.R:15-16), ``fit$hessian``
(server.R:117-126) and the Birge ratio through ``printBr`` (plotMonoExp.R:10,
FitOCT.R:100).  FitOCTLib itself is not in the reference tree, so the model is
restated (⚑, include/fitoct.h FITOCT_MODEL_MONOEXP):

    y_i ~ N(theta1 + theta2 exp(-c x_i / theta3), uy_i),  theta > 0, flat prior.

``method='optim'`` is rstan::optimizing (:func:`fitoct_amd.optim_vb.optimizing`:
native L-BFGS on the log density without the Jacobian -- the mode in theta --
then the Hessian of that function in the unconstrained (log theta) space by
central differences of the gradient, as rstan's optimHess computes it).  Every
log density / gradient is a launch of the HIP gradient kernel.
``method='sample'`` runs the device NUTS sampler on the same model.
"""
from __future__ import annotations

import numpy as np

from .api import ExpGPProblem, SamplerConfig, sample
from .optim_vb import OptimFit, optimizing


def initial_theta(x, y, dataType=2):
    """A rough (theta1, theta2, theta3) from the data alone (log-linear fit of the
    decay above its tail level; ``fitoct_mono_initial_theta``, shared with the R
    shim); only the optimiser's / sampler's start."""
    import ctypes as C

    from . import _lib
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    if x.shape != y.shape or x.ndim != 1:
        raise ValueError("x and y must be 1-D arrays of equal length")
    out = np.empty(3)
    _lib.check(_lib.lib().fitoct_mono_initial_theta(x.size, _lib.dptr(x), _lib.dptr(y),
                                                    int(dataType), _lib.dptr(out)))
    return out


def mono_problem(x, y, uy, dataType=2, theta0=None) -> ExpGPProblem:
    t0 = initial_theta(x, y, dataType) if theta0 is None else np.asarray(theta0, float)
    return ExpGPProblem(x, y, uy, dataType=dataType, Nn=2, theta0=t0,
                        Sigma0=np.eye(3), prior_type="monoexp")


def decay(x, theta, dataType=2):
    """``theta1 + theta2 exp(-c x / theta3)`` (ShinyInterface/ui.R:88)."""
    x = np.asarray(x, float)
    return theta[0] + theta[1] * np.exp(-float(dataType) * x / theta[2])


def fitMonoExp(x, y, uy, dataType=2, method="optim", *, nb_warmup=500, nb_iter=1500,
               nb_chains=4, seed=None, theta0=None, device=0, hessian_step=1e-3):
    """Drop-in for ``FitOCTLib::fitMonoExp`` (FitOCT.R:95).  Returns
    ``dict(fit, method, best.theta, cor.theta)``."""
    prob = mono_problem(x, y, uy, dataType, theta0)
    if seed is None and method != "optim":
        seed = int(np.random.SeedSequence().entropy & 0xFFFFFFFF)
    if method == "sample":
        from .stanfit import StanFit
        cfg = SamplerConfig(chains=nb_chains, warmup=nb_warmup, samples=nb_iter - nb_warmup,
                            seed=seed, device=device)
        fit = StanFit.from_output(sample(prob, cfg), prob)
        th = fit.as_matrix("theta")
        return {"fit": fit, "method": method, "best.theta": th.mean(axis=0),
                "cor.theta": np.corrcoef(th.T)}
    if method != "optim":
        raise ValueError(f"method={method!r}: 'optim' or 'sample'")
    fit = optimizing(prob, np.log(prob.theta0), hessian_step=hessian_step, device=device)
    theta = fit.par["theta"]
    m = decay(x, theta, dataType)
    fit.par["m"] = m
    fit.par["resid"] = (np.asarray(y, float) - m) / np.asarray(uy, float)
    cov_q = np.linalg.inv(-fit.hessian)
    cov = cov_q * np.outer(theta, theta)           # delta method back to theta
    sd = np.sqrt(np.diag(cov))
    return {"fit": fit, "method": method, "best.theta": theta,
            "cor.theta": cov / np.outer(sd, sd)}


def printBr(fit, N=None, silent=False, prob=0.95):
    """Birge ratio and its probability interval (FitOCTLib::printBr, used at
    plotMonoExp.R:10 and FitOCT.R:100).  Under the model, N * br ~ chi2_N, so
    ``br`` outside the central ``prob`` interval of chi2_N / N raises ``alert``."""
    from scipy.stats import chi2
    if isinstance(fit, OptimFit):
        br = fit.par["br"]
        N = N or fit.N or len(fit.par["resid"])
    else:
        draws = fit.extract("br", permuted=True)["br"]
        br = float(np.mean(draws))
        if N is None:
            raise ValueError("N (number of bins) is required for a sampled fit")
    lo, hi = chi2.ppf([(1 - prob) / 2, (1 + prob) / 2], N) / N
    alert = None
    if not (lo <= br <= hi):
        alert = (f"br = {br:.4g} outside the {100 * prob:g} % probability interval "
                 f"[{lo:.4g}, {hi:.4g}]")
    if not silent:
        print(f"br = {br:.4g}, {100 * prob:g} % probability interval [{lo:.4g}, {hi:.4g}]"
              + (f"\nAlert: {alert}" if alert else ""))
    return {"br": br, "interval": (float(lo), float(hi)), "alert": alert}
