"""``method='optim'`` and ``method='vb'`` of FitOCTLib::fitExpGP / fitMonoExp
(FitOCT.R:42, ui.R:107-114) over the C ABI.

* :func:`optimizing` -- ``rstan::optimizing``: L-BFGS on the log density
  without Jacobian, Hessian of the unconstrained log density by central
  differences of the gradient (rstan's optimHess).  Returns an
  :class:`OptimFit` with ``par`` (named like ``fit$par[['theta']]``,
  server.R:66,114,161), ``value`` and ``hessian`` (``sqrt(-1/H[p,p])`` is the
  standard error the Shiny app shows, server.R:70-77).
* :func:`vb` -- ``rstan::vb`` mean-field ADVI; returns a
  :class:`fitoct_amd.stanfit.StanFit` of ``output_samples`` draws, which
  ``print(fit, pars)`` / ``extract(fit, 'br')`` read as for a sampled fit
  (plotExpGP.R:8-11).

Both drivers run natively in libfitoct (fitoct_amd/csrc/optimize.cpp); every
density evaluation is a batched launch of the sampler's gradient kernel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import PREC, check, dptr, lib


class Evaluator:
    """Persistent batched log density / gradient (``fitoct_evaluator``)."""

    def __init__(self, prob, capacity: int, precision: str = "f64", device: int = 0):
        self.prob = prob
        self._p = prob.to_c()
        h = C.c_void_p()
        check(lib().fitoct_evaluator_create(C.byref(self._p), int(capacity), PREC[precision],
                                            int(device), C.byref(h)))
        self._h = h
        self.capacity = int(capacity)

    def __call__(self, q, jacobian: bool = True, normalised: bool = False, grad: bool = True):
        q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
        n, D = q.shape
        if D != self.prob.D:
            raise ValueError(f"q has {D} columns, model dimension is {self.prob.D}")
        lp, s2 = np.empty(n), np.empty(n)
        g = np.empty((n, D)) if grad else None
        for a in range(0, n, self.capacity):
            b = min(n, a + self.capacity)
            check(lib().fitoct_evaluator_run(
                self._h, b - a, dptr(q[a:b]), int(jacobian), int(normalised), dptr(lp[a:b]),
                dptr(g[a:b]) if grad else None, dptr(s2[a:b])))
        return lp, g, s2

    def close(self):
        if getattr(self, "_h", None):
            lib().fitoct_evaluator_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def constrain(prob, q: np.ndarray) -> np.ndarray:
    """Unconstrained q[n, D] -> constrained parameters in draw-column order."""
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
    out = np.empty_like(q)
    check(lib().fitoct_constrain(prob.family, prob.Nn, q.shape[0], dptr(q), dptr(out)))
    return out


def param_columns(prob) -> list:
    """Names of the D model parameters (draw columns 7..7+D-1)."""
    return prob.column_names()[7:7 + prob.D]


def _named(prob, values: np.ndarray, sumr2: float) -> dict:
    """``fit$par`` (rstan as_vector=FALSE): base name -> array or scalar, with the
    transformed parameters of the horseshoe model and the Birge ratio."""
    from .stanfit import _base, materialise, output_columns
    row = materialise(np.concatenate([values, [sumr2 / prob.N]])[None, :], prob, n_lead=0)
    par = {}
    for c, v in zip(output_columns(prob, lead=()), row[0]):
        par.setdefault(_base(c), []).append(float(v))
    return {k: (np.array(v) if len(v) > 1 or k in ("theta", "yGP") else v[0])
            for k, v in par.items()}


class OptimFit:
    """rstan::optimizing-shaped result: ``par``, ``value``, ``hessian``."""

    def __init__(self, par, value, hessian, names, return_code=0, iterations=0,
                 termination="", unconstrained=None, sumr2=None, N=None):
        self.par = par
        self.value = value
        self.hessian = hessian
        self.hessian_names = names
        self.return_code = return_code
        self.iterations = iterations
        self.termination = termination
        self.unconstrained = unconstrained
        self.sumr2 = sumr2
        self.N = N                      # depth bins (printBr's chi2_N interval)

    def se(self):
        """Standard errors on the unconstrained scale, ``sqrt(-1/H[p,p])``
        (server.R:70-77)."""
        return dict(zip(self.hessian_names, np.sqrt(-1.0 / np.diag(self.hessian))))

    def __repr__(self):
        return f"OptimFit(theta={self.par['theta']}, value={self.value:.6g})"


def optimizing(prob, init=None, *, iter=2000, history=5, init_alpha=1e-3, tol_obj=1e-12,
               tol_rel_obj=1e4, tol_grad=1e-8, tol_rel_grad=1e7, tol_param=1e-8,
               hessian=True, hessian_step=1e-3, jacobian=False, precision="f64",
               device=0) -> OptimFit:
    """``rstan::optimizing(model, hessian=TRUE)`` on the GPU density (Stan defaults)."""
    c = _lib.OptimConfig()
    lib().fitoct_default_optim_config(C.byref(c))
    c.iter, c.history, c.init_alpha = int(iter), int(history), float(init_alpha)
    c.tol_obj, c.tol_rel_obj, c.tol_grad = tol_obj, tol_rel_obj, tol_grad
    c.tol_rel_grad, c.tol_param = tol_rel_grad, tol_param
    c.hessian, c.hessian_step, c.jacobian = int(hessian), float(hessian_step), int(jacobian)
    c.precision, c.device = PREC[precision], int(device)
    D = prob.D
    x = np.empty(D)
    H = np.empty((D, D)) if hessian else None
    r = _lib.OptimResult()
    r.par, r.hessian = dptr(x), dptr(H)
    q0 = None if init is None else np.ascontiguousarray(init, dtype=np.float64).reshape(D)
    p = prob.to_c()
    check(lib().fitoct_optimize(C.byref(p), C.byref(c), dptr(q0), C.byref(r)))
    par = _named(prob, constrain(prob, x)[0], r.sumr2)
    return OptimFit(par, float(r.value), H, param_columns(prob), int(r.return_code),
                    int(r.iterations), _lib.TERMINATION.get(r.termination, str(r.termination)),
                    unconstrained=x, sumr2=float(r.sumr2), N=prob.N)


def vb(prob, init=None, *, iter=10000, grad_samples=1, elbo_samples=100, eval_elbo=100,
       eta=1.0, adapt_engaged=True, adapt_iter=50, tol_rel_obj=0.01, output_samples=1000,
       seed=1234, precision="f64", device=0):
    """``rstan::vb(model)`` (algorithm='meanfield', Stan defaults) -> StanFit."""
    from .genquant import expgp_curves
    from .stanfit import StanFit, materialise, output_columns
    c = _lib.VbConfig()
    lib().fitoct_default_vb_config(C.byref(c))
    c.iter, c.grad_samples, c.elbo_samples = int(iter), int(grad_samples), int(elbo_samples)
    c.eval_elbo, c.eta, c.adapt_engaged = int(eval_elbo), float(eta), int(adapt_engaged)
    c.adapt_iter, c.tol_rel_obj, c.output_samples = int(adapt_iter), tol_rel_obj, int(output_samples)
    c.seed, c.precision, c.device = int(seed), PREC[precision], int(device)
    D, S = prob.D, int(output_samples)
    mu, om = np.empty(D), np.empty(D)
    q = np.empty((S, D))
    lp, lg, s2 = np.empty(S), np.empty(S), np.empty(S)
    r = _lib.VbResult()
    r.mu, r.omega, r.draws = dptr(mu), dptr(om), dptr(q)
    r.log_p, r.log_g, r.sumr2 = dptr(lp), dptr(lg), dptr(s2)
    q0 = None if init is None else np.ascontiguousarray(init, dtype=np.float64).reshape(D)
    p = prob.to_c()
    check(lib().fitoct_vb(C.byref(p), C.byref(c), dptr(q0), C.byref(r)))
    lead = ["lp__", "log_p__", "log_g__"]
    raw = np.concatenate([np.zeros((S, 1)), lp[:, None], lg[:, None], constrain(prob, q),
                          (s2 / prob.N)[:, None]], axis=1)[None]
    body, cols = materialise(raw, prob, n_lead=3), output_columns(prob, lead=lead)
    mean = _named(prob, constrain(prob, mu)[0], float("nan"))
    # br at the mean of the approximation (the first row of CmdStan's variational CSV)
    ygp = mean.get("yGP", np.zeros(0)) if prob.prior_type != "monoexp" else None
    mean_s2 = float(expgp_curves(prob, mean["theta"], ygp)["br"][0] * prob.N)
    return StanFit(body, cols, 0, model_name="ExpGP (meanfield ADVI)",
                   source=("vb", prob, c, mu, mean_s2, q, lp, lg, s2, float(r.eta)),
                   meta={"method": "vb", "mu": mu, "omega": om, "mean": mean,
                         "eta": float(r.eta), "elbo": float(r.elbo),
                         "iterations": int(r.iterations), "converged": bool(r.converged),
                         "n_evals": int(r.n_evals), "prior_type": prob.prior_type,
                         "prior_PD": prob.prior_PD})
