"""ORACLE (test infrastructure only) -- restatement of Stan's mean-field ADVI
(rstan::vb defaults; stan/variational/advi.hpp, families/normal_meanfield.hpp
-- an external dependency, not in /root/reference) over the C oracle's log
density (oracle/fitoct_oracle.c).  It addresses the same Philox normals as
libfitoct's fitoct_vb (key = (seed, stream), counter = (iteration, tag,
draw, d/2)), so the two trajectories agree up to floating-point rounding of
the gradients.  Parity vs rstan: **unpinned** (Stan draws its normals from
boost's ecuyer1988 sequentially; no reference test pins vb output).

Only tests/ may import this module.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import gammaln

from . import nuts_c

GRAD, ELBO, OUT = 0xAD01, 0xAD02, 0xAD03
S_ELBO_INIT, S_SGA, S_OUT = 16, 17, 18
ETAS = (100.0, 10.0, 1.0, 0.1, 0.01)


def lp_constant(prob) -> float:
    """Constants of the model's sampling statements (log_prob<propto=false>)."""
    l2pi = math.log(2 * math.pi)
    c = 0.0
    if not prob.prior_PD:
        c += -0.5 * prob.N * l2pi - float(np.log(prob.uy).sum())
    if prob.prior_type == "monoexp":
        return c
    c += -1.5 * l2pi - 0.5 * math.log(np.linalg.det(prob.Sigma0))
    c += -0.5 * l2pi - math.log(prob.sigma_scale)
    Nn = prob.Nn
    if prob.prior_type == "normal":
        rate = 1.0 / prob.lambda_rate if prob.lambda_conv == 0 else prob.lambda_rate
        c += -0.5 * Nn * l2pi + math.log(rate)
    elif prob.prior_type == "horseshoe":
        a = 0.5 * prob.nu
        c += -Nn * l2pi + Nn * (a * math.log(a) - gammaln(a))
        c += -0.5 * l2pi + 0.5 * math.log(0.5) - gammaln(0.5)
    return c


def default_init(prob) -> np.ndarray:
    q = np.zeros(prob.D)
    q[:3] = np.log(prob.theta0)
    if prob.prior_type == "normal":
        rate = 1.0 / prob.lambda_rate if prob.lambda_conv == 0 else prob.lambda_rate
        q[3 + prob.Nn] = -math.log(rate)
    return q


class _Advi:
    def __init__(self, prob, seed, grad_samples, elbo_samples):
        self.prob, self.seed = prob, seed
        self.gs, self.es = grad_samples, elbo_samples
        self.D = prob.D
        self.const = lp_constant(prob)

    def eta(self, stream, tag, it, s):
        return nuts_c.normals(self.seed, stream, tag, it, s, self.D)

    def elbo(self, mu, om, stream, it):
        E = np.stack([self.eta(stream, ELBO, it, s) for s in range(self.es)])
        lp, _, _ = nuts_c.logp_grad(self.prob, mu + np.exp(om) * E)
        lp = lp + self.const
        ok = np.isfinite(lp)
        if not ok.any():
            return -math.inf
        return lp[ok].sum() / self.es + 0.5 * self.D * (1 + math.log(2 * math.pi)) + om.sum()

    def grad(self, mu, om, stream, it):
        """Draws with a non-finite density or gradient are dropped (count in the
        mean as 0); all dropped -> zero step (libfitoct's documented deviation
        from Stan, which throws)."""
        E = np.stack([self.eta(stream, GRAD, it, s) for s in range(self.gs)])
        lp, G, _ = nuts_c.logp_grad(self.prob, mu + np.exp(om) * E)
        valid = np.isfinite(lp) & np.all(np.isfinite(G), axis=1)
        if not valid.any():
            return np.zeros_like(mu), np.zeros_like(om), False
        Gv = np.where(valid[:, None], G, 0.0)
        gmu = Gv.sum(axis=0) / self.gs
        gom = (Gv * E).sum(axis=0) / self.gs * np.exp(om) + 1.0
        return gmu, gom, True


def _step(mu, om, gmu, gom, hmu, hom, it, eta):
    if it == 1:
        hmu, hom = hmu + gmu ** 2, hom + gom ** 2
    else:
        hmu, hom = 0.9 * hmu + 0.1 * gmu ** 2, 0.9 * hom + 0.1 * gom ** 2
    es = eta / math.sqrt(it)
    return mu + es * gmu / (1 + np.sqrt(hmu)), om + es * gom / (1 + np.sqrt(hom)), hmu, hom


def vb(prob, seed=1234, init=None, iter=10000, grad_samples=1, elbo_samples=100,
       eval_elbo=100, adapt_iter=50, tol_rel_obj=0.01, adapt_engaged=True, eta=1.0):
    """-> dict(mu, omega, eta, elbo, iterations, converged)."""
    A = _Advi(prob, seed, grad_samples, elbo_samples)
    D = prob.D
    q0 = default_init(prob) if init is None else np.asarray(init, float)
    eta_best = eta if not adapt_engaged else _adapt(A, prob, q0, adapt_iter)
    return _ascent(A, q0, eta_best, iter, eval_elbo, tol_rel_obj)


def _adapt(A, prob, q0, adapt_iter):
    D = prob.D
    # eta adaptation: each candidate from the initial point, then the sequential rule
    elbos = []
    for k, eta in enumerate(ETAS):
        mu, om = q0.copy(), np.zeros(D)
        hmu, hom = np.zeros(D), np.zeros(D)
        for it in range(1, adapt_iter + 1):
            gmu, gom, _ = A.grad(mu, om, k, it)
            mu, om, hmu, hom = _step(mu, om, gmu, gom, hmu, hom, it, eta)
        elbos.append(A.elbo(mu, om, k, 0))
    elbo_init = A.elbo(q0, np.zeros(D), S_ELBO_INIT, 0)
    best, eta_best, found = -math.inf, 0.0, False
    for k, el in enumerate(elbos):
        if el < best and best > elbo_init:
            found = True
            break
        if k < len(ETAS) - 1:
            best, eta_best = el, ETAS[k]
        elif el > elbo_init:
            eta_best, found = ETAS[k], True
    if not found:
        raise RuntimeError("all proposed step-sizes failed")
    return eta_best


def _ascent(A, q0, eta_best, iter, eval_elbo, tol_rel_obj):
    D = q0.size
    mu, om = q0.copy(), np.zeros(D)
    hmu, hom = np.zeros(D), np.zeros(D)
    cb, cb_size = [], int(max(0.1 * iter / eval_elbo, 2.0))
    elbo, it, conv = 0.0, 1, False
    while True:
        gmu, gom, _ = A.grad(mu, om, S_SGA, it)
        mu, om, hmu, hom = _step(mu, om, gmu, gom, hmu, hom, it, eta_best)
        if it % eval_elbo == 0:
            prev, elbo = elbo, A.elbo(mu, om, S_SGA, it)
            if not np.isfinite(elbo):
                raise RuntimeError("every ELBO draw was dropped")
            cb = (cb + [abs((prev - elbo) / elbo)])[-cb_size:]
            med = sorted(cb)[len(cb) // 2]
            if np.mean(cb) < tol_rel_obj or med < tol_rel_obj:
                conv = True
                break
        if it >= iter:
            break
        it += 1
    return {"mu": mu, "omega": om, "eta": eta_best, "elbo": elbo, "iterations": it,
            "converged": conv}
