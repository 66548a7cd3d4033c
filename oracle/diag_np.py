"""ORACLE (test infrastructure only) -- numpy restatement of the convergence
diagnostics rstan::summary prints (server.R:88-104): split R-hat
(stan::analyze::compute_split_potential_scale_reduction) and n_eff
(compute_split_effective_sample_size: Geyer's initial positive + monotone
sequence).  Checks libfitoct's C++ implementation (fitoct_split_rhat_ess).
Parity unpinned against rstan (not installable here); the formulas follow
Stan's published algorithm (Stan Reference Manual, "Effective sample size").
"""
from __future__ import annotations

import numpy as np


def _split(x):
    n = x.shape[1]
    h = n // 2
    return np.concatenate([x[:, :h], x[:, n - h:]], axis=0)


def psr(chains):
    m, n = chains.shape
    means = chains.mean(1)
    var = chains.var(1, ddof=1)
    B = n * means.var(ddof=1)
    W = var.mean()
    return float(np.sqrt((B / W + n - 1) / n))


def split_rhat(x):
    return psr(_split(np.asarray(x, float)))


def _acov(v):
    n = v.size
    c = v - v.mean()
    f = np.fft.rfft(c, 2 * n)
    ac = np.fft.irfft(f * np.conj(f))[:n]
    return ac / n


def ess(chains):
    m, n = chains.shape
    acov = np.array([_acov(c) for c in chains])
    mean_var = (acov[:, 0] * n / (n - 1)).mean()
    var_plus = mean_var * (n - 1) / n
    if m > 1:
        var_plus += chains.mean(1).var(ddof=1)
    rho = np.zeros(n + 2)
    rho[0] = 1.0
    rho_even = 1.0
    rho_odd = 1 - (mean_var - acov[:, 1].mean()) / var_plus
    rho[1] = rho_odd
    t = 1
    while t < n - 4 and rho_even + rho_odd > 0:
        rho_even = 1 - (mean_var - acov[:, t + 1].mean()) / var_plus
        rho_odd = 1 - (mean_var - acov[:, t + 2].mean()) / var_plus
        if rho_even + rho_odd >= 0:
            rho[t + 1] = rho_even
            rho[t + 2] = rho_odd
        t += 2
    max_t = t
    if rho_even > 0:
        rho[max_t + 1] = rho_even
    t = 1
    while t <= max_t - 2:
        if rho[t + 1] + rho[t + 2] > rho[t - 1] + rho[t]:
            rho[t + 1] = (rho[t - 1] + rho[t]) / 2
            rho[t + 2] = rho[t + 1]
        t += 2
    N = m * n
    tau = -1 + 2 * rho[:max_t + 1].sum() + rho[max_t + 1]
    tau = max(tau, 1 / np.log10(N))
    return float(N / tau)


def split_ess(x):
    return ess(_split(np.asarray(x, float)))
