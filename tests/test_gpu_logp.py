"""HIP log-density + gradient (fitoct_logp_grad -> logp_kernel) vs the oracles.

Tolerances (written here):
* f64 path: |lp - lp_ref| <= 1e-11 (1 + |lp_ref|); |g - g_ref| <= 1e-8 (1 + |g_ref|)
  (differences are summation order only: wave-tree vs sequential sums).
* mixed path (f32 per-bin sweep, f64 reductions + state):
  lp 1e-5 (1 + |lp|), grad 2e-3 (1 + |g|).
The factorised polynomial basis (MODE_POLY, chosen automatically in f64) and the
explicit row basis (MODE_ROWS: user-supplied B, or mixed precision) are both covered.
"""
from __future__ import annotations

import math
import os

import numpy as np
import pytest

from conftest import golden_files, load_golden, problems_from_fixture
from fitoct_amd import ExpGPProblem, logp_grad
from fitoct_amd.synth import default_prior, synth_decay
from oracle import model_np as M

pytestmark = pytest.mark.gpu

TOL = {"f64": (1e-11, 1e-8), "mixed": (1e-5, 2e-3)}


def _check(lp, g, s2, prob_np, Q, prec):
    tl, tg = TOL[prec]
    for i, q in enumerate(Q):
        rl, rg, rs = M.logp_grad(q, prob_np)
        if not math.isfinite(rl):
            assert lp[i] == -math.inf
            continue
        assert abs(lp[i] - rl) <= tl * (1 + abs(rl)), (i, lp[i], rl)
        err = np.abs(g[i] - rg) / (1 + np.abs(rg))
        assert err.max() <= tg, (i, err.max(), int(err.argmax()))
        if math.isfinite(rs):
            assert abs(s2[i] - rs) <= 10 * tl * (1 + abs(rs))


def _points(prob, rng, P=9, spread=0.3):
    t0 = prob.theta0
    q = rng.normal(0, spread, (P, prob.D))
    q[:, 0:3] = np.log(t0) + rng.normal(0, 0.02, (P, 3))
    q[:, -1] = rng.normal(0, 0.3, P)
    return q


@pytest.mark.parametrize("path", golden_files("logp"), ids=lambda p: os.path.basename(p))
@pytest.mark.parametrize("prec", ["f64", "mixed"])
def test_golden_vectors(path, prec):
    fx = load_golden(path)
    prob, npp = problems_from_fixture(fx)
    lp, g, s2 = logp_grad(prob, fx["q"], prec)
    _check(lp, g, s2, npp, fx["q"], prec)


CASES = [
    # (N, family, Nn, grid, prior_PD, data_type, kernel_conv, lambda_conv)
    (512, "normal", 15, "extremal", 0, 2, 0, 0),        # config 2 shape
    (2048, "horseshoe", 15, "extremal", 0, 2, 0, 0),    # config 3 shape
    (4096, "lasso", 15, "extremal", 0, 2, 0, 0),        # config 4 shape
    (481, "normal", 15, "extremal", 0, 2, 0, 0),        # config 5 / synthData.R x = 20:500
    (481, "horseshoe", 10, "internal", 1, 2, 0, 0),     # prior predictive (priPost.R:14)
    (700, "horseshoe", 20, "internal", 0, 1, 1, 1),     # amplitude data, RMgauss, rate conv
    (2047, "lasso", 5, "internal", 0, 2, 0, 0),         # ragged
    (8192, "normal", 15, "extremal", 0, 2, 0, 0),       # > 4096 bins: streamed from HBM
    (3001, "horseshoe", 15, "extremal", 0, 2, 0, 0),    # 16 bins per lane, padded
    (2049, "normal", 15, "internal", 0, 1, 0, 0),       # 16 bins per lane, mostly padding
    (2, "normal", 2, "extremal", 0, 2, 0, 0),           # minimum shape
    (97, "horseshoe", 24, "extremal", 0, 2, 0, 0),      # maximum Nn
    (1025, "normal", 8, "internal", 0, 2, 0, 0),        # just over a bins-per-thread step
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"N{c[0]}-{c[1]}-Nn{c[2]}-pd{c[4]}")
@pytest.mark.parametrize("prec", ["f64", "mixed"])
def test_config_shapes(case, prec):
    N, fam, Nn, grid, pd, dt, kc, lc = case
    t0, S0 = default_prior()
    if dt == 1:
        t0 = np.array([1000.0, 2000.0, 150.0])
        S0 = np.diag((0.05 * t0) ** 2)
    d = synth_decay(N, "sincExp", N + 3)
    kw = dict(Nn=Nn, theta0=t0, Sigma0=S0, prior_PD=pd, kernel_conv=kc, lambda_conv=lc)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], dataType=dt, gridType=grid, prior_type=fam, **kw)
    npp = M.Problem(d["x"], d["y"], d["uy"], data_type=dt, grid_type=grid,
                    family=M.FAMILIES[fam], **kw)
    Q = _points(prob, np.random.default_rng(N + Nn))
    lp, g, s2 = logp_grad(prob, Q, prec)
    _check(lp, g, s2, npp, Q, prec)


def test_user_basis_rows_mode():
    """A caller-supplied B (fitoct_problem.B) bypasses the factorised basis."""
    t0, S0 = default_prior()
    d = synth_decay(1000, "sincExp3", 5)
    B, _ = M.gp_basis(d["x"], 12, "extremal", 1 / 12)
    B = B * 0.9 + 0.01                 # not an SE basis: the polynomial mode cannot represent it
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=12, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="lasso", B=B)
    npp = M.Problem(d["x"], d["y"], d["uy"], Nn=12, grid_type="extremal", theta0=t0, Sigma0=S0,
                    family=M.LASSO, B=B)
    Q = _points(prob, np.random.default_rng(3))
    _check(*logp_grad(prob, Q, "f64"), npp, Q, "f64")


def test_non_physical_guard_and_many_points():
    """1+dL <= 0 -> lp = -inf; thousands of points in one call (multi-tile batches)."""
    t0, S0 = default_prior()
    d = synth_decay(512, "sincExp", 1)
    prob = ExpGPProblem(d["x"], d["y"], d["uy"], Nn=15, gridType="extremal", theta0=t0,
                        Sigma0=S0, prior_type="normal")
    npp = M.Problem(d["x"], d["y"], d["uy"], Nn=15, grid_type="extremal", theta0=t0, Sigma0=S0)
    rng = np.random.default_rng(11)
    Q = _points(prob, rng, P=3000, spread=0.05)
    Q[::7, 3:18] = -4.0                # guard rows
    lp, g, s2 = logp_grad(prob, Q, "f64")
    assert np.all(lp[::7] == -np.inf)
    sel = rng.choice(3000, 40, replace=False)
    _check(lp[sel], g[sel], s2[sel], npp, Q[sel], "f64")


def test_large_y_over_uy_conditioning():
    """Rounding of the staged residual: the kernel stages y / uy per bin and
    forms (y - m) / uy as fma(-m, 1/uy, y/uy); the oracles compute (y - m) * (1/uy).  Both
    are exact to a few ulps of y/uy, so with |y/uy| ~ 4e6 and residuals ~ 1 each residual
    carries ~1e-9 absolute error whichever form is used.  The tolerances below are the
    1e-11 / 1e-8 of the other tests plus that conditioning term: 8 eps sum |d_i| |y_i/uy_i|
    on lp (d_i = residual), and the same amplification (|y/uy| / |d|) on the gradient."""
    t0 = np.array([2.0e6, 3000.0, 300.0])
    x = np.linspace(20.0, 500.0, 512)
    uy = np.full(512, 0.5)
    rng = np.random.default_rng(5)
    y = t0[0] + t0[1] * np.exp(-2.0 * x / t0[2]) + uy * rng.standard_normal(512)
    S0 = np.diag((0.05 * t0) ** 2)
    prob = ExpGPProblem(x, y, uy, Nn=10, gridType="extremal", theta0=t0, Sigma0=S0,
                        prior_type="normal")
    npp = M.Problem(x, y, uy, Nn=10, grid_type="extremal", theta0=t0, Sigma0=S0)
    Q = np.zeros((6, prob.D))
    Q[:, 0:3] = np.log(t0) + rng.normal(0, 1e-7, (6, 3))   # residuals O(1)
    Q[:, 3:13] = rng.normal(0, 1e-4, (6, 10))
    Q[:, 13] = np.log(0.1)
    lp, g, _ = logp_grad(prob, Q, "f64")
    eps = np.finfo(float).eps
    for i, q in enumerate(Q):
        rl, rg, _ = M.logp_grad(q, npp)
        th = np.exp(q[:3])
        d = (y - (th[0] + th[1] * np.exp(-2.0 * x / th[2]))) / uy
        kappa = float(np.median(np.abs(y / uy)) / max(np.median(np.abs(d)), 1e-300))
        tol = 1e-11 * (1 + abs(rl)) + 8 * eps * float(np.sum(np.abs(d) * np.abs(y / uy)))
        assert abs(lp[i] - rl) <= tol, (i, lp[i], rl, tol)
        err = np.abs(g[i] - rg) / (1 + np.abs(rg))
        assert err.max() <= 1e-8 * max(1.0, kappa), (i, err.max(), kappa)
