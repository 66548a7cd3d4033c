"""The oracles themselves: numpy restatement vs finite differences and the
golden fixtures, C oracle vs numpy, Philox known answers.  (CPU only.)

What pins the model restatement (the reference has no golden
vectors, rstan is absent -> parity unpinned vs rstan): analytic gradients vs
central finite differences, the GP basis' interpolation property
(server.R:623-650), and the committed fixtures of tests/golden/make_golden.py.
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_files, load_golden, problems_from_fixture, rel_err
from oracle import model_np as M

FIXTURES = golden_files("logp")


@pytest.fixture(scope="module")
def oracle_c():
    from oracle import nuts_c
    return nuts_c


def test_fixtures_present():
    assert len(FIXTURES) >= 6
    assert len(golden_files("draws")) >= 2


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p))
def test_numpy_oracle_reproduces_golden(path):
    fx = load_golden(path)
    _, P = problems_from_fixture(fx)
    np.testing.assert_allclose(P.B, fx["B"], rtol=0, atol=1e-12)
    for q, lp, g, s2 in zip(fx["q"], fx["lp"], fx["grad"], fx["sumr2"]):
        lp2, g2, s22 = M.logp_grad(q, P)
        assert lp2 == pytest.approx(lp, rel=1e-13, abs=1e-9)
        np.testing.assert_allclose(g2, g, rtol=1e-11, atol=1e-9)
        if np.isfinite(s2):
            assert s22 == pytest.approx(s2, rel=1e-12)


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p))
def test_gradient_matches_finite_differences(path):
    fx = load_golden(path)
    _, P = problems_from_fixture(fx)
    for q in fx["q"][:2]:
        _, g, _ = M.logp_grad(q, P)
        fd = M.fd_grad(q, P, h=1e-6)
        scale = np.maximum(1.0, np.abs(g))
        assert np.max(np.abs(fd - g) / scale) < 2e-4


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p))
def test_c_oracle_matches_numpy(path, oracle_c):
    fx = load_golden(path)
    prob, _ = problems_from_fixture(fx)
    if fx["meta"]["family"] != "monoexp":   # no GP basis in the mono-exponential model
        np.testing.assert_allclose(oracle_c.basis(prob), fx["B"], rtol=0, atol=1e-11)
    lp, g, s2 = oracle_c.logp_grad(prob, fx["q"])
    np.testing.assert_allclose(lp, fx["lp"], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(g, fx["grad"], rtol=1e-10, atol=1e-8)
    fin = np.isfinite(fx["sumr2"])
    np.testing.assert_allclose(s2[fin], fx["sumr2"][fin], rtol=1e-12)


def test_philox_known_answers(oracle_c):
    with open(os.path.join(GOLDEN, "philox_kat.json")) as f:
        kats = json.load(f)
    for k in kats:
        assert oracle_c.philox(k["ctr"], k["key"]) == k["out"]


@pytest.mark.parametrize("grid", ["internal", "extremal"])
@pytest.mark.parametrize("Nn", [5, 10, 15, 20])
def test_gp_grid_and_interpolation(grid, Nn):
    """server.R:627-631 grid; B = K_xG K_GG^-1 reproduces the control values
    at the control points (conditional-mean interpolator)."""
    xg = M.gp_grid(Nn, grid)
    if grid == "extremal":
        np.testing.assert_allclose(xg, np.linspace(0, 1, Nn))
    else:
        dx = 1 / (Nn + 1)
        assert xg[0] == pytest.approx(dx / 2) and xg[-1] == pytest.approx(1 - dx / 2)
    x = 20 + 480 * xg if grid == "extremal" else np.r_[20.0, 20 + 480 * xg, 500.0]
    B, _ = M.gp_basis(x, Nn, grid, 1.0 / Nn)
    rows = B if grid == "extremal" else B[1:-1]
    np.testing.assert_allclose(rows, np.eye(Nn), atol=2e-6)


def test_non_physical_decay_length_guard():
    """Appendix A guard: 1 + dL <= 0 -> lp = -inf (a rejected/divergent state)."""
    fx = load_golden(os.path.join(GOLDEN, "logp_normal_n64.npz"))
    _, P = problems_from_fixture(fx)
    q = fx["q"][0].copy()
    q[3:3 + P.Nn] = -5.0
    lp, _, _ = M.logp_grad(q, P)
    assert lp == -math.inf


def test_prior_pd_drops_likelihood():
    """priPost.R:14: prior_PD=1 -> lp independent of the data."""
    fx = load_golden(os.path.join(GOLDEN, "logp_normal_prior_n64.npz"))
    _, P = problems_from_fixture(fx)
    q = fx["q"][0]
    lp1 = M.logp_grad(q, P)[0]
    P.y = P.y + 100.0
    assert M.logp_grad(q, P)[0] == lp1


def test_dims_and_names():
    for fam, D in [(M.NORMAL, 20), (M.LASSO, 19), (M.HORSESHOE, 51)]:
        assert M.dim(fam, 15) == D
        assert len(M.param_names(fam, 15)) == D
