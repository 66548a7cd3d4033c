"""Upstream preparation of one OCT decay: the host-side
steps FitOCT.R runs before ``fitExpGP`` (FitOCT.R:84-107, server.R:304-406).

``selX``, ``estimateNoise`` and ``estimateExpPrior`` live in FitOCTLib, which is
not in the reference tree, so their behaviour is restated from
the call sites and the UI's descriptions (⚑ = assumption; "parity unpinned"):

* ``selX(x, y, depthSel, subSample)`` (FitOCT.R:85, server.R:304): keep the bins
  with ``depthSel[0] <= x <= depthSel[1]`` (``None``: all; Tests/statsSplineSmooth.R
  selects ``x > 20 & x <= 500`` the same way), then every ``subSample``-th one.
* ``estimateNoise(x, y, df)`` (FitOCT.R:89-91, ui.R:58-63,81): a cubic smoothing
  spline with ``df`` equivalent degrees of freedom (R ``smooth.spline(x, y, df)``;
  Tests/statsSplineSmooth.R:19-22) gives ``ySmooth``; the residuals are fitted
  by the noise model ``uy(x) = a_1 exp(-x / a_2)`` (ui.R:81) at its maximum
  likelihood (the reference runs Stan ``optimizing``, server.R:59-79 reads
  ``fit$par$theta``).  ⚑ smoothing spline with a knot at every distinct x (R
  uses all knots below 50 points and a reduced set above).
* ``estimateExpPrior(x, uy, dataType, priorType, out, ru_theta, eps)``
  (FitOCT.R:103-107, server.R:396-404, ui.R:166-189) -> ``theta0, Sigma0``:
  'mono' ⚑: ``theta0 = out['best.theta']``, ``Sigma0 = D cor D`` with
  ``D = diag(ru_theta * theta0)`` and ``cor = out['cor.theta']``;
  'abc' ⚑: rejection ABC around the mono-exponential MAP: parameters drawn
  log-uniformly over a factor 2 around ``best.theta``, the curves
  ``b1 + b2 exp(-c x / b3)`` compared with the MAP curve in units of ``uy``,
  the ``eps`` fraction closest kept; ``theta0`` / ``Sigma0`` are their mean and
  covariance.
* ``read_courbe(path)``: a ``Courbe.csv`` (FitOCT.R:84: first column depth,
  second intensity, one header line).

Everything here is host numpy/scipy work (milliseconds per file); the GPU work
of a batch is the sampler launch (:mod:`fitoct_amd.pipeline`).
"""
from __future__ import annotations

import csv
import math

import numpy as np


def selX(x, y, depthSel=None, subSample=1):
    """Depth window and sub-sampling (FitOCTLib::selX).  Returns ``dict(x, y, sel)``
    with ``sel`` the kept indices of the input."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    if x.shape != y.shape or x.ndim != 1:
        raise ValueError("x and y must be 1-D arrays of equal length")
    idx = np.arange(x.size)
    if depthSel is not None:
        lo, hi = float(depthSel[0]), float(depthSel[1])
        idx = idx[(x >= lo) & (x <= hi)]
    step = int(subSample) if subSample else 1
    if step < 1:
        raise ValueError("subSample must be >= 1")
    idx = idx[::step]
    return {"x": x[idx], "y": y[idx], "sel": idx}


class SmoothingSpline:
    """Cubic smoothing spline (natural boundary) in Reinsch form, parametrised by
    its equivalent degrees of freedom ``df = trace(S(lambda))`` as R's
    ``smooth.spline(x, y, df=)`` is.  The penalty matrix K = Q R^-1 Q^T is
    diagonalised once, so ``S(lambda) = U diag(1 / (1 + lambda d)) U^T`` and the
    df -> lambda search is a scalar bisection."""

    def __init__(self, x):
        x = np.asarray(x, np.float64)
        order = np.argsort(x, kind="stable")
        xs = x[order]
        if xs.size < 4 or np.any(np.diff(xs) <= 0):
            raise ValueError("need >= 4 distinct abscissae")
        n = xs.size
        h = np.diff(xs)
        Q = np.zeros((n, n - 2))
        R = np.zeros((n - 2, n - 2))
        for j in range(n - 2):
            Q[j, j] = 1.0 / h[j]
            Q[j + 1, j] = -1.0 / h[j] - 1.0 / h[j + 1]
            Q[j + 2, j] = 1.0 / h[j + 1]
            R[j, j] = (h[j] + h[j + 1]) / 3.0
            if j + 1 < n - 2:
                R[j, j + 1] = R[j + 1, j] = h[j + 1] / 6.0
        K = Q @ np.linalg.solve(R, Q.T)
        d, U = np.linalg.eigh(0.5 * (K + K.T))
        self.d = np.clip(d, 0.0, None)
        self.U = U
        self.order = order
        self.n = n

    def df(self, lam):
        return float(np.sum(1.0 / (1.0 + lam * self.d)))

    def lam_for_df(self, df):
        if not (2.0 < df < self.n):
            raise ValueError(f"df must be in (2, {self.n})")
        lo, hi = -30.0, 30.0            # log10(lambda) bracket relative to the spectrum
        scale = 1.0 / max(float(np.median(self.d[self.d > 0])), 1e-300)
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if self.df(scale * 10.0 ** mid) > df:
                lo = mid
            else:
                hi = mid
        return scale * 10.0 ** (0.5 * (lo + hi))

    def fit(self, y, df):
        lam = self.lam_for_df(df)
        y = np.asarray(y, np.float64)[self.order]
        ys = self.U @ ((self.U.T @ y) / (1.0 + lam * self.d))
        out = np.empty_like(ys)
        out[self.order] = ys
        return out, lam


def smooth_spline(x, y, df=15):
    """``smooth.spline(x, y, df)$y`` restated (fitted values at the data x)."""
    ys, _ = SmoothingSpline(x).fit(y, df)
    return ys


def _noise_nll(a2, x, r2):
    # -log L of r ~ N(0, (a1 exp(-x/a2))^2) with a1 profiled out:
    # a1^2 = mean(r^2 exp(2x/a2)),  -log L = n log a1 - sum x / a2 + n/2 (+const)
    z = 2.0 * x / a2
    zmax = float(z.max())
    s = float(np.mean(r2 * np.exp(z - zmax)))
    log_a1 = 0.5 * (math.log(max(s, 1e-300)) + zmax)
    return x.size * log_a1 - float(np.sum(x)) / a2, math.exp(log_a1)


def estimateNoise(x, y, df=15):
    """FitOCTLib::estimateNoise restated: smoothing spline + ML fit of
    ``uy = a_1 exp(-x / a_2)`` to the residuals.  Returns
    ``dict(uy, ySmooth, theta=(a_1, a_2), resid, lam)``."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    if not np.isfinite(np.subtract(*np.percentile(x, [75, 25]))):
        raise ValueError("IQR(x) is not finite (server.R:306-307 guard)")
    ys, lam = SmoothingSpline(x).fit(y, df)
    r = y - ys
    r2 = r * r
    span = float(x.max() - x.min()) or 1.0
    # a_2 on a log grid, then golden-section refinement of the profiled likelihood
    grid = span * np.logspace(-2, 3, 101)
    vals = [_noise_nll(a, x, r2)[0] for a in grid]
    k = int(np.argmin(vals))
    lo, hi = math.log(grid[max(k - 1, 0)]), math.log(grid[min(k + 1, grid.size - 1)])
    g = (math.sqrt(5.0) - 1.0) / 2.0
    c, d = hi - g * (hi - lo), lo + g * (hi - lo)
    fc, fd = _noise_nll(math.exp(c), x, r2)[0], _noise_nll(math.exp(d), x, r2)[0]
    for _ in range(80):
        if fc < fd:
            hi, d, fd = d, c, fc
            c = hi - g * (hi - lo)
            fc = _noise_nll(math.exp(c), x, r2)[0]
        else:
            lo, c, fc = c, d, fd
            d = lo + g * (hi - lo)
            fd = _noise_nll(math.exp(d), x, r2)[0]
    a2 = math.exp(0.5 * (lo + hi))
    _, a1 = _noise_nll(a2, x, r2)
    uy = a1 * np.exp(-x / a2)
    return {"uy": uy, "ySmooth": ys, "theta": np.array([a1, a2]), "resid": r, "lam": lam}


def estimateExpPrior(x, uy, dataType=2, priorType="abc", out=None, ru_theta=0.05, eps=1e-3,
                     n_sim=200_000, seed=1234):
    """FitOCTLib::estimateExpPrior restated (see the module docstring, ⚑).
    ``out`` is a :func:`fitoct_amd.fitMonoExp` result.  Returns
    ``dict(theta0, Sigma0, priorType)``."""
    if out is None:
        raise ValueError("out (a fitMonoExp result) is required")
    th = np.asarray(out["best.theta"], np.float64)
    if priorType == "mono":
        cor = np.asarray(out.get("cor.theta", np.eye(3)), np.float64)
        D = np.diag(ru_theta * th)
        return {"theta0": th.copy(), "Sigma0": D @ cor @ D, "priorType": priorType}
    if priorType != "abc":
        raise ValueError("priorType must be 'abc' or 'mono' (ui.R:166-173)")
    x = np.asarray(x, np.float64)
    uy = np.asarray(uy, np.float64)
    c = float(dataType)
    m_ref = th[0] + th[1] * np.exp(-c * x / th[2])
    rng = np.random.Generator(np.random.PCG64(seed))
    keep_n = max(int(round(eps * n_sim)), 10)
    best = np.empty((0, 3))
    best_d = np.empty(0)
    for _ in range(max(1, n_sim // 20_000)):   # chunks keep the (chunk, N) curves small
        u = rng.uniform(-math.log(2.0), math.log(2.0), size=(20_000, 3))
        t = th * np.exp(u)
        m = t[:, :1] + t[:, 1:2] * np.exp(-c * x[None, :] / t[:, 2:3])
        dist = np.mean(((m - m_ref) / uy) ** 2, axis=1)
        best = np.concatenate([best, t])
        best_d = np.concatenate([best_d, dist])
        k = np.argsort(best_d)[:keep_n]
        best, best_d = best[k], best_d[k]
    theta0 = best.mean(axis=0)
    Sigma0 = np.cov(best.T)
    return {"theta0": theta0, "Sigma0": Sigma0, "priorType": priorType,
            "accepted": best.shape[0], "tolerance": float(best_d.max())}


def read_courbe(path):
    """A ``Courbe.csv`` (FitOCT.R:84): header line, then ``depth, intensity`` rows."""
    xs, ys = [], []
    with open(path, newline="") as f:
        rows = csv.reader(f)
        header = next(rows, None)
        if header is None:
            raise ValueError(f"{path}: empty file")
        for row in rows:
            if len(row) < 2 or not row[0].strip():
                continue
            xs.append(float(row[0]))
            ys.append(float(row[1]))
    if len(xs) < 4:
        raise ValueError(f"{path}: fewer than 4 data rows")
    return np.asarray(xs), np.asarray(ys)


def write_courbe(path, x, y):
    """Write a decay in the Courbe.csv layout (synthData.R:25-27 writes x, y)."""
    with open(path, "w", newline="") as f:
        f.write('"x","y"\n')                  # R write.csv header
        w = csv.writer(f)
        for a, b in zip(np.asarray(x), np.asarray(y)):
            w.writerow([repr(float(a)), repr(float(b))])
