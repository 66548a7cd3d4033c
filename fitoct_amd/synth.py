"""Seeded, N-parametrised restatement of the reference's synthetic-data generator.

``synthData.R:1-74`` writes five ``DataSynth/*/Courbe.csv`` decays on
``x = 20:500`` (N = 481) with ``a=1000, b=2000, l0=150, s=0.5`` (:3-7):

* ``monoExp``  : ``y0 = a + b*exp(-x/l0)``                          (:10)
* ``sincExp``  : ``m = 10*sin(x/50)/x``                              (:21)
* ``sincExp1`` : ``m = 10*sin(x/25)/x``                              (:35)
* ``sincExp2`` : ``m = 10*sin(x/75)/x``                              (:49)
* ``sincExp3`` : ``m = 1*sin((x-250)/20)/(x-250+0.1)``              (:63)

with ``y1 = a + b*exp(-x/(l0*(1+m)))`` (:22) and noise
``rnorm(sd = s*sqrt(y0-a+1))`` (:11,23).  The R script sets no seed; here the
noise comes from numpy ``PCG64(seed)`` so fixtures are reproducible, and the
depth grid is ``linspace(20, 500, N)`` so N can be chosen.
The returned ``uy`` is the true noise sd (bypassing ``estimateNoise``).
"""
from __future__ import annotations

import numpy as np

A, B, L0, S = 1000.0, 2000.0, 150.0, 0.5

MODULATIONS = ("sincExp", "sincExp1", "sincExp2", "sincExp3")


def modulation(x: np.ndarray, kind: str) -> np.ndarray:
    if kind == "monoExp":
        return np.zeros_like(x)
    if kind == "sincExp":
        return 10.0 * np.sin(x / 50.0) / x
    if kind == "sincExp1":
        return 10.0 * np.sin(x / 25.0) / x
    if kind == "sincExp2":
        return 10.0 * np.sin(x / 75.0) / x
    if kind == "sincExp3":
        return 1.0 * np.sin((x - 250.0) / 20.0) / (x - 250.0 + 0.1)
    raise ValueError(kind)


def synth_decay(N: int = 481, kind: str = "sincExp", seed: int = 1234,
                x_range=(20.0, 500.0)):
    """Return dict(x, y, uy, m, y_true) for one synthetic OCT decay."""
    x = np.linspace(x_range[0], x_range[1], N)
    y0 = A + B * np.exp(-x / L0)
    m = modulation(x, kind)
    y1 = A + B * np.exp(-x / (L0 * (1.0 + m)))
    uy = S * np.sqrt(y0 - A + 1.0)
    rng = np.random.Generator(np.random.PCG64(seed))
    y = y1 + rng.standard_normal(N) * uy
    return {"x": x, "y": y, "uy": uy, "m": m, "y_true": y1}


def default_prior(theta0=(1000.0, 2000.0, 300.0), ru_theta=0.05):
    """theta0 / Sigma0 used by the benchmarks: ``Sigma0 = diag((ru_theta*theta0)^2)``
    (``ru_theta`` default 0.05, FitOCT.R:46; dataType=2 gives theta3 = 2*l0 = 300)."""
    t0 = np.asarray(theta0, np.float64)
    return t0, np.diag((ru_theta * t0) ** 2)
