"""ORACLE (test infrastructure only) -- numpy restatement of the FitOCT ExpGP
log-posterior and its gradient.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  The product path (``fitoct_amd``) never does.

Parity status: **parity unpinned** against rstan/FitOCTLib.  The hot-path
arithmetic lives in the external R package FitOCTLib (``README.md:14``,
``ShinyInterface/server.R:12-15``) and in rstan/Stan, none of which exist in
this container (no R, no Stan toolchain).  This file restates
the model contract of SURVEY.md Appendix A from the reference's own in-tree
anchors:

* forward model ``y = b1 + b2*exp(-c*depth/b3)``            ShinyInterface/ui.R:88
* decay-length modulation ``l0*(1+m)``                        synthData.R:22
* normalised depth and GP grid (internal / extremal)          ShinyInterface/server.R:623-635
* squared-exponential GP kernel family (RMgauss)              ShinyInterface/server.R:647-650, Tests/simulGP.R:26
* horseshoe hyper-prior                                        Tests/horseShoePrior.stan:16-43
* lasso / elastic-net hyper-prior                              Tests/lassoPrior.stan:9-12
* exponential hyper-prior ``exponential(1/lambda_scale)``      Tests/testGamma.R:19-28
* ``theta ~ multi_normal(theta0, Sigma0)``                     FitOCT.R:116-117
* ``prior_PD`` switches the likelihood off                      priPost.R:14
* parameter names theta, yGP, lambda, sigma, br, lp__          plotExpGP.R:9,41-43

The flagged (⚑) assumptions of Appendix A are explicit keyword switches here
(``kernel_conv``, ``lambda_conv``, ``sigma_scale``, ``nugget``) and carry the
same meaning in the C oracle and in the HIP library.

What pins it instead: analytic prior-only known answers (tests/kat_cases.py, run by
tests/test_oracle_nuts.py and tests/test_gpu_sampler.py),
finite-difference gradient checks, and the golden vectors this file generates
(tests/golden/make_golden.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# prior families (same integer codes as include/fitoct.h FITOCT_PRIOR_*)
NORMAL, LASSO, HORSESHOE, MONOEXP = 0, 1, 2, 3
FAMILIES = {"normal": NORMAL, "lasso": LASSO, "horseshoe": HORSESHOE, "monoexp": MONOEXP}


# --------------------------------------------------------------------------
# GP basis  (server.R:623-650)
# --------------------------------------------------------------------------
def gp_grid(Nn: int, grid_type: str) -> np.ndarray:
    """Control-point abscissae on [0,1].  server.R:627-631:
    ``dx = 1/(n+1); internal: seq(dx/2, 1-dx/2, length.out=n); else seq(0,1,length.out=n)``."""
    if grid_type == "internal":
        dx = 1.0 / (Nn + 1)
        return np.linspace(dx / 2, 1 - dx / 2, Nn)
    if grid_type == "extremal":
        return np.linspace(0.0, 1.0, Nn)
    raise ValueError(f"gridType must be 'internal' or 'extremal', got {grid_type!r}")


def normalize_depth(x: np.ndarray) -> np.ndarray:
    """``xp <- (x-min(x)) / (max(x)-min(x))`` -- server.R:635."""
    x = np.asarray(x, dtype=np.float64)
    return (x - x.min()) / (x.max() - x.min())


def se_kernel(d: np.ndarray, rho: float, kernel_conv: int = 0) -> np.ndarray:
    """Squared-exponential kernel.  kernel_conv 0 = Stan ``cov_exp_quad``
    ``exp(-d^2/(2 rho^2))`` (default); 1 = RandomFields ``RMgauss(scale=rho)``
    ``exp(-(d/rho)^2)`` (server.R:648-650).  ⚑ SURVEY Appendix A."""
    if kernel_conv == 0:
        return np.exp(-(d * d) / (2.0 * rho * rho))
    return np.exp(-(d / rho) ** 2)


def gp_basis(x, Nn, grid_type="extremal", rho=None, kernel_conv=0, nugget=1e-9):
    """``B = K(x~, xGP) K(xGP, xGP)^-1`` (fp64 Cholesky).  Returns (B[N,Nn], xGP)."""
    if rho is None or rho == 0:
        rho = 1.0 / Nn  # FitOCT.R:119 rho_scale==0 -> 1/Nn
    xt = normalize_depth(x)
    xg = gp_grid(Nn, grid_type)
    Kgg = se_kernel(xg[:, None] - xg[None, :], rho, kernel_conv) + nugget * np.eye(Nn)
    Kxg = se_kernel(xt[:, None] - xg[None, :], rho, kernel_conv)
    L = np.linalg.cholesky(Kgg)
    # B^T = Kgg^-1 Kxg^T  (Kgg symmetric)
    Z = np.linalg.solve(L, Kxg.T)
    Bt = np.linalg.solve(L.T, Z)
    return Bt.T.copy(), xg


# --------------------------------------------------------------------------
# problem container
# --------------------------------------------------------------------------
@dataclass
class Problem:
    x: np.ndarray
    y: np.ndarray
    uy: np.ndarray
    data_type: int = 2
    Nn: int = 15
    grid_type: str = "extremal"
    rho: float = 0.0
    theta0: np.ndarray = field(default_factory=lambda: np.array([1000.0, 2000.0, 300.0]))
    Sigma0: np.ndarray = None
    family: int = NORMAL
    lambda_rate: float = 0.1      # normal family: lambda ~ Exponential (see lambda_conv)
    lambda_scale: float = 10.0    # lasso family: lambda_s (lassoPrior.stan:4)
    nu: float = 1.0               # horseshoe family (horseShoePrior.stan:13)
    prior_PD: int = 0
    kernel_conv: int = 0
    lambda_conv: int = 0          # 0: rate = 1/lambda_rate (mean lambda_rate); 1: rate = lambda_rate
    sigma_scale: float = 10.0     # ⚑ sigma ~ half-normal(0, sigma_scale)
    nugget: float = 1e-9
    B: np.ndarray = None
    xGP: np.ndarray = None
    theta_prior: int = 0          # monoexp: 1 = theta_k ~ exponential(1/lambda_scale) (testGamma.R)

    def __post_init__(self):
        self.x = np.asarray(self.x, np.float64)
        self.y = np.asarray(self.y, np.float64)
        self.uy = np.asarray(self.uy, np.float64)
        self.theta0 = np.asarray(self.theta0, np.float64)
        if self.Sigma0 is None:
            self.Sigma0 = np.diag((0.05 * self.theta0) ** 2)
        self.Sigma0 = np.asarray(self.Sigma0, np.float64).reshape(3, 3)
        if self.rho is None or self.rho == 0:
            self.rho = 1.0 / self.Nn
        if self.family == MONOEXP:          # no GP term (FitOCTLib::fitMonoExp)
            self.B = np.zeros((self.x.size, 0))
            self.xGP = np.zeros(0)
        elif self.B is None:
            self.B, self.xGP = gp_basis(self.x, self.Nn, self.grid_type, self.rho,
                                        self.kernel_conv, self.nugget)

    @property
    def N(self):
        return self.x.size

    @property
    def D(self):
        return dim(self.family, self.Nn)


def dim(family: int, Nn: int) -> int:
    """Unconstrained dimension (SURVEY §8 shape symbols)."""
    return {NORMAL: Nn + 5, LASSO: Nn + 4, HORSESHOE: 3 * Nn + 6, MONOEXP: 3}[family]


def param_names(family: int, Nn: int):
    th = ["theta[1]", "theta[2]", "theta[3]"]
    if family == MONOEXP:
        return th
    if family == NORMAL:
        return th + [f"yGP[{k+1}]" for k in range(Nn)] + ["lambda", "sigma"]
    if family == LASSO:
        return th + [f"yGP[{k+1}]" for k in range(Nn)] + ["sigma"]
    return (th + [f"z[{k+1}]" for k in range(Nn)] + ["r1_global", "r2_global"]
            + [f"r1_local[{k+1}]" for k in range(Nn)] + [f"r2_local[{k+1}]" for k in range(Nn)]
            + ["sigma"])


def constrain(q: np.ndarray, family: int, Nn: int) -> np.ndarray:
    """Unconstrained -> constrained (exp on every <lower=0> parameter)."""
    q = np.asarray(q, np.float64)
    c = q.copy()
    c[..., 0:3] = np.exp(q[..., 0:3])
    if family == MONOEXP:
        return c
    if family == NORMAL:
        c[..., 3 + Nn:] = np.exp(q[..., 3 + Nn:])
    elif family == LASSO:
        c[..., 3 + Nn] = np.exp(q[..., 3 + Nn])
    else:
        c[..., 3 + Nn:] = np.exp(q[..., 3 + Nn:])
    return c


def horseshoe_ygp(qc: np.ndarray, Nn: int):
    """``tau = r1_g*sqrt(r2_g); lambda = r1_l.*sqrt(r2_l); yGP = z.*lambda*tau``
    -- Tests/horseShoePrior.stan:30-32.  ``qc`` is the constrained vector."""
    z = qc[..., 3:3 + Nn]
    r1g = qc[..., 3 + Nn]
    r2g = qc[..., 4 + Nn]
    r1l = qc[..., 5 + Nn:5 + 2 * Nn]
    r2l = qc[..., 5 + 2 * Nn:5 + 3 * Nn]
    tau = r1g * np.sqrt(r2g)
    lam = r1l * np.sqrt(r2l)
    return z * lam * tau[..., None], tau, lam


# --------------------------------------------------------------------------
# log density and gradient  
# --------------------------------------------------------------------------
def logp_grad(q, prob: Problem):
    """Return (lp, grad[D], sumr2) at unconstrained ``q``.

    lp follows Stan's ``log_prob<propto=true, jacobian=true>``: constants
    dropped, log-Jacobians of the exp transforms included.  ``sumr2`` is
    ``sum(((y-m)/uy)^2)`` (sigma excluded), so ``br = sumr2/N`` (⚑ normaliser).
    """
    q = np.asarray(q, np.float64)
    Nn, fam = prob.Nn, prob.family
    D = dim(fam, Nn)
    assert q.shape == (D,)
    g = np.zeros(D)
    th = np.exp(q[0:3])
    if fam == MONOEXP:
        # FitOCTLib::fitMonoExp (⚑ SURVEY §8f row 2): no GP term, flat prior on
        # theta > 0, sigma fixed at 1 (uy is the noise sd)
        Nn = 0
        ygp = np.zeros(0)
        sigma = 1.0
    elif fam == HORSESHOE:
        sigma = math.exp(q[D - 1])
        qc = constrain(q, fam, Nn)
        ygp, tau, lam = horseshoe_ygp(qc, Nn)
    elif fam == NORMAL:
        ygp = q[3:3 + Nn]
        lam_s = math.exp(q[3 + Nn])
        sigma = math.exp(q[4 + Nn])
    else:
        ygp = q[3:3 + Nn]
        sigma = math.exp(q[3 + Nn])

    lp = 0.0
    # ---- likelihood over N depth bins -------------------------------------
    c = float(prob.data_type)
    dL = prob.B @ ygp                                       # GP modulation
    u = 1.0 + dL
    sumr2 = math.nan
    gy = np.zeros(Nn)
    gth = np.zeros(3)
    gsig = 0.0
    if prob.prior_PD == 0 and np.any(u <= 0.0):
        lp = -math.inf                                      # non-physical decay length guard
        sumr2 = math.inf
    elif prob.prior_PD != 0:
        pass                                                # likelihood off (priPost.R:14)
    else:
        L = th[2] * u
        e = np.exp(-c * prob.x / L)
        m = th[0] + th[1] * e                               # ui.R:88, synthData.R:22
        d = (prob.y - m) / prob.uy
        sumr2 = float(d @ d)
        if True:
            r = d / sigma
            lp += -0.5 * float(r @ r) - prob.N * math.log(sigma)
            gm = r / (sigma * prob.uy)                      # dlp/dm_i
            w = gm * e * c * prob.x / L
            gth[0] = gm.sum()
            gth[1] = float(gm @ e)
            gth[2] = th[1] * w.sum() / th[2]
            gy = th[1] * th[2] * (prob.B.T @ (w / L))       # dlp/dyGP = B^T (dlp/ddL)
            gsig = (float(r @ r) - prob.N) / sigma

    if fam == MONOEXP:
        g[0:3] = gth * th + 1.0                             # flat prior + log-Jacobian
        lp += float(q[0:3].sum())
        if prob.theta_prior == 1:                           # Tests/testGamma.R:19-28
            rate = 1.0 / prob.lambda_scale
            lp += -rate * float(th.sum())
            g[0:3] -= rate * th
        return (lp if math.isfinite(lp) else -math.inf), g, sumr2
    # ---- theta ~ multi_normal(theta0, Sigma0)   FitOCT.R:116-117 -------------
    S = np.linalg.inv(prob.Sigma0)
    dth = th - prob.theta0
    lp += -0.5 * float(dth @ S @ dth)
    gth += -(S @ dth)
    g[0:3] = gth * th + 1.0                                 # log-Jacobian of exp
    lp += float(q[0:3].sum())

    # ---- sigma ~ half-normal(0, sigma_scale)  ⚑ -----------------------------
    ss = prob.sigma_scale
    lp += -0.5 * (sigma / ss) ** 2 + q[D - 1]
    g[D - 1] = sigma * (gsig - sigma / ss ** 2) + 1.0

    # ---- yGP hyper-prior ----------------------------------------------------
    if fam == NORMAL:
        # yGP ~ normal(0, lambda) ⚑ ; lambda ~ exponential(rate) ⚑ (testGamma.R:27)
        rate = 1.0 / prob.lambda_rate if prob.lambda_conv == 0 else prob.lambda_rate
        s2 = float(ygp @ ygp)
        lp += -Nn * math.log(lam_s) - s2 / (2 * lam_s ** 2)
        lp += -rate * lam_s + q[3 + Nn]
        g[3:3 + Nn] = gy - ygp / lam_s ** 2
        dlam = -Nn / lam_s + s2 / lam_s ** 3 - rate
        g[3 + Nn] = lam_s * dlam + 1.0
    elif fam == LASSO:
        # target += -lambda_s*sum|yGP| - lambda_s*dot_self(yGP)   lassoPrior.stan:10-12
        ls = prob.lambda_scale
        lp += -ls * float(np.abs(ygp).sum()) - ls * float(ygp @ ygp)
        g[3:3 + Nn] = gy - ls * np.sign(ygp) - 2 * ls * ygp
    else:
        # horseShoePrior.stan:37-42 with log-transformed positive parameters
        nu = prob.nu
        z = q[3:3 + Nn]
        r1g, r2g = qc[3 + Nn], qc[4 + Nn]
        r1l = qc[5 + Nn:5 + 2 * Nn]
        r2l = qc[5 + 2 * Nn:5 + 3 * Nn]
        lp += -0.5 * float(z @ z)
        lp += -0.5 * float(r1l @ r1l)
        lp += float(np.sum(-(0.5 * nu + 1) * np.log(r2l) - 0.5 * nu / r2l))
        lp += -0.5 * r1g * r1g
        lp += -1.5 * math.log(r2g) - 0.5 / r2g
        lp += float(q[3 + Nn:5 + 3 * Nn].sum())             # log-Jacobians
        Gy = gy * ygp                                       # G_k * yGP_k
        g[3:3 + Nn] = gy * lam * tau - z
        g[3 + Nn] = Gy.sum() - r1g * r1g + 1.0
        g[4 + Nn] = 0.5 * Gy.sum() - 1.5 + 0.5 / r2g + 1.0
        g[5 + Nn:5 + 2 * Nn] = Gy - r1l * r1l + 1.0
        g[5 + 2 * Nn:5 + 3 * Nn] = 0.5 * Gy - (0.5 * nu + 1) + 0.5 * nu / r2l + 1.0
    if not math.isfinite(lp):
        lp = -math.inf
    return lp, g, sumr2


def logp(q, prob):
    return logp_grad(q, prob)[0]


def fd_grad(q, prob, h=1e-6):
    """Central finite differences (test helper)."""
    q = np.asarray(q, np.float64)
    g = np.zeros_like(q)
    for i in range(q.size):
        qp, qm = q.copy(), q.copy()
        qp[i] += h
        qm[i] -= h
        g[i] = (logp(qp, prob) - logp(qm, prob)) / (2 * h)
    return g
