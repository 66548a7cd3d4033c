"""Host-side mirror of FitOCTLib's ExpGP interface over the libfitoct C ABI.

``fitExpGP`` keeps the R signature used by the reference's callers
(FitOCT.R:110-124, priPost.R:2-16, ShinyInterface/server.R:408-426) -- same
argument names, meanings and defaults -- and returns the same list shape
``list(fit, method, xGP, prior_PD)`` (plotExpGP.R:29-32) as a dict whose ``fit``
is a :class:`fitoct_amd.stanfit.StanFit` (print / extract / as_matrix / summary
with Rhat and n_eff, as used at plotExpGP.R:7-50 and server.R:88-237).
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import sys
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import GRID, PREC, PRIOR, FitOCTError, check, dptr, lib


@dataclass
class ExpGPProblem:
    """Inputs of one ExpGP fit (fields of ``fitoct_problem``)."""

    x: np.ndarray
    y: np.ndarray
    uy: np.ndarray
    dataType: int = 2
    Nn: int = 10
    gridType: str = "internal"
    rho: float = 0.0                      # <= 0 -> 1/Nn
    theta0: np.ndarray = field(default_factory=lambda: np.array([1000.0, 2000.0, 300.0]))
    Sigma0: np.ndarray = None
    prior_type: str = "normal"
    lambda_rate: float = 0.1
    lambda_scale: float = 10.0
    nu: float = 1.0
    prior_PD: int = 0
    kernel_conv: int = 0
    lambda_conv: int = 0
    sigma_scale: float = 10.0
    nugget: float = 1e-9
    B: np.ndarray = None
    # monoexp only: 1 = theta_k ~ exponential(1/lambda_scale), Tests/testGamma.R's model
    # (the sampler's known answer, include/fitoct.h theta_prior)
    theta_prior: int = 0

    def __post_init__(self):
        self.x = np.ascontiguousarray(self.x, dtype=np.float64)
        self.y = np.ascontiguousarray(self.y, dtype=np.float64)
        self.uy = np.ascontiguousarray(self.uy, dtype=np.float64)
        if not (self.x.shape == self.y.shape == self.uy.shape) or self.x.ndim != 1:
            raise ValueError("x, y, uy must be 1-D arrays of equal length")
        self.theta0 = np.ascontiguousarray(self.theta0, dtype=np.float64).reshape(3)
        if self.Sigma0 is None:
            self.Sigma0 = np.diag((0.05 * self.theta0) ** 2)
        self.Sigma0 = np.ascontiguousarray(self.Sigma0, dtype=np.float64).reshape(3, 3)
        if self.B is not None:
            self.B = np.ascontiguousarray(self.B, dtype=np.float64).reshape(self.x.size, self.Nn)
        if self.gridType not in GRID:
            raise ValueError(f"gridType must be one of {list(GRID)}")
        if self.prior_type not in PRIOR:
            raise ValueError(f"prior_type must be one of {list(PRIOR)}")

    @property
    def N(self) -> int:
        return self.x.size

    @property
    def family(self) -> int:
        return PRIOR[self.prior_type]

    @property
    def D(self) -> int:
        return lib().fitoct_dim(self.family, self.Nn)

    def to_c(self) -> _lib.Problem:
        p = _lib.Problem()
        p.N = self.N
        p.x, p.y, p.uy = dptr(self.x), dptr(self.y), dptr(self.uy)
        p.data_type = int(self.dataType)
        p.Nn = int(self.Nn)
        p.grid_type = GRID[self.gridType]
        p.rho = float(self.rho if self.rho else 0.0)
        p.B = dptr(self.B) if self.B is not None else None
        p.theta0[:] = list(self.theta0)
        p.Sigma0[:] = list(self.Sigma0.ravel())
        p.prior_type = self.family
        p.lambda_rate = float(self.lambda_rate)
        p.lambda_scale = float(self.lambda_scale)
        p.nu = float(self.nu)
        p.prior_PD = int(self.prior_PD)
        p.kernel_conv = int(self.kernel_conv)
        p.lambda_conv = int(self.lambda_conv)
        p.sigma_scale = float(self.sigma_scale)
        p.nugget = float(self.nugget)
        p.theta_prior = int(self.theta_prior)
        return p

    def basis(self):
        """(B[N, Nn], xGP[Nn]) as built by the library (fp64 Cholesky, host)."""
        B = np.zeros((self.N, self.Nn))
        xg = np.zeros(self.Nn)
        p = self.to_c()
        check(lib().fitoct_build_basis(C.byref(p), dptr(B), dptr(xg)))
        return B, xg

    def column_names(self):
        return _lib.column_names(self.family, self.Nn)


@dataclass
class SamplerConfig:
    """``rstan::sampling`` controls (testGamma.R:42-47) + sharding."""

    chains: int = 4
    warmup: int = 500
    samples: int = 1000
    seed: int = 1234
    adapt_delta: float = 0.8
    max_treedepth: int = 10
    adapt_engaged: bool = True
    stepsize: float = 1.0
    gamma: float = 0.05
    kappa: float = 0.75
    t0: float = 10.0
    init_buffer: int = 75
    term_buffer: int = 50
    window: int = 25
    init_radius: float = 2.0
    save_warmup: bool = True
    precision: str = "f64"
    device: int = 0
    chain_offset: int = 0
    # device list (fitoct_config.devices): the chains are split into contiguous blocks
    # of global chain ids, one per device, each run by its own host thread in the
    # library; draws equal a one-device run bit for bit.  Empty: ``device`` alone.
    devices: tuple = ()

    def to_c(self) -> _lib.Config:
        c = _lib.Config()
        c.chains = int(self.chains)
        c.chain_offset = int(self.chain_offset)
        c.warmup = int(self.warmup)
        c.samples = int(self.samples)
        c.seed = int(self.seed) & 0xFFFFFFFFFFFFFFFF
        c.adapt_delta = float(self.adapt_delta)
        c.max_treedepth = int(self.max_treedepth)
        c.adapt_engaged = 1 if self.adapt_engaged else 0
        c.stepsize = float(self.stepsize)
        c.gamma, c.kappa, c.t0 = float(self.gamma), float(self.kappa), float(self.t0)
        c.init_buffer, c.term_buffer, c.window = (int(self.init_buffer), int(self.term_buffer),
                                                  int(self.window))
        c.init_radius = float(self.init_radius)
        c.save_warmup = 1 if self.save_warmup else 0
        c.precision = PREC[self.precision]
        c.device = int(self.device)
        devs = tuple(int(d) for d in self.devices)
        if len(devs) > _lib.MAX_DEVICES:
            raise ValueError(f"at most {_lib.MAX_DEVICES} devices per call")
        c.n_devices = len(devs)
        for i, d in enumerate(devs):
            c.devices[i] = d
        return c


def logp_grad(prob: ExpGPProblem, q: np.ndarray, precision: str = "f64", device: int = 0):
    """Batched log density / gradient on the GPU: q[P, D] -> (lp[P], grad[P, D], sumr2[P])."""
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
    P, D = q.shape
    if D != prob.D:
        raise ValueError(f"q has {D} columns, model dimension is {prob.D}")
    lp = np.zeros(P)
    g = np.zeros((P, D))
    s2 = np.zeros(P)
    p = prob.to_c()
    check(lib().fitoct_logp_grad(C.byref(p), P, dptr(q), dptr(lp), dptr(g), dptr(s2),
                                 PREC[precision], device))
    return lp, g, s2


@dataclass
class SampleOutput:
    draws: np.ndarray          # [chains, iters_saved, n_cols]
    columns: list
    warmup_saved: int          # leading warmup iterations included in draws
    stepsize: np.ndarray
    inv_metric: np.ndarray
    last_q: np.ndarray
    total_leapfrogs: int
    kernel_ms: float
    wall_ms: float
    chain_offset: int = 0
    migrations: int = 0        # chains handed between tiles (work balance)
    cfg: object = None         # the SamplerConfig of the run (Stan-CSV header)
    two_ended_transitions: int = 0   # transitions grown at both ends at once (no effect on draws)
    paired_transitions: int = 0      # ... whose forward end grew in a partner tile (no effect)


class Plan:
    """A planned sampler run: inputs staged in HBM once, run many times."""

    def __init__(self, prob: ExpGPProblem, cfg: SamplerConfig):
        self.prob, self.cfg = prob, cfg
        self._p = prob.to_c()
        self._c = cfg.to_c()
        h = C.c_void_p()
        check(lib().fitoct_plan_create(C.byref(self._p), C.byref(self._c), C.byref(h)))
        self._h = h
        info = _lib.PlanInfo()
        check(lib().fitoct_plan_get_info(self._h, C.byref(info)))
        self.info = {f: getattr(info, f) for f, _ in _lib.PlanInfo._fields_}

    def run(self, d_draws: int = 0, stream: int = 0, progress=None, poll_s: float = 0.2):
        """Run on ``stream`` (hipStream_t as int); draws to the device buffer
        ``d_draws`` (int pointer, >= info['draws_bytes']) or a plan-internal one.

        ``progress(done, total)``, if given, is called from this thread every
        ``poll_s`` seconds while the kernel runs (done / total = transitions over all
        chains; this replaces rstan's stan.log progress, server.R:457-484).  A
        KeyboardInterrupt during the run cancels the chains at their next transition
        boundary, waits for the kernel to drain and re-raises: the R shim does the
        same around R_CheckUserInterrupt."""
        if progress is None:
            check(lib().fitoct_plan_run(self._h, C.c_void_p(d_draws or None),
                                        C.c_void_p(stream or None)))
            return
        self.launch(d_draws, stream)
        try:
            while True:
                done, total, finished = self.poll()
                progress(done, total)
                if finished:
                    break
                time.sleep(poll_s)
        except KeyboardInterrupt:
            self.cancel()
            self.wait()
            raise
        self.wait()

    def set_init(self, q_init=None, stepsize=None, inv_metric=None):
        """Warm restart (``fitoct_plan_set_init``): per-chain start position q_init
        [chains, D] (unconstrained), initial step size [chains] and diagonal inverse
        metric [chains, D] for the next runs; None keeps the default (jittered start
        around theta0, ``cfg.stepsize``, unit metric).  A previous run's ``last_q``,
        ``stepsize`` and ``inv_metric`` resume it (``adapt_engaged=False`` keeps them)."""
        C_, D = self.info["chains"], self.info["dim"]
        self._init = []   # kept alive only for the call (the library copies them)

        def arr(a, shape):
            if a is None:
                return None
            a = np.ascontiguousarray(np.broadcast_to(np.asarray(a, dtype=np.float64), shape))
            self._init.append(a)
            return dptr(a)
        check(lib().fitoct_plan_set_init(self._h, arr(q_init, (C_, D)), arr(stepsize, (C_,)),
                                         arr(inv_metric, (C_, D))))
        self._init = []

    def launch(self, d_draws: int = 0, stream: int = 0):
        """Enqueue the run and return at once (see :meth:`poll`, :meth:`wait`)."""
        check(lib().fitoct_plan_launch(self._h, C.c_void_p(d_draws or None),
                                       C.c_void_p(stream or None)))

    def poll(self):
        """(transitions done over all chains, chains * (warmup + samples), finished)."""
        d, t, f = C.c_int64(), C.c_int64(), C.c_int32()
        check(lib().fitoct_plan_poll(self._h, C.byref(d), C.byref(t), C.byref(f)))
        return int(d.value), int(t.value), bool(f.value)

    def cancel(self):
        """Ask every chain to stop at its next (8th) transition boundary; the run then
        reports FITOCT_E_CANCELLED from :meth:`download`."""
        check(lib().fitoct_plan_cancel(self._h))

    def wait(self):
        """Block until the launched run has drained."""
        check(lib().fitoct_plan_wait(self._h))

    def download(self, with_draws: bool = True) -> SampleOutput:
        """Copy results to the host.  ``with_draws=False`` leaves the draws in HBM
        (``SampleOutput.draws`` is None), e.g. when they are gathered over RCCL."""
        i = self.info
        C_, D = i["chains"], i["dim"]
        draws = np.empty((C_, i["iters_saved"], i["n_cols"])) if with_draws else None
        eps = np.empty(C_)
        minv = np.empty((C_, D))
        lq = np.empty((C_, D))
        st = np.zeros(C_, dtype=np.int32)
        r = _lib.Result()
        r.draws = dptr(draws)
        r.draws_capacity = draws.size if with_draws else 0
        r.stepsize, r.inv_metric, r.last_q = dptr(eps), dptr(minv), dptr(lq)
        r.chain_status = st.ctypes.data_as(C.POINTER(C.c_int32))
        check(lib().fitoct_plan_download(self._h, C.byref(r)))
        return SampleOutput(draws, self.prob.column_names(),
                            self.cfg.warmup if self.cfg.save_warmup else 0, eps, minv, lq,
                            int(r.total_leapfrogs), float(r.kernel_ms), 0.0,
                            self.cfg.chain_offset, int(r.migrations), self.cfg,
                            int(r.two_ended_transitions), int(r.paired_transitions))

    def close(self):
        if getattr(self, "_h", None):
            lib().fitoct_plan_destroy(self._h)
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


class Batch:
    """Many problems (FitOCT.R's per-file fits, FitOCT.R:70-124) sampled by one
    launch (``fitoct_batch_*``).  Problem ``p``'s chains are global chains
    ``cfg.chain_offset + p*cfg.chains + c``, so its draws equal a :class:`Plan`
    of that problem with ``chain_offset = cfg.chain_offset + p*cfg.chains``."""

    def __init__(self, probs, cfg: SamplerConfig):
        self.probs, self.cfg = list(probs), cfg
        if not self.probs:
            raise ValueError("a batch needs at least one problem")
        arr = (_lib.Problem * len(self.probs))()
        for i, p in enumerate(self.probs):
            arr[i] = p.to_c()
        self._arr = arr    # the problems' numpy buffers stay referenced by self.probs
        self._c = cfg.to_c()
        h = C.c_void_p()
        check(lib().fitoct_batch_create(arr, len(self.probs), C.byref(self._c), C.byref(h)))
        self._h = h
        info = _lib.PlanInfo()
        check(lib().fitoct_batch_get_info(self._h, C.byref(info)))
        self.info = {f: getattr(info, f) for f, _ in _lib.PlanInfo._fields_}

    def __len__(self):
        return len(self.probs)

    def run(self, d_draws: int = 0, stream: int = 0):
        """One launch for every problem; draws to ``d_draws`` (device pointer,
        >= info['draws_bytes'], layout [problem][chain][iter][col]) or internal."""
        check(lib().fitoct_batch_run(self._h, C.c_void_p(d_draws or None),
                                     C.c_void_p(stream or None)))

    def download(self, problem: int, with_draws: bool = True) -> SampleOutput:
        i, C_ = self.info, self.cfg.chains
        D = i["dim"]
        draws = np.empty((C_, i["iters_saved"], i["n_cols"])) if with_draws else None
        eps, minv, lq = np.empty(C_), np.empty((C_, D)), np.empty((C_, D))
        st = np.zeros(C_, dtype=np.int32)
        r = _lib.Result()
        r.draws = dptr(draws)
        r.draws_capacity = draws.size if with_draws else 0
        r.stepsize, r.inv_metric, r.last_q = dptr(eps), dptr(minv), dptr(lq)
        r.chain_status = st.ctypes.data_as(C.POINTER(C.c_int32))
        check(lib().fitoct_batch_download(self._h, int(problem), C.byref(r)))
        return SampleOutput(draws, self.probs[problem].column_names(),
                            self.cfg.warmup if self.cfg.save_warmup else 0, eps, minv, lq,
                            int(r.total_leapfrogs), float(r.kernel_ms), 0.0,
                            self.cfg.chain_offset + problem * C_, 0,
                            dataclasses.replace(self.cfg,
                                                chain_offset=self.cfg.chain_offset + problem * C_),
                            int(r.two_ended_transitions), int(r.paired_transitions))

    def close(self):
        if getattr(self, "_h", None):
            lib().fitoct_batch_destroy(self._h)
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


def sample_batch(probs, cfg: SamplerConfig):
    """One launch over every problem; returns one SampleOutput per problem."""
    t0 = time.perf_counter()
    with Batch(probs, cfg) as b:
        b.run()
        outs = [b.download(p) for p in range(len(b))]
    wall = (time.perf_counter() - t0) * 1e3
    for o in outs:
        o.wall_ms = wall
    return outs


def sample(prob: ExpGPProblem, cfg: SamplerConfig, progress=None,
           resume: SampleOutput | None = None) -> SampleOutput:
    """One-shot sampler run (plan + run + download); ``progress`` as in :meth:`Plan.run`.
    ``resume``: a previous run of the same chains whose last position, step size and
    inverse metric start this one (:meth:`Plan.set_init`)."""
    t0 = time.perf_counter()
    with Plan(prob, cfg) as pl:
        if resume is not None:
            pl.set_init(resume.last_q, resume.stepsize, resume.inv_metric)
        pl.run(progress=progress)
        out = pl.download()
    out.wall_ms = (time.perf_counter() - t0) * 1e3
    return out


def progress_printer(warmup, samples, stream=None):
    """rstan-format progress lines ("Chain k: Iteration: i / n [ p%]  (Warmup|Sampling)",
    ``fitoct_progress_line``: the overall fraction in the 4-serial-chains convention the
    Shiny server decodes, server.R:457-472) printed whenever the overall percentage
    changes -- the lines the R shim prints to R's stdout."""
    last = [-1]
    buf = C.create_string_buffer(160)

    def cb(done, total):
        if total <= 0:
            return
        pct = lib().fitoct_progress_line(int(done), int(total), int(warmup), int(samples), buf, 160)
        if pct < 0 or pct == last[0]:
            return
        last[0] = pct
        print(buf.value.decode(), file=stream or sys.stdout, flush=True)
    return cb


# --------------------------------------------------------------------------
# FitOCTLib-compatible entry point
# --------------------------------------------------------------------------
def fitExpGP(x, y, uy, dataType=2, Nn=10, gridType="internal", method="sample",
             theta0=None, Sigma0=None, lambda_rate=0.1, rho_scale=0.0, nb_warmup=500,
             nb_iter=1000, prior_PD=0, open_progress=False, *, nb_chains=4,
             prior_type="normal", lambda_scale=10.0, nu=1.0, adapt_delta=0.8,
             max_treedepth=10, seed=None, precision="f64", device=0, n_gpus=None,
             devices=None, refresh=1, **model_switches):
    """Drop-in for ``FitOCTLib::fitExpGP`` (FitOCT.R:110-124).

    ``nb_iter`` counts warmup + sampling iterations, as the callers pass
    ``nb_iter = nb_warmup + nb_sample`` (FitOCT.R:121).  ``rho_scale`` <= 0 means
    ``1/Nn`` (FitOCT.R:119).  Only ``method='sample'`` runs on the GPU; 'optim'
    and 'vb' run rstan::optimizing / rstan::vb natively over the same device
    density (:mod:`fitoct_amd.optim_vb`): ``fit`` is then an ``OptimFit``
    (``fit$par``, ``fit$hessian``) or a StanFit of ADVI draws.
    Progress lines are printed to stdout in rstan's format whatever
    ``open_progress`` is, as the R shim does (the Shiny server parses them from its
    stdout sink, server.R:391-393,457-484); ``refresh=0`` silences them.
    ``n_gpus`` (replaces ``options(mc.cores = detectCores())``,
    FitOCT.R:13): the chains are split over devices ``device .. device + n_gpus - 1``
    (the library runs one host thread per device; the draws do not depend on it);
    ``devices`` gives the ordinals explicitly instead (repeats allowed).
    Returns ``dict(fit, method, xGP, prior_PD, lasso)``.
    """
    from .stanfit import StanFit

    if method not in ("sample", "optim", "vb"):
        raise ValueError(f"method={method!r}: 'sample', 'optim' or 'vb' (FitOCT.R:42)")
    if theta0 is None:
        raise ValueError("theta0 is required (FitOCTLib::estimateExpPrior output)")
    nb_sample = int(nb_iter) - int(nb_warmup)
    if nb_sample < 1:
        raise ValueError("nb_iter must exceed nb_warmup")
    prob = ExpGPProblem(x, y, uy, dataType=dataType, Nn=Nn, gridType=gridType,
                        rho=rho_scale if rho_scale and rho_scale > 0 else 0.0, theta0=theta0,
                        Sigma0=Sigma0, prior_type=prior_type, lambda_rate=lambda_rate,
                        lambda_scale=lambda_scale, nu=nu, prior_PD=prior_PD, **model_switches)
    if seed is None:
        seed = int(np.random.SeedSequence().entropy & 0xFFFFFFFF)
    _, xGP = prob.basis()
    if method != "sample":
        from .genquant import expgp_curves
        from .optim_vb import optimizing, vb
        fit = (optimizing(prob, precision=precision, device=device) if method == "optim"
               else vb(prob, seed=seed, precision=precision, device=device))
        if method == "optim":   # fit$par$m / $resid / $dL (server.R:351,636)
            g = expgp_curves(prob, fit.par["theta"], fit.par["yGP"])
            for k in ("m", "resid", "dL"):
                fit.par[k] = g[k][0]
        return {"fit": fit, "method": method, "xGP": xGP, "prior_PD": prior_PD,
                "lasso": prior_type == "lasso"}
    if n_gpus is not None and not 1 <= int(n_gpus) <= 16:
        raise ValueError("fitExpGP: n_gpus must be in 1..16")   # as the R shim (fitoct_devices)
    if devices is None:
        devices = tuple(range(int(device), int(device) + int(n_gpus))) if n_gpus and n_gpus > 1 else ()
    cfg = SamplerConfig(chains=nb_chains, warmup=nb_warmup, samples=nb_sample, seed=seed,
                        adapt_delta=adapt_delta, max_treedepth=max_treedepth,
                        precision=precision, device=device, devices=devices)
    out = sample(prob, cfg, progress=progress_printer(nb_warmup, nb_sample) if refresh else None)
    fit = StanFit.from_output(out, prob)
    return {"fit": fit, "method": method, "xGP": xGP, "prior_PD": prior_PD,
            "lasso": prior_type == "lasso"}
