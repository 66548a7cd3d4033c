"""FitOCT.R's batch mode on the HIP engine (BASELINE.json configs[4]).

FitOCT.R:70-131 loops over data sets: ``read.csv(Courbe.csv)`` -> ``selX`` ->
``estimateNoise`` -> ``fitMonoExp`` -> ``printBr`` (skip the GP fit when the
mono-exponential Birge ratio raises no alert, FitOCT.R:100) ->
``estimateExpPrior`` -> ``fitExpGP`` (-> ``priPost.R``'s prior-predictive fit).
Here the host preparation runs per file (:mod:`fitoct_amd.prep`,
:func:`fitoct_amd.fitMonoExp` on the device evaluator) and every file's
``fitExpGP(method='sample')`` goes into ONE batched sampler launch
(``fitoct_batch_*``: one tile per file's chains), instead of one rstan run per
file.  Control parameters follow FitOCT.R:37-53 overridden by a
``ctrlParams.yaml`` (FitOCT.R:56-63).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from .api import Batch, ExpGPProblem, SamplerConfig, fitExpGP
from .monoexp import fitMonoExp, printBr
from .prep import estimateExpPrior, estimateNoise, read_courbe, selX

# FitOCT.R:37-53
DEFAULT_CTRL = {
    "depthSel": None, "dataType": 2, "subSample": 1, "smooth_df": 15, "method": "sample",
    "nb_warmup": 500, "nb_sample": 1000, "modRange": 0.5, "ru_theta": 0.05,
    "lambda_rate": 0.1, "gridType": "internal", "Nn": 10, "rho_scale": 0.1, "priPost": True,
    "priorType": "abc",
}


def load_ctrl(path=None, **overrides):
    """ctrlPars of FitOCT.R:37-53, overridden by a YAML control file (FitOCT.R:56-63)
    and then by keyword arguments."""
    ctrl = dict(DEFAULT_CTRL)
    if path is not None and os.path.exists(path):
        import yaml
        with open(path) as f:
            ctrl.update(yaml.safe_load(f) or {})
    ctrl.update(overrides)
    return ctrl


@dataclass
class FileResult:
    tag: str
    x: np.ndarray
    y: np.ndarray
    noise: dict
    mono: dict
    br_mono: dict
    prior: dict = None
    fitGP: dict = None
    fitGP_pri: dict = None
    extra: dict = field(default_factory=dict)


def prepare(tag, x, y, ctrl, device=0):
    """selX -> estimateNoise -> fitMonoExp -> printBr -> estimateExpPrior (FitOCT.R:84-107)."""
    C = selX(x, y, ctrl["depthSel"], ctrl["subSample"])
    x, y = C["x"], C["y"]
    noise = estimateNoise(x, y, df=ctrl["smooth_df"])
    fitm = fitMonoExp(x, y, noise["uy"], dataType=ctrl["dataType"], device=device)
    br = printBr(fitm["fit"], silent=True)
    r = FileResult(tag, x, y, noise, fitm, br)
    if br["alert"] is not None:    # FitOCT.R:100: a GP fit only when the mono-exp fit fails
        r.prior = estimateExpPrior(x, noise["uy"], ctrl["dataType"], ctrl["priorType"],
                                   out=fitm, ru_theta=ctrl["ru_theta"], eps=1e-3)
    return r


def _gp_problem(r, ctrl, prior_PD, prior_type, **kw):
    Nn = int(ctrl["Nn"])
    rho = ctrl["rho_scale"]
    rho = 1.0 / Nn if not rho else float(rho)          # FitOCT.R:119
    return ExpGPProblem(r.x, r.y, r.noise["uy"], dataType=ctrl["dataType"], Nn=Nn,
                        gridType=ctrl["gridType"], rho=rho, theta0=r.prior["theta0"],
                        Sigma0=r.prior["Sigma0"], prior_type=prior_type,
                        lambda_rate=ctrl["lambda_rate"], prior_PD=prior_PD, **kw)


def run_batch(datasets, ctrl=None, *, nb_chains=4, seed=1234, prior_type="normal",
              device=0, force_gp=False, **model_kw):
    """Run FitOCT.R's pipeline over ``datasets`` = iterable of (tag, Courbe.csv path)
    or (tag, x, y).  Every file needing ExpGP (all if ``force_gp``) is sampled in
    one batched launch; with ``ctrl['priPost']`` a second launch draws the prior
    predictive fits (priPost.R:2-16).  Returns a list of :class:`FileResult`."""
    from .stanfit import StanFit
    ctrl = load_ctrl(**(ctrl or {}))
    results = []
    for item in datasets:
        if len(item) == 2:
            tag, path = item
            x, y = read_courbe(path)
        else:
            tag, x, y = item
        results.append(prepare(tag, x, y, ctrl, device))
    todo = [r for r in results if r.prior is not None or force_gp]
    for r in todo:
        if r.prior is None:
            r.prior = estimateExpPrior(r.x, r.noise["uy"], ctrl["dataType"], ctrl["priorType"],
                                       out=r.mono, ru_theta=ctrl["ru_theta"], eps=1e-3)
    if not todo:
        return results
    if ctrl["method"] != "sample":   # optim / vb: per-file device optimiser runs
        for r in todo:
            p = _gp_problem(r, ctrl, 0, prior_type, **model_kw)
            r.fitGP = fitExpGP(r.x, r.y, r.noise["uy"], dataType=ctrl["dataType"], Nn=p.Nn,
                               gridType=p.gridType, method=ctrl["method"], theta0=p.theta0,
                               Sigma0=p.Sigma0, lambda_rate=p.lambda_rate, rho_scale=p.rho,
                               nb_warmup=ctrl["nb_warmup"],
                               nb_iter=ctrl["nb_warmup"] + ctrl["nb_sample"],
                               prior_type=prior_type, seed=seed, device=device, **model_kw)
        return results
    cfg = SamplerConfig(chains=nb_chains, warmup=int(ctrl["nb_warmup"]),
                        samples=int(ctrl["nb_sample"]), seed=seed, device=device)
    passes = [(0, "fitGP")] + ([(1, "fitGP_pri")] if ctrl["priPost"] else [])
    for prior_PD, slot in passes:
        probs = [_gp_problem(r, ctrl, prior_PD, prior_type, **model_kw) for r in todo]
        with Batch(probs, cfg) as b:
            b.run()
            for i, (r, p) in enumerate(zip(todo, probs)):
                out = b.download(i)
                _, xGP = p.basis()
                setattr(r, slot, {"fit": StanFit.from_output(out, p), "method": "sample",
                                  "xGP": xGP, "prior_PD": prior_PD,
                                  "lasso": prior_type == "lasso"})
    return results
