"""Result object mirroring the parts of rstan's ``stanfit`` the reference reads.

The reference's consumers use (plotExpGP.R:7-50, server.R:88-237, priPost.R:20-23):

* ``print(fit, pars)``                        -> :meth:`StanFit.print`
* ``rstan::extract(fit, 'br')[[1]]``           -> :meth:`StanFit.extract`
* ``as.matrix(fit, pars=pars)``                -> :meth:`StanFit.as_matrix`
* ``rstan::summary(fit, pars, use_cache, probs)$summary`` with ``Rhat`` and
  ``n_eff`` columns                            -> :meth:`StanFit.summary`
* ``traceplot(fit, inc_warmup=TRUE)``          -> :meth:`StanFit.extract` (``inc_warmup=True``)
* Stan CSV (``rstan::read_stan_csv`` builds a real stanfit from it in R)
                                               -> :meth:`StanFit.write_stan_csv`

Parameter naming follows Stan's flattening (``theta.1``, ``yGP.3`` ...); a
parameter *base* name (``theta``) selects all of its elements, as in rstan.
The column layout (transformed parameters of the horseshoe model, ``yGP``, ``tau``,
``lambda``, Tests/horseShoePrior.stan:25-33; the lasso's ``lambda``; ``br`` dropped
for a prior run) and the Stan-CSV writer are the library's (include/fitoct.h,
"Stan output"), shared with the R shim.
R-hat / n_eff come from libfitoct's C++ diagnostics (fitoct_split_rhat_ess).
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

from . import _lib

SAMPLER_COLS = ["lp__", "accept_stat__", "stepsize__", "treedepth__", "n_leapfrog__",
                "divergent__", "energy__"]


def _base(name: str) -> str:
    return re.sub(r"\.\d+$", "", name)


def split_rhat_ess(x: np.ndarray):
    """x[chains, n] -> (split R-hat, n_eff) via the library (rstan::summary convention)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    r, e = C.c_double(), C.c_double()
    _lib.check(_lib.lib().fitoct_split_rhat_ess(_lib.dptr(x), x.shape[0], x.shape[1],
                                                C.byref(r), C.byref(e)))
    return r.value, e.value


def rank_rhat(x: np.ndarray) -> float:
    x = np.ascontiguousarray(x, dtype=np.float64)
    r = C.c_double()
    _lib.check(_lib.lib().fitoct_rank_rhat(_lib.dptr(x), x.shape[0], x.shape[1], C.byref(r)))
    return r.value


def trapped_chains(divergent: np.ndarray) -> np.ndarray:
    """The fixed definition of a funnel-trapped chain used by bench.py's lines and the
    tests: more than half of its post-warmup transitions diverge over the
    run or over either half of it (a chain can fall into the horseshoe funnel's neck
    mid-run and stay there).  divergent[chains, draws] (the divergent__ column) -> bool
    [chains].  ``trapped_whole_run`` is the rule of rounds 1-3 (whole run only)."""
    d = np.asarray(divergent, dtype=np.float64)
    h = d.shape[1] // 2
    return (d.mean(1) > 0.5) | (d[:, :h].mean(1) > 0.5) | (d[:, h:].mean(1) > 0.5)


def trapped_whole_run(divergent: np.ndarray) -> np.ndarray:
    return np.asarray(divergent, dtype=np.float64).mean(1) > 0.5


def output_columns(prob, lead=SAMPLER_COLS) -> list:
    """Column names of the output layout (include/fitoct.h, "Stan output"): the
    leading columns, the model's parameters, the transformed parameters of the
    horseshoe (``tau``, ``lambda``, ``yGP``; Tests/horseShoePrior.stan:25-33) and the
    lasso's ``lambda``, and ``br`` unless ``prior_PD`` (plotExpGP.R:42-43)."""
    L = _lib.lib()
    p = prob.to_c()
    n = L.fitoct_output_n_params(C.byref(p))
    if n < 0:
        _lib.check(-1)
    buf = C.create_string_buffer(64)
    names = []
    for i in range(n):
        _lib.check(L.fitoct_output_param_name(C.byref(p), i, buf, 64))
        names.append(buf.value.decode())
    return list(lead) + names


def materialise(raw: np.ndarray, prob, n_lead: int = len(SAMPLER_COLS)) -> np.ndarray:
    """Raw rows ``[..., n_lead + D + 1]`` (leading columns, constrained parameters,
    ``br``) -> the output layout, by the library (``fitoct_output_rows``): the same
    code that writes the Stan CSV files the R shim hands to rstan::read_stan_csv."""
    raw = np.ascontiguousarray(raw, dtype=np.float64)
    lead_shape = raw.shape[:-1]
    rows = int(np.prod(lead_shape)) if lead_shape else 1
    width = len(output_columns(prob, lead=())) + n_lead
    out = np.empty(lead_shape + (width,))
    p = prob.to_c()
    _lib.check(_lib.lib().fitoct_output_rows(C.byref(p), int(n_lead), rows, _lib.dptr(raw),
                                             _lib.dptr(out)))
    return out


class StanFit:
    """Draws of one sampler run: ``draws[chain, iteration, column]``."""

    def __init__(self, draws: np.ndarray, columns: list, warmup: int, model_name="ExpGP",
                 stepsize=None, inv_metric=None, meta=None, source=None):
        self.columns = list(columns)
        self.warmup = int(warmup)              # leading warmup iterations stored
        self.model_name = model_name
        self.stepsize = stepsize
        self.inv_metric = inv_metric
        self.meta = dict(meta or {})
        self._draws = np.asarray(draws, dtype=np.float64)
        # what the library's Stan-CSV writer needs: ("sample", prob, cfg, raw draws,
        # kernel_ms) or ("vb", prob, vb config, mu, mean_sumr2, q, log_p, log_g, sumr2, eta)
        self._source = source

    # ------------------------------------------------------------------ build
    @classmethod
    def from_output(cls, out, prob, cfg=None) -> "StanFit":
        """From a :class:`fitoct_amd.api.SampleOutput`: the output layout (transformed
        parameters added, ``br`` dropped for a prior run) by the library."""
        cfg = cfg if cfg is not None else getattr(out, "cfg", None)
        return cls(materialise(out.draws, prob), output_columns(prob), out.warmup_saved,
                   stepsize=out.stepsize, inv_metric=out.inv_metric,
                   meta={"kernel_ms": out.kernel_ms, "total_leapfrogs": out.total_leapfrogs,
                         "prior_type": prob.prior_type, "prior_PD": prob.prior_PD},
                   source=("sample", prob, cfg, out.draws, out.kernel_ms))

    # --------------------------------------------------------------- access
    @property
    def chains(self) -> int:
        return self._draws.shape[0]

    @property
    def iterations(self) -> int:
        return self._draws.shape[1] - self.warmup

    def _select(self, pars):
        if pars is None:
            return list(range(len(self.columns)))
        if isinstance(pars, str):
            pars = [pars]
        sel = []
        for p in pars:
            hit = [i for i, c in enumerate(self.columns) if c == p or _base(c) == p]
            if not hit:
                raise KeyError(f"no parameter {p!r} in the fit")
            sel += hit
        return sel

    def extract(self, pars=None, inc_warmup=False, permuted=False):
        """dict name -> array[chains, iterations] (``rstan::extract``-like)."""
        sl = slice(None) if inc_warmup else slice(self.warmup, None)
        out = {}
        for i in self._select(pars):
            a = self._draws[:, sl, i]
            out[self.columns[i]] = a.reshape(-1) if permuted else a
        return out

    def as_matrix(self, pars=None):
        """``as.matrix(fit, pars)``: rows = post-warmup draws (chains stacked)."""
        sel = self._select(pars)
        return self._draws[:, self.warmup:, :][..., sel].reshape(-1, len(sel))

    def summary(self, pars=None, probs=(0.025, 0.25, 0.5, 0.75, 0.975)):
        """rstan::summary(fit)$summary: mean, se_mean, sd, quantiles, n_eff, Rhat."""
        rows = {}
        for i in self._select(pars):
            x = self._draws[:, self.warmup:, i]
            flat = x.reshape(-1)
            if np.all(np.isnan(flat)):
                continue
            rh, ne = split_rhat_ess(x)
            sd = float(np.std(flat, ddof=1))
            row = {"mean": float(np.mean(flat)),
                   "se_mean": sd / np.sqrt(ne) if ne and ne > 0 else float("nan"),
                   "sd": sd}
            for p in probs:
                row[f"{100 * p:g}%"] = float(np.quantile(flat, p))
            row["n_eff"] = ne
            row["Rhat"] = rh
            rows[self.columns[i]] = row
        return rows

    def print(self, pars=None, digits=3):
        s = self.summary(pars)
        if not s:
            return ""
        keys = list(next(iter(s.values())).keys())
        w = max(len(k) for k in s) + 2
        lines = [f"Inference for Stan-compatible model: {self.model_name}.",
                 f"{self.chains} chains, warmup={self.warmup}, post-warmup draws per chain="
                 f"{self.iterations}.", "", " " * w + "".join(f"{k:>11}" for k in keys)]
        for name, row in s.items():
            lines.append(f"{name:<{w}}" + "".join(f"{v:>11.{digits}g}" for v in row.values()))
        txt = "\n".join(lines)
        print(txt)
        return txt

    # ------------------------------------------------------------- export
    def write_stan_csv(self, directory: str, prefix: str = "chain"):
        """CmdStan CSV files, one per chain (``fitoct_write_stan_csv`` /
        ``fitoct_write_vb_csv``: the same writer the R shim uses), readable by
        ``rstan::read_stan_csv``.  Sampled fits keep their warmup rows (save_warmup)
        and the adaptation block; an ADVI fit gives one variational CSV."""
        if self._source is None or (self._source[0] == "sample" and self._source[2] is None):
            raise ValueError("this fit was not produced by the sampler or ADVI with a known "
                             "configuration: nothing to write")
        os.makedirs(directory, exist_ok=True)
        L = _lib.lib()
        kind, prob = self._source[0], self._source[1]
        p = prob.to_c()
        if kind == "vb":
            _, _, vcfg, mu, mean_s2, q, lp, lg, s2, eta = self._source
            path = os.path.join(directory, f"{prefix}_vb.csv")
            _lib.check(L.fitoct_write_vb_csv(path.encode(), C.byref(p), C.byref(vcfg),
                                             _lib.dptr(mu), float(mean_s2), q.shape[0],
                                             _lib.dptr(q), _lib.dptr(lp), _lib.dptr(lg),
                                             _lib.dptr(s2), float(eta)))
            return [path]
        _, _, cfg, raw, kernel_ms = self._source
        c = cfg.to_c()
        raw = np.ascontiguousarray(raw, dtype=np.float64)
        wrows = self.warmup
        paths = []
        for ch in range(raw.shape[0]):
            path = os.path.join(directory, f"{prefix}_{ch + 1}.csv")
            lf = raw[ch, :, 4]           # elapsed time split by the chain's n_leapfrog__
            t = kernel_ms / 1e3
            tw = t * lf[:wrows].sum() / lf.sum() if lf.sum() > 0 else 0.0
            minv = (np.ascontiguousarray(self.inv_metric[ch]) if self.inv_metric is not None
                    else None)
            _lib.check(L.fitoct_write_stan_csv(
                path.encode(), C.byref(p), C.byref(c), ch, _lib.dptr(raw[ch]),
                float(self.stepsize[ch]) if self.stepsize is not None else float("nan"),
                _lib.dptr(minv), float(tw), float(t - tw)))
            paths.append(path)
        return paths

    def __repr__(self):
        return (f"StanFit({self.model_name}: {self.chains} chains x {self.iterations} draws, "
                f"{len(self.columns)} columns)")
