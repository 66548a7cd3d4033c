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
Transformed parameters of the horseshoe model (``yGP``, ``tau``, ``lambda``;
Tests/horseShoePrior.stan:25-33) are derived from the draws on the host.
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


def add_transformed(draws: np.ndarray, cols: list, prob):
    """Append the transformed parameters of the horseshoe model (yGP, tau,
    lambda; Tests/horseShoePrior.stan:25-33) before ``br`` and drop ``br`` for a
    prior run (plotExpGP.R:42-43).  ``draws[..., len(cols)]`` in column order."""
    cols = list(cols)
    if prob.prior_type == "horseshoe":
        Nn = prob.Nn
        idx = {c: i for i, c in enumerate(cols)}
        z = draws[..., [idx[f"z.{k+1}"] for k in range(Nn)]]
        r1g, r2g = draws[..., idx["r1_global"]], draws[..., idx["r2_global"]]
        r1l = draws[..., [idx[f"r1_local.{k+1}"] for k in range(Nn)]]
        r2l = draws[..., [idx[f"r2_local.{k+1}"] for k in range(Nn)]]
        tau = r1g * np.sqrt(r2g)
        lam = r1l * np.sqrt(r2l)
        ygp = z * lam * tau[..., None]
        br_i = idx["br"]
        extra = np.concatenate([ygp, tau[..., None], lam], axis=-1)
        draws = np.concatenate([draws[..., :br_i], extra, draws[..., br_i:]], axis=-1)
        cols = (cols[:br_i] + [f"yGP.{k+1}" for k in range(Nn)] + ["tau"]
                + [f"lambda.{k+1}" for k in range(Nn)] + cols[br_i:])
    if prob.prior_PD:   # plotExpGP.R:42-43: br is not a quantity of the prior run
        j = cols.index("br")
        draws = np.delete(draws, j, axis=-1)
        cols = cols[:j] + cols[j + 1:]
    return draws, cols


class StanFit:
    """Draws of one sampler run: ``draws[chain, iteration, column]``."""

    def __init__(self, draws: np.ndarray, columns: list, warmup: int, model_name="ExpGP",
                 stepsize=None, inv_metric=None, meta=None):
        self.columns = list(columns)
        self.warmup = int(warmup)              # leading warmup iterations stored
        self.model_name = model_name
        self.stepsize = stepsize
        self.inv_metric = inv_metric
        self.meta = dict(meta or {})
        self._draws = np.asarray(draws, dtype=np.float64)

    # ------------------------------------------------------------------ build
    @classmethod
    def from_output(cls, out, prob) -> "StanFit":
        """From a :class:`fitoct_amd.api.SampleOutput` (adds transformed parameters)."""
        draws, cols = add_transformed(out.draws, list(out.columns), prob)
        return cls(draws, cols, out.warmup_saved, stepsize=out.stepsize,
                   inv_metric=out.inv_metric,
                   meta={"kernel_ms": out.kernel_ms, "total_leapfrogs": out.total_leapfrogs,
                         "prior_type": prob.prior_type, "prior_PD": prob.prior_PD})

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
        """One Stan-CSV file per chain (warmup draws included, as save_warmup=1),
        readable by ``rstan::read_stan_csv`` / CmdStan tooling."""
        os.makedirs(directory, exist_ok=True)
        paths = []
        for c in range(self.chains):
            p = os.path.join(directory, f"{prefix}_{c + 1}.csv")
            with open(p, "w") as f:
                f.write(f"# model = {self.model_name}\n# method = sample (Default)\n")
                f.write(f"#   num_warmup = {self.warmup}\n#   num_samples = {self.iterations}\n")
                f.write(f"#   save_warmup = {1 if self.warmup else 0}\n")
                f.write(",".join(self.columns) + "\n")
                if self.stepsize is not None:
                    f.write("# Adaptation terminated\n")
                    f.write(f"# Step size = {self.stepsize[c]:.8g}\n")
                if self.inv_metric is not None:
                    f.write("# Diagonal elements of inverse mass matrix:\n# "
                            + ", ".join(f"{v:.8g}" for v in self.inv_metric[c]) + "\n")
                np.savetxt(f, self._draws[c], delimiter=",", fmt="%.10g")
            paths.append(p)
        return paths

    def __repr__(self):
        return (f"StanFit({self.model_name}: {self.chains} chains x {self.iterations} draws, "
                f"{len(self.columns)} columns)")
