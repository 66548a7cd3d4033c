"""Per-chain behaviour fixtures of the C oracle at BASELINE shapes (tests/golden/).

Why: at rstan's default controls (adapt_delta 0.8, the control FitOCTLib's
``rstan::sampling`` call uses; ShinyInterface/server.R:97-100 colours R-hat per
parameter) the headline horseshoe posterior (Tests/horseShoePrior.stan:37-42,
N = 2048, Nn = 15) traps ~1-2 % of chains in the funnel between the global and
local scales, and config 4's lasso (Tests/lassoPrior.stan:10-12, N = 4096) mixes
slowly on yGP.6-8.  These fixtures record what the *algorithm* does on those
posteriors -- the C oracle (oracle/fitoct_oracle.c, the sequential restatement of
Stan's NUTS) on the exact bench problems (bench.py:make_problem, data seed 1234,
step seed 1000) -- so that ``tests/test_gpu_funnel.py`` can check the HIP sampler's
per-chain behaviour against it on the same global chain ids.

Stored per chain (``chain_stats``): divergence rate, trapped flag (> 50 %
divergent), adapted step size, mean tree depth / n_leapfrog / accept_stat, and for
every parameter column the two half-chain means and variances (split R-hat of any
chain subset follows from them) plus the single-chain Geyer ESS (bulk, of the
post-warmup draws).  No draws are stored.

The ``batch`` case (config 5, FitOCT.R's batch mode) is per FILE instead: the 256
synthetic files of bench.py's config-5 line (the four synthData.R modulations cycled, data
seeds 1234 + f, N = 481, normal prior), 4 chains each with global ids 4f .. 4f + 3, at
ctrlParams.yaml:1-2's 100 warmup + 100 draws and bench step 0's seed 2000.  Stored per
file: the max split R-hat over the parameter columns (the config-5 line's statistic; the
Shiny app paints R-hat >= 1.1 red, ShinyInterface/server.R:98-100), the chains' mean
adapted step size, tree depth and divergence rate (``batch_files.npz``).

Run:  python tests/golden/make_trapped.py [headline|lasso|batch|all] [--threads T]
(deterministic; ~40 min for the headline case on 8 cores, ~15 min for lasso, ~1 min batch).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

# name: (prior, N, chain ids [0, chains), warmup, samples, seed, adapt_delta, max_treedepth)
CASES = {
    "headline": ("horseshoe", 2048, 512, 500, 1000, 1000, 0.8, 10),
    "lasso": ("lasso", 4096, 256, 500, 1000, 1000, 0.8, 10),
}
BLOCK = 64
SAMPLER = ["lp__", "accept_stat__", "stepsize__", "treedepth__", "n_leapfrog__",
           "divergent__", "energy__"]


def make_problem(prior, N):
    """bench.py:make_problem, restated here so the fixture does not import bench.py."""
    from fitoct_amd import ExpGPProblem
    from fitoct_amd.synth import default_prior, synth_decay
    t0, S0 = default_prior()
    d = synth_decay(N, "sincExp", 1234)
    return ExpGPProblem(d["x"], d["y"], d["uy"], dataType=2, Nn=15, gridType="extremal",
                        theta0=t0, Sigma0=S0, prior_type=prior, nu=1.0, lambda_scale=10.0)


def param_columns(cols):
    """The columns bench.py's convergence() judges: parameters, without the
    horseshoe's inverse-gamma auxiliaries r2_*."""
    return [j for j, n in enumerate(cols) if j >= 7 and not n.startswith("r2_")]


def _geyer_ess_1(x):
    """Single-chain ESS (Geyer initial positive + monotone sequence), x[n]."""
    from oracle.diag_np import ess
    return ess(x[None, :])


def chain_stats(draws, W, cols):
    """draws[chains, W + S, n_cols] (save_warmup layout) -> dict of per-chain arrays."""
    post = np.asarray(draws[:, W:, :], dtype=np.float64)
    C, S, _ = post.shape
    par = param_columns(cols)
    h = S // 2
    halves = np.stack([post[:, :h, :][:, :, par], post[:, S - h:, :][:, :, par]], axis=1)
    ess = np.array([[_geyer_ess_1(post[c, :, j]) for j in par] for c in range(C)])
    div = post[:, :, 5].mean(1)
    return {
        "div_rate": div, "trapped": div > 0.5, "stepsize": post[:, 0, 2],
        "treedepth": post[:, :, 3].mean(1), "n_leapfrog": post[:, :, 4].mean(1),
        "accept_stat": post[:, :, 1].mean(1),
        "half_mean": halves.mean(2), "half_var": halves.var(2, ddof=1),
        "ess": ess, "param_cols": np.array([cols[j] for j in par]),
    }


def split_rhat_from_halves(half_mean, half_var, n):
    """Split R-hat per column from half-chain means / variances [chains, 2, cols]
    (oracle/diag_np.psr over the 2*chains half chains of length n)."""
    m = half_mean.reshape(-1, half_mean.shape[-1])
    v = half_var.reshape(-1, half_var.shape[-1])
    B = n * m.var(0, ddof=1)
    Wv = v.mean(0)
    return np.sqrt((B / Wv + n - 1) / n)


def make(name, threads):
    from fitoct_amd import SamplerConfig
    from oracle import nuts_c
    prior, N, chains, W, S, seed, ad, mtd = CASES[name]
    prob = make_problem(prior, N)
    cols = prob.column_names()
    parts = []
    t = time.time()
    for off in range(0, chains, BLOCK):
        cfg = SamplerConfig(chains=BLOCK, chain_offset=off, warmup=W, samples=S, seed=seed,
                            adapt_delta=ad, max_treedepth=mtd)
        o = nuts_c.sample(prob, cfg, nthreads=threads)
        st = chain_stats(o["draws"], W, cols)
        st["leapfrogs"] = o["leapfrogs"]
        parts.append(st)
        print(f"[{name}] chains [{off}, {off + BLOCK}) done, {time.time() - t:.0f} s, "
              f"trapped {int(st['trapped'].sum())}", flush=True)
    out = {k: (parts[0][k] if k == "param_cols" else np.concatenate([p[k] for p in parts]))
           for k in parts[0]}
    meta = dict(case=name, prior=prior, N=N, Nn=15, chains=chains, chain_offset=0, warmup=W,
                samples=S, seed=seed, adapt_delta=ad, max_treedepth=mtd, data_seed=1234,
                modulation="sincExp", generator="oracle/fitoct_oracle.c via oracle/nuts_c.py")
    path = os.path.join(HERE, f"trapped_{name}.npz")
    np.savez_compressed(path, meta=np.array(json.dumps(meta)),
                        **{k: (v.astype(np.float32) if v.dtype == np.float64 and v.ndim > 1
                               else v) for k, v in out.items()})
    print(f"[{name}] wrote {path}: trapped {int(out['trapped'].sum())}/{chains}, "
          f"median div {np.median(out['div_rate']):.4f}", flush=True)


# config 5 (bench.py CONFIGS[5], bench_batch): files, N, chains per file, W, S, seed
BATCH = dict(files=256, N=481, chains=4, warmup=100, samples=100, seed=2000, adapt_delta=0.8,
             max_treedepth=10)


def batch_problem(f):
    """bench.py:bench_batch's file_problems(f, 1), restated (no bench.py import)."""
    from fitoct_amd import ExpGPProblem
    from fitoct_amd.synth import MODULATIONS, default_prior, synth_decay
    t0, S0 = default_prior()
    d = synth_decay(BATCH["N"], MODULATIONS[f % 4], 1234 + f)
    return ExpGPProblem(d["x"], d["y"], d["uy"], dataType=2, Nn=15, gridType="extremal",
                        theta0=t0, Sigma0=S0, prior_type="normal")


def file_stats(draws, W, cols):
    """One file's draws[chains, W + S, n_cols] -> (max split R-hat over the parameter
    columns, mean step size, mean tree depth, divergence rate), with oracle/diag_np."""
    from oracle.diag_np import split_rhat
    post = np.asarray(draws[:, W:, :], dtype=np.float64)
    rh = max(split_rhat(post[:, :, j]) for j in param_columns(cols))
    return (float(rh), float(post[:, 0, 2].mean()), float(post[:, :, 3].mean()),
            float(post[:, :, 5].mean()))


def make_batch(threads):
    from fitoct_amd import SamplerConfig
    from oracle import nuts_c
    B = BATCH
    C = B["chains"]
    rows = []
    t = time.time()
    for f in range(B["files"]):
        prob = batch_problem(f)
        cfg = SamplerConfig(chains=C, chain_offset=f * C, warmup=B["warmup"],
                            samples=B["samples"], seed=B["seed"], adapt_delta=B["adapt_delta"],
                            max_treedepth=B["max_treedepth"])
        o = nuts_c.sample(prob, cfg, nthreads=min(threads, C))
        rows.append(file_stats(o["draws"], B["warmup"], prob.column_names()))
        if f % 32 == 31:
            print(f"[batch] files [0, {f + 1}) done, {time.time() - t:.0f} s", flush=True)
    a = np.array(rows)
    meta = dict(case="batch", prior="normal", modulations="synthData.R sincExp..sincExp3 cycled",
                data_seed="1234 + file", chain_ids="4 file + c", Nn=15,
                generator="oracle/fitoct_oracle.c via oracle/nuts_c.py", **B)
    path = os.path.join(HERE, "batch_files.npz")
    np.savez_compressed(path, meta=np.array(json.dumps(meta)), rhat_max=a[:, 0],
                        stepsize=a[:, 1], treedepth=a[:, 2], div_rate=a[:, 3])
    print(f"[batch] wrote {path}: median max R-hat {np.median(a[:, 0]):.4f}, "
          f"files >= 1.1: {int((a[:, 0] >= 1.1).sum())}/{len(a)}", flush=True)


def load(path):
    with np.load(path, allow_pickle=False) as z:
        out = {k: z[k] for k in z.files}
    out["meta"] = json.loads(str(out["meta"]))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("case", nargs="?", default="all", choices=["all", "batch", *CASES])
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    for n in (CASES if a.case == "all" else [] if a.case == "batch" else [a.case]):
        make(n, a.threads)
    if a.case in ("all", "batch"):
        make_batch(a.threads)
