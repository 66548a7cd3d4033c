"""Which chains carry the split R-hat of a hard-geometry run (adapt_delta 0.99,
max_treedepth 12, headline problem): per-chain adapted step size, tree depth and the
share of transitions at max_treedepth, divergences, and the standardised offset of each
chain's half-chain means of the worst columns from the pooled mean (the B term of R-hat).

    python scripts/hard_diag.py SEED [--top 12]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("seed", type=int)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--adapt-delta", type=float, default=0.99)
    ap.add_argument("--max-treedepth", type=int, default=12)
    a = ap.parse_args()
    from fitoct_amd import Plan
    from fitoct_amd.stanfit import split_rhat_ess
    prob = bench.make_problem("horseshoe", 2048)
    cols = prob.column_names()
    W, S = 500, 1000
    cfg = bench.make_config(a.seed, 1024, 0, 0, W, S, a.adapt_delta, a.max_treedepth)
    with Plan(prob, cfg) as pl:
        pl.run()
        out = pl.download()
    post = out.draws[:, W:, :]
    warm = out.draws[:, :W, :]
    res = {"seed": a.seed, "chains": 1024}
    eps = out.stepsize
    td = post[:, :, 3]
    res["stepsize_quantiles"] = np.quantile(eps, [0, 0.01, 0.5, 0.99, 1]).round(6).tolist()
    res["treedepth_mean_quantiles"] = np.quantile(td.mean(1), [0, 0.01, 0.5, 0.99, 1]).round(3).tolist()
    res["frac_at_max_treedepth"] = float((td >= a.max_treedepth).mean())
    for name in ("theta.1", "theta.3", "theta.2"):
        j = cols.index(name)
        x = post[:, :, j]
        rh, ess = split_rhat_ess(x)
        h = S // 2
        hm = np.concatenate([x[:, :h].mean(1), x[:, S - h:].mean(1)])
        hv = np.concatenate([x[:, :h].var(1, ddof=1), x[:, S - h:].var(1, ddof=1)])
        mu, sd = x.mean(), np.sqrt(hv.mean())
        z = (hm - mu) / (sd / np.sqrt(h))          # half-chain means in within-sd / sqrt(n) units
        zc = np.maximum(np.abs(z[:1024]), np.abs(z[1024:]))
        top = np.argsort(-zc)[:a.top]
        # R-hat without the top chains
        keep = np.setdiff1d(np.arange(1024), top)
        rh_wo = split_rhat_ess(x[keep])[0]
        res[name] = {
            "split_rhat": round(rh, 5), "ess": round(ess, 1), "rhat_without_top": round(rh_wo, 5),
            "top_chains": [{"chain": int(c), "z_first_half": round(float(z[c]), 2),
                            "z_second_half": round(float(z[1024 + c]), 2),
                            "stepsize": round(float(eps[c]), 6),
                            "treedepth": round(float(td[c].mean()), 2),
                            "at_max_depth": round(float((td[c] >= a.max_treedepth).mean()), 3),
                            "div": round(float(post[c, :, 5].mean()), 3),
                            "inv_metric": round(float(out.inv_metric[c, j]), 8),
                            "warmup_mean": round(float(warm[c, -100:, j].mean()), 3),
                            "mean_1": round(float(x[c, :h].mean()), 3),
                            "mean_2": round(float(x[c, h:].mean()), 3)} for c in top],
            "pooled_mean": round(float(mu), 4), "within_sd": round(float(sd), 4),
            "inv_metric_quantiles": np.quantile(out.inv_metric[:, j], [0, 0.01, 0.5, 0.99, 1]).tolist(),
        }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
