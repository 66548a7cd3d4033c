"""Hard-geometry profile (Tests/testGamma.R:45: adapt_delta 0.99, max_treedepth 12) of the
headline problem at several step seeds: split / rank R-hat, trapped chains, divergences
and the worst columns per seed (one JSON line each).  The north-star R-hat < 1.01 claim
must hold on seeds nobody tuned on.

    python scripts/hard_seeds.py 1000 1019 1001 ...   [--adapt-delta 0.99 --max-treedepth 12]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("seeds", type=int, nargs="+")
    ap.add_argument("--adapt-delta", type=float, default=0.99)
    ap.add_argument("--max-treedepth", type=int, default=12)
    ap.add_argument("--chains", type=int, default=1024)
    ap.add_argument("--iters", default="500,1000")
    ap.add_argument("--prior", default="horseshoe")
    ap.add_argument("--N", type=int, default=2048)
    a = ap.parse_args()
    W, S = (int(v) for v in a.iters.split(","))
    from fitoct_amd import Plan
    prob = bench.make_problem(a.prior, a.N)
    cols = prob.column_names()
    for seed in a.seeds:
        cfg = bench.make_config(seed, a.chains, 0, 0, W, S, a.adapt_delta, a.max_treedepth)
        with Plan(prob, cfg) as pl:
            t0 = time.perf_counter()
            pl.run()
            wall = time.perf_counter() - t0
            out = pl.download()
        conv = bench.convergence(out.draws, out.warmup_saved, cols)
        print(json.dumps({"seed": seed, "prior": a.prior, "N": a.N, "adapt_delta": a.adapt_delta,
                          "max_treedepth": a.max_treedepth, "wall_s": round(wall, 2),
                          "gradients_per_iteration": round(out.total_leapfrogs / (a.chains * (W + S)), 1),
                          **conv}), flush=True)


if __name__ == "__main__":
    main()
