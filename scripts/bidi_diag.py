"""Two-ended trajectories vs the one-ended deep path on a few chains: the first iteration
whose draws differ, with its sampler columns (diagnosis aid for scripts/archive/gpu_r4_bidi.sh)."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fitoct_amd import Plan, SamplerConfig  # noqa: E402
from test_gpu_sampler import _prob  # noqa: E402

COLS = ["lp", "acc", "eps", "depth", "nlf", "div", "energy", "q0", "q1"]


def run(env):
    for k in ("FITOCT_NO_BIDI", "FITOCT_BIDI_RB"):
        os.environ.pop(k, None)
    os.environ.update(env)
    prob = _prob("normal", 512, 15)
    cfg = SamplerConfig(chains=int(os.environ.get("DIAG_CHAINS", "2")), warmup=int(os.environ.get("DIAG_WARMUP", "30")),
                        samples=int(os.environ.get("DIAG_SAMPLES", "10")),
                        seed=int(os.environ.get("DIAG_SEED", "35")), max_treedepth=int(os.environ.get("DIAG_DEPTH", "10")))
    with Plan(prob, cfg) as pl:
        pl.run()
        return pl.download()


def compare(a, b):
    for c in range(a.draws.shape[0]):
        d = np.where((a.draws[c] != b.draws[c]).any(axis=1))[0]
        if d.size == 0:
            print("chain", c, "equal")
            continue
        i = d[0]
        print("chain", c, "first differing iteration", i, "of", a.draws.shape[1])
        for j in range(max(0, i - 1), min(i + 2, a.draws.shape[1])):
            print(" bidi ", j, dict(zip(COLS, np.round(a.draws[c, j, :9], 6))))
            print(" plain", j, dict(zip(COLS, np.round(b.draws[c, j, :9], 6))))


base = run({"FITOCT_NO_BIDI": "1"})
for env in ({}, {"FITOCT_BIDI_RB": "1"}):
    out = run(env)
    print("=== bidi", env, "leapfrogs", out.total_leapfrogs, "vs", base.total_leapfrogs)
    compare(out, base)
