"""Diagnosis aid: a migrating launch with two-ended tails against the same launch without
(FITOCT_NO_TAIL_BIDI=1): per family and tail threshold, the two-ended transition count,
the chains whose draws differ and the first differing iteration / column."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fitoct_amd import Plan, SamplerConfig  # noqa: E402
from test_gpu_sampler import _prob  # noqa: E402


def run(prob, cfg, **env):
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        with Plan(prob, cfg) as pl:
            pl.run()
            return pl.download()
    finally:
        for k, v in old.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


def compare(tag, a, b):
    diff = ~np.all((a.draws == b.draws) | (np.isnan(a.draws) & np.isnan(b.draws)), axis=2)
    bad = np.where(diff.any(1))[0]
    first = [int(np.argmax(diff[c])) for c in bad[:10]]
    print(f"{tag}: chains differing {len(bad)}, first ids {bad[:10].tolist()} at iterations {first}",
          flush=True)
    for c in bad[:2]:
        it = int(np.argmax(diff[c]))
        cols = np.where(a.draws[c, it] != b.draws[c, it])[0]
        print("   chain", c, "it", it, "cols", cols[:8].tolist(), "a", a.draws[c, it, :9].round(5).tolist(),
              "b", b.draws[c, it, :9].round(5).tolist(), flush=True)


if len(sys.argv) > 1 and sys.argv[1] == "mig":
    for fam, N in [("lasso", 1024), ("lasso", 512), ("normal", 1024), ("horseshoe", 1024)]:
        prob = _prob(fam, N, 15)
        cfg = SamplerConfig(chains=1024, warmup=100, samples=100, seed=23, max_treedepth=8)
        a = run(prob, cfg, FITOCT_NO_TAIL_BIDI="1", FITOCT_NO_MIGRATE=None, FITOCT_NO_SPEC=None)
        c = run(prob, cfg, FITOCT_NO_TAIL_BIDI=None, FITOCT_NO_MIGRATE="1", FITOCT_NO_SPEC=None)
        d = run(prob, cfg, FITOCT_NO_TAIL_BIDI="1", FITOCT_NO_MIGRATE=None, FITOCT_NO_SPEC="1")
        compare(f"{fam} N={N} mig-spec vs nomig", a, c)
        compare(f"{fam} N={N} mig-nospec vs nomig", d, c)
    sys.exit(0)
for fam, N, left in [("lasso", 1024, "1024"), ("lasso", 1024, None), ("horseshoe", 512, "1024"),
                     ("normal", 512, "1024"), ("lasso", 1024, "400")]:
    prob = _prob(fam, N, 15)
    cfg = SamplerConfig(chains=1024, warmup=100, samples=100, seed=23, max_treedepth=8)
    a = run(prob, cfg, FITOCT_NO_TAIL_BIDI=None, FITOCT_TAIL_LEFT=left)
    b = run(prob, cfg, FITOCT_NO_TAIL_BIDI="1", FITOCT_TAIL_LEFT=None)
    diff = ~np.all((a.draws == b.draws) | (np.isnan(a.draws) & np.isnan(b.draws)), axis=2)
    bad = np.where(diff.any(1))[0]
    first = [int(np.argmax(diff[c])) for c in bad[:10]]
    print(f"{fam} N={N} left={left}: two-ended {a.two_ended_transitions}, migrations {a.migrations}, "
          f"chains differing {len(bad)}, first ids {bad[:10].tolist()} at iterations {first}", flush=True)
    for c in bad[:3]:
        it = int(np.argmax(diff[c]))
        cols = np.where(a.draws[c, it] != b.draws[c, it])[0]
        print("   chain", c, "it", it, "cols", cols[:8].tolist(), "a", a.draws[c, it, :7].round(4).tolist(),
              "b", b.draws[c, it, :7].round(4).tolist(), flush=True)
